/*
 * koord_oracle.h -- TEST INFRASTRUCTURE.  CPU restatement of koord-scheduler's
 * Filter/Score hot path (NodeResourcesFit, LoadAwareScheduling, NodeNUMAResource, Reservation) used ONLY as the
 * checker by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
 * Nothing in the product (koordinator_amd/, libkoordhip.so) links or calls it.
 *
 * Parity pinning: the per-plugin arithmetic is pinned by the known-answer
 * tables of the reference's own tests (tests/golden/ JSON files, each case carrying
 * its reference file:line).  NodeResourcesFit and the selectHost loop live in
 * un-vendored upstream k8s v1.24.15: those rules are marked UPSTREAM-ASSUMED in
 * koord_oracle.c and are parity-unpinned by reference fixtures.
 *
 * It consumes exactly the boundary's data format (include/koordhip.h).
 */
#ifndef KOORD_ORACLE_H
#define KOORD_ORACLE_H

#include <stdint.h>

#include "../include/koordhip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* derived per-node bits (same meaning as the device's node flags) */
#define ORC_LA_OK_NONPROD 1u
#define ORC_LA_OK_PROD 2u
#define ORC_LA_SCORE_ZERO 4u

/* int64(math.Round(float64(used)/float64(total)*100)), load_aware.go:214,248 */
int64_t orc_usage_percent(int64_t used_milli, int64_t total_milli);
/* leastRequestedScore, load_aware.go:388-397 / (upstream) least_allocated.go */
int64_t orc_least_requested(int64_t requested, int64_t capacity);

/* LoadAware Filter masks, one byte per node (ORC_LA_* bits). */
void orc_la_flags(const koordhip_node_soa *soa, int32_t n, uint8_t *out);

/* Mutable node state owned by the oracle (a copy of the snapshot's mutable columns). */
typedef struct orc_state {
  int32_t n;
  const koordhip_node_soa *soa; /* static columns */
  uint8_t *flags;               /* ORC_LA_* */
  int64_t *requested[KOORDHIP_NRES];
  int64_t *nz_cpu_m, *nz_mem;
  int32_t *npods;
  int64_t *la_used_cpu_m, *la_used_mem;
  int64_t *la_used_prod_cpu_m, *la_used_prod_mem;
  /* NodeNUMAResource NodeAllocation (maxRefCount 1) */
  uint64_t *numa_free[KOORDHIP_NUMA_WORDS];
  uint64_t *numa_excl_pcpu[KOORDHIP_NUMA_WORDS];
  uint64_t *numa_excl_numa[KOORDHIP_NUMA_WORDS];
  int32_t *numa_alloc_cnt;
  int64_t *numa_zone_used; /* [n][2][KOORDHIP_NUMA_MAX_NODES] NUMA zone allocations */
  uint64_t *cpuset_out; /* optional [n_pods][WORDS] output of orc_place_stream */
  /* Reservation: Allocated (cpu milli, memory) and len(AssignedPods) of each node's reservation */
  int64_t *resv_allocated[2];
  int32_t *resv_assigned;
  /* NodeNUMAResource RestoreReservation: the reserved CPUs each reservation
   * slot has left ([WORDS][slots x n]; NULL when the snapshot has none) */
  uint64_t *resv_cpus[KOORDHIP_NUMA_WORDS];
  /* set by orc_place_stream around the Reserve of a pod with exactly one
   * feasible node: upstream then skips PreScore / Score, so no reservation is
   * nominated before the NodeNUMAResource Reserve */
  int32_t no_prescore;
  /* DeviceShare deviceUsed [n][TYPES][dev_slots][RES] and NodeResourcesFit's
   * extended scalar Requested [NXRES][n] (dev_oracle.c) */
  int64_t *dev_used;
  int64_t *xrequested;
  uint32_t *dev_out; /* optional [n_pods][TYPES] device slots of the last orc_place_stream_ext call */
  /* PodTopologySpread: each table constraint's matching pods per node [cons][n] (pts_oracle.c) */
  int32_t *pts_cnt;
  /* InterPodAffinity: each count entry's pods per node [ents][n] (ipa_oracle.c) */
  int32_t *ipa_cnt;
  /* DeviceShare: the resv_dev column of the snapshot's device-holding
   * reservations, its allocated half advanced by Reserve (NULL: none) */
  int64_t *resv_dev;
  /* ABI 14: the extended scalars' Allocated of each node's device-holding
   * reservation [NXRES][n] (the resv_xallocated column, advanced by Reserve;
   * NULL: no snapshot column) */
  int64_t *resv_xallocated;
  /* the koordhip_pod_ext record of the pod being scheduled (NULL: none): the
   * nomination's DeviceShare FilterReservation reads it */
  const koordhip_pod_ext *cur_ext;
  /* the Reservation plugin's BeforePreFilter runs (orc_resv_on): the
   * DeviceShare reservation restore exists */
  int32_t resv_restore;
} orc_state;

/* PodTopologySpread per-pod state (pts_oracle.c): PreFilter's pairs and
 * minima per topology key, PreScore's ignored nodes, pairs and weights */
typedef struct orc_pts {
  int on, scored, nh, ns;
  int hj[KOORDHIP_PTS_POD], sj[KOORDHIP_PTS_POD];
  uint8_t *fpres[KOORDHIP_PTS_KEYS];
  int64_t *fmatch[KOORDHIP_PTS_KEYS];
  int64_t fmin[KOORDHIP_PTS_KEYS];
  uint8_t *ignored;
  uint8_t *spres[KOORDHIP_PTS_KEYS];
  int64_t *scount[KOORDHIP_PTS_KEYS];
  double weight[KOORDHIP_PTS_POD];
} orc_pts;
int orc_pts_active(const koordhip_config *cfg, const orc_state *st, const koordhip_pod_ext *x);
int orc_pts_prefilter(const koordhip_config *cfg, const orc_state *st, const koordhip_pod_ext *x, orc_pts *ps);
int orc_pts_filter(const orc_state *st, const koordhip_pod_ext *x, const orc_pts *ps, int32_t i);
int orc_pts_prescore(const orc_state *st, const koordhip_pod_ext *x, orc_pts *ps, const int32_t *feas, int32_t nf);
int64_t orc_pts_score(const orc_state *st, const koordhip_pod_ext *x, const orc_pts *ps, int32_t i);
void orc_pts_normalize(const orc_pts *ps, const int32_t *feas, int64_t *scores, int32_t nf);
void orc_pts_commit(orc_state *st, const koordhip_pod_ext *x, int32_t i);
void orc_pts_free(orc_pts *ps);

/* InterPodAffinity per-pod state (ipa_oracle.c): PreFilter's pair maps per
 * topology key (affinityCounts; antiAffinityCounts + existingAntiAffinityCounts)
 * and PreScore's topologyScore */
typedef struct orc_ipa {
  int on, filt, scored, aff_empty;
  int64_t *aff[KOORDHIP_PTS_KEYS];
  int64_t *anti[KOORDHIP_PTS_KEYS];
  int64_t *score[KOORDHIP_PTS_KEYS];
} orc_ipa;
int orc_ipa_active(const koordhip_config *cfg, const orc_state *st, const koordhip_pod_ext *x);
int orc_ipa_prefilter(const koordhip_config *cfg, const orc_state *st, const koordhip_pod_ext *x, orc_ipa *ia);
int orc_ipa_filter(const orc_state *st, const koordhip_pod_ext *x, const orc_ipa *ia, int32_t i);
int orc_ipa_prescore(const orc_state *st, const koordhip_pod_ext *x, orc_ipa *ia);
int64_t orc_ipa_score(const orc_state *st, const orc_ipa *ia, int32_t i);
void orc_ipa_normalize(int64_t *scores, int32_t nf);
void orc_ipa_commit(orc_state *st, const koordhip_pod_ext *x, int32_t i);
void orc_ipa_free(orc_ipa *ia);

int orc_state_init(orc_state *st, const koordhip_node_soa *soa, int32_t n);
void orc_state_free(orc_state *st);

/* Per-plugin reference-form evaluators for one (pod, node). */
int orc_fit_filter(const koordhip_config *cfg, const orc_state *st, const koordhip_pod *pod, int32_t node);
int64_t orc_fit_score(const koordhip_config *cfg, const orc_state *st, const koordhip_pod *pod, int32_t node);
int orc_la_filter(const koordhip_config *cfg, const orc_state *st, const koordhip_pod *pod, int32_t node);
int64_t orc_la_score(const koordhip_config *cfg, const orc_state *st, const koordhip_pod *pod, int32_t node);
/* upstream static node filters (host-resolved static_allow lookup) and
 * NodeResourcesBalancedAllocation (k8s v1.24.15, parity unpinned) */
int orc_static_filter(const orc_state *st, const koordhip_pod *pod, int32_t node);
int64_t orc_bal_score(const koordhip_config *cfg, const orc_state *st, const koordhip_pod *pod, int32_t node);
/* the KOORDHIP_PLUGIN_* bit of plugin_weight[p] / score plane p */
uint32_t orc_score_plugin_bit(int p);

/* NodeNUMAResource (numa_oracle.c). */
int orc_numa_filter(const koordhip_config *cfg, const orc_state *st, const koordhip_pod *pod, int32_t node);
int64_t orc_amplify(int64_t origin, double ratio);
int64_t orc_numa_score(const koordhip_config *cfg, const orc_state *st, const koordhip_pod *pod, int32_t node);
int orc_numa_allocate(const orc_state *st, const koordhip_pod *pod, int32_t node, uint64_t *cpus_out);
int orc_numa_reserve_active(const orc_state *st, const koordhip_pod *pod, int32_t i);
/* pref: the reservation-preferred CPUs (orc_resv_pref), NULL = none */
int orc_numa_reserve(orc_state *st, const koordhip_pod *pod, int32_t node, uint64_t *cpus_out, const uint64_t *pref);
void orc_numa_release(orc_state *st, int32_t node, const uint64_t *cpus);
/* takeCPUs on one topology (cpu_accumulator.go:87-232), maxRefCount 1; 1 = ok. */
int orc_take_cpus(const koordhip_numa_class *t, const uint64_t *avail, const uint64_t *excl_pcpu,
                  const uint64_t *excl_numa, int need, int bind_policy, int excl_policy, int most_allocated,
                  uint64_t *out);
int orc_spread_order(const koordhip_numa_class *t, const uint64_t *avail, int most_allocated, int32_t *cpu_ids);

/* Topology manager Merge (frameworkext/topologymanager/policy*.go) over the
 * provider hints as filterProvidersHints (policy.go:93-117) sees them: one
 * entry per provider without hints (ORC_TM_PROVIDER_EMPTY) or per resource of
 * a provider (a nil slice: ORC_TM_RES_NIL, an empty one: ORC_TM_RES_EMPTY,
 * else ORC_TM_RES_HINTS with n hints).  numa_nodes = the default affinity
 * mask.  Returns admit (canAdmitPodResult); *out = the best hint. */
#define ORC_TM_PROVIDER_EMPTY 0
#define ORC_TM_RES_NIL 1
#define ORC_TM_RES_EMPTY 2
#define ORC_TM_RES_HINTS 3
#define ORC_TM_MAX_HINTS 255
typedef struct orc_tm_hint {
  uint64_t mask;
  int32_t preferred;
  int32_t nil; /* NUMANodeAffinity == nil */
} orc_tm_hint;
typedef struct orc_tm_entry {
  int32_t kind;
  int32_t n;
  orc_tm_hint h[ORC_TM_MAX_HINTS];
} orc_tm_entry;
int orc_tm_merge(int policy, uint64_t numa_nodes, const orc_tm_entry *e, int32_t ne, orc_tm_hint *out);
/* The NUMA-zone part of Allocate for node i under its topology policy: the
 * merged hint (nil -> *nil = 1), admit, and allocateResourcesByHint's amounts
 * [2][KOORDHIP_NUMA_MAX_NODES]; returns 1 when Admit + Allocate succeed. */
int orc_numa_allocate_hint(const orc_state *st, const koordhip_pod *pod, int32_t node, uint64_t mask, int64_t *zones,
                           uint64_t *cpus);
int orc_numa_hint_alloc(const orc_state *st, const koordhip_pod *pod, int32_t node, uint64_t *mask, int32_t *nil,
                        int32_t *admit, int64_t *zones);

/* Reservation (resv_oracle.c): the cycle's restore (sign +1 apply, -1 undo),
 * classification, filterWithReservations on the restored state, nomination,
 * scoreReservation, the normalized scores over a feasible list, Reserve, and
 * the device's ranking total. */
int orc_resv_on(const koordhip_config *cfg, const orc_state *st);
int orc_resv_slots(const orc_state *st); /* reservation slots per node (resv_* columns hold slots x n) */
int orc_resv_nominate(const orc_state *st, const koordhip_pod *pod, int32_t i); /* nominated slot, -1 none */
/* Oracle-internal pod flag bit (never from the ABI): DeviceShare is in the
 * profile and the pod requests devices (PreparePod: not skip), so DeviceShare's
 * FilterReservation takes part in the nomination (deviceshare/plugin.go:325-356). */
#define ORC_POD_DEVSHARE (1u << 29)
/* `pod` with ORC_POD_DEVSHARE set when it applies (x: its ext record or NULL) */
koordhip_pod orc_devshare_pod(const koordhip_config *cfg, const koordhip_pod *pod, const koordhip_pod_ext *x);
int orc_resv_node_present(const orc_state *st, int32_t i);
int orc_resv_node_matchable(const orc_state *st, const koordhip_pod *pod, int32_t i);
void orc_resv_classify(const orc_state *st, const koordhip_pod *pod, int32_t i, int *matched, int *unmatched);
void orc_resv_restore_delta(const orc_state *st, const koordhip_pod *pod, int32_t i, int64_t *dreq, int64_t *dnz,
                            int32_t *dpods);
void orc_resv_restore(orc_state *st, const koordhip_pod *pod, int sign);
int orc_resv_filter(const orc_state *st, const koordhip_pod *pod, int32_t i);
int orc_resv_nominated(const orc_state *st, const koordhip_pod *pod, int32_t i);
int64_t orc_resv_score(const orc_state *st, const koordhip_pod *pod, int32_t i);
void orc_resv_assume(orc_state *st, const koordhip_pod *pod, int32_t i, const uint64_t *cpus);
/* getReservationReservedCPUs (nodenumaresource/plugin.go:503-524): the reserved
 * CPUs left in the reservation PreScore nominated on node i, for a cpuset pod;
 * zero when none */
/* the Reservation Filter of a KOORDHIP_POD_RESERVE pod (x: its ext record or NULL) */
int orc_resv_reserve_pod_ok(const orc_state *st, const koordhip_pod *pod, const koordhip_pod_ext *x, int32_t i);
void orc_resv_pref(const koordhip_config *cfg, const orc_state *st, const koordhip_pod *pod, int32_t i, uint64_t *P);
void orc_resv_normalized(const orc_state *st, const koordhip_pod *pod, const int32_t *feasible, int32_t nf,
                         int64_t *norm);
int64_t orc_resv_rank_total(const koordhip_config *cfg, const orc_state *st, const koordhip_pod *pod, int32_t i,
                            int64_t b);

/* DeviceShare, extended scalars, upstream normalized Scores (dev_oracle.c).
 * pod (NULL: no reservation context) is the pod being scheduled. */
int orc_dev_node_present(const orc_state *st, int32_t i);
int orc_dev_filter(const orc_state *st, const koordhip_pod *pod, const koordhip_pod_ext *x, int32_t i);
int64_t orc_dev_score(const koordhip_config *cfg, const orc_state *st, const koordhip_pod *pod,
                      const koordhip_pod_ext *x, int32_t i, int nominated);
/* apply = 0: the allocation only (nothing changes); apply with `assumed`
 * (the Reservation Reserve assumed the pod into the node's device-holding
 * reservation) also advances that reservation's allocated devices */
int orc_dev_reserve(const koordhip_config *cfg, orc_state *st, const koordhip_pod *pod, const koordhip_pod_ext *x,
                    int32_t i, int nominated, uint32_t *slots, int apply);
int orc_dev_try_from_reservation(const orc_state *st, const koordhip_pod *pod, const koordhip_pod_ext *x, int32_t i,
                                 int fromResv, uint32_t *slots);
void orc_dev_apply(orc_state *st, const koordhip_pod_ext *x, int32_t i, const uint32_t *slots, int assumed);
/* the slot of node i's reservation holding devices, -1 none */
int orc_dev_resv_slot(const orc_state *st, int32_t i);
/* DeviceShare FilterReservation of that reservation (plugin.go:325-356) */
int orc_dev_filter_reservation(const orc_state *st, const koordhip_pod *pod, const koordhip_pod_ext *x, int32_t i);
int orc_resv_slot_class(const orc_state *st, const koordhip_pod *pod, int s, int32_t i);
int orc_xfit_filter(const orc_state *st, const koordhip_pod_ext *x, int32_t i);
int64_t orc_static_score(const orc_state *st, const koordhip_pod *pod, int32_t i, int which);
void orc_default_normalize(int64_t *scores, int32_t nf, int reverse);
/* 100 x the score weights of every enabled plugin but Reservation (the
 * ranking total's B, DESIGN.md Reservation key) */
int64_t orc_bmax(const koordhip_config *cfg);

/* Same contract as koordhip_eval (status / scores / topk all optional). */
int orc_eval(const koordhip_config *cfg, const orc_state *st, const koordhip_pod *pods, int32_t n_pods,
             uint8_t *status, int32_t *scores, koordhip_topk *topk, int32_t k);

/* Reserve / Unreserve delta.  Reserve returns KOORDHIP_ERESERVE (nothing
 * committed) when the NUMA Allocate fails; cpus: the cpuset given / taken back. */
int orc_commit(const koordhip_config *cfg, orc_state *st, const koordhip_pod *pod, int32_t node, int sign,
               uint64_t *cpus);
/* ... with the pod's koordhip_pod_ext (NULL: none): DeviceShare Reserve
 * (`nominated`: a reservation PreScore nominated on the node; devs: the slots
 * allocated [TYPES], optional) and the extended scalars.  Reserve only. */
int orc_commit_ext(const koordhip_config *cfg, orc_state *st, const koordhip_pod *pod, const koordhip_pod_ext *x,
                   int32_t node, uint64_t *cpus, int nominated, uint32_t *devs);
/* koordhip_eval_ext: scores [n_pods][NPLUGINS + NEXT_PLUGINS][n] (raw), topk
 * by the ranking total with the normalized plugins' weighted scores added. */
int orc_eval_ext(const koordhip_config *cfg, const orc_state *st, const koordhip_pod *pods, const koordhip_pod_ext *ext,
                 int32_t n_pods, uint16_t *status, int32_t *scores, koordhip_topk *topk, int32_t k);

/* Greedy stream with the reference loop structure: per pod a parallel Filter
 * over all nodes, a parallel Score per plugin over the feasible nodes
 * (parallelize.Until: `threads` workers, chunk = max(1, min(sqrt(n), n/16+1))),
 * serial lowest-index argmax, serial Reserve.  threads <= 1 runs serially. */
int orc_place_stream(const koordhip_config *cfg, orc_state *st, const koordhip_pod *pods, int32_t n_pods,
                     int32_t *out_node, int32_t threads);
/* ... with koordhip_pod_ext records (NULL: none): DeviceShare, the extended
 * scalars and the normalized Scores (NodeAffinity, TaintToleration,
 * DeviceShare: DefaultNormalizeScore over the feasible nodes). */
int orc_place_stream_ext(const koordhip_config *cfg, orc_state *st, const koordhip_pod *pods,
                         const koordhip_pod_ext *ext, int32_t n_pods, int32_t *out_node, int32_t threads);
void orc_set_dev_out(orc_state *st, uint32_t *devs);
/* cpusets of the last orc_place_stream call are written here when non-NULL ([n_pods][WORDS]). */
void orc_set_cpuset_out(orc_state *st, uint64_t *cpus);

#ifdef __cplusplus
}
#endif

#endif
