/*
 * koord_oracle.h -- TEST INFRASTRUCTURE.  CPU restatement of koord-scheduler's
 * Filter/Score hot path (NodeResourcesFit, LoadAwareScheduling) used ONLY as the
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
} orc_state;

int orc_state_init(orc_state *st, const koordhip_node_soa *soa, int32_t n);
void orc_state_free(orc_state *st);

/* Per-plugin reference-form evaluators for one (pod, node). */
int orc_fit_filter(const koordhip_config *cfg, const orc_state *st, const koordhip_pod *pod, int32_t node);
int64_t orc_fit_score(const koordhip_config *cfg, const orc_state *st, const koordhip_pod *pod, int32_t node);
int orc_la_filter(const koordhip_config *cfg, const orc_state *st, const koordhip_pod *pod, int32_t node);
int64_t orc_la_score(const koordhip_config *cfg, const orc_state *st, const koordhip_pod *pod, int32_t node);

/* Same contract as koordhip_eval (status / scores / topk all optional). */
int orc_eval(const koordhip_config *cfg, const orc_state *st, const koordhip_pod *pods, int32_t n_pods,
             uint8_t *status, int32_t *scores, koordhip_topk *topk, int32_t k);

/* Reserve / Unreserve delta. */
void orc_commit(const koordhip_config *cfg, orc_state *st, const koordhip_pod *pod, int32_t node, int sign);

/* Greedy stream with the reference loop structure: per pod a parallel Filter
 * over all nodes, a parallel Score per plugin over the feasible nodes
 * (parallelize.Until: `threads` workers, chunk = max(1, min(sqrt(n), n/16+1))),
 * serial lowest-index argmax, serial Reserve.  threads <= 1 runs serially. */
int orc_place_stream(const koordhip_config *cfg, orc_state *st, const koordhip_pod *pods, int32_t n_pods,
                     int32_t *out_node, int32_t threads);

#ifdef __cplusplus
}
#endif

#endif
