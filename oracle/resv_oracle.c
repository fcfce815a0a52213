/*
 * resv_oracle.c -- TEST INFRASTRUCTURE (see koord_oracle.h).  The Reservation
 * plugin's part of one scheduling cycle, restated from the reference:
 *
 *   BeforePreFilter restore   reservation/transformer.go:48-293
 *   filterWithReservations    reservation/plugin.go:373-494 (no preemption state:
 *                             preemptible / preemptibleInRRs are empty in a stream)
 *   FilterReservation         reservation/plugin.go:504-535
 *   NominateReservation       reservation/nominator.go:32-85
 *   PreScore / Score          reservation/scoring.go:42-200
 *   NormalizeScore            (upstream) helper.DefaultNormalizeScore, k8s v1.24.15
 *   Reserve                   reservation/plugin.go:537-575 -> cache.go:170-191 ->
 *                             ReservationInfo.AddAssignedPod reservation_info.go:297-306
 *
 * quotav1 (k8s.io/apiserver v0.24.15 pkg/quota/v1, not vendored in the
 * reference) is restated as used here: SubtractWithNonNegativeResult keeps a's
 * keys with max(0, a - b); Mask keeps the named keys; IsZero = every value 0;
 * LessThanOrEqual(a, b) compares a[k] <= b[k] for the keys of b present in a.
 *
 * One reservation per node (KOORDHIP_RESV_*); a node's reservation state is
 * Allocated (cpu, memory; masked to ResourceNames) and len(AssignedPods).
 */
#include <string.h>

#include "koord_oracle.h"

#define NZ_DEFAULT_CPU 100                 /* (upstream) schedutil.DefaultMilliCPURequest */
#define NZ_DEFAULT_MEM (200ll * 1024 * 1024) /* (upstream) schedutil.DefaultMemoryRequest */

static int64_t max0(int64_t v) { return v > 0 ? v : 0; }

int orc_resv_on(const koordhip_config *cfg, const orc_state *st) {
  return ((cfg->filter_plugins | cfg->score_plugins) & KOORDHIP_PLUGIN_RESERVATION) && st->soa->resv_flags;
}

static int has_key(uint32_t rf, int r) { return (rf & (r == 0 ? KOORDHIP_RESV_KEY_CPU : KOORDHIP_RESV_KEY_MEM)) != 0; }
static int pod_key(const koordhip_pod *p, int r) {
  return (p->flags & (r == 0 ? KOORDHIP_POD_KEY_CPU : KOORDHIP_POD_KEY_MEM)) != 0;
}

/* transformer.go:86-103: matched / unmatched classification of node i's
 * reservation for `pod` (isReservedPod is false: reserve pods are not streamed). */
void orc_resv_classify(const orc_state *st, const koordhip_pod *pod, int32_t i, int *matched, int *unmatched) {
  *matched = *unmatched = 0;
  const uint32_t rf = st->soa->resv_flags ? st->soa->resv_flags[i] : 0;
  if (!(rf & KOORDHIP_RESV_PRESENT)) return;                                       /* :87-89 */
  const int32_t assigned = st->resv_assigned[i];
  if ((rf & KOORDHIP_RESV_ALLOCATE_ONCE) && assigned > 0) return;                 /* :93-95 */
  const int match = (int)((pod->resv_match >> KOORDHIP_RESV_GROUP(rf)) & 1u);     /* matchReservation :335-359 */
  if (!(rf & KOORDHIP_RESV_UNSCHEDULABLE) && match) *matched = 1;                 /* :97-98 */
  else if (assigned > 0) *unmatched = 1;                                           /* :100-101 */
}

/* The NodeInfo delta the restore applies for `pod` on node i (requested cpu /
 * memory, non-zero cpu / memory, pod count): restoreUnmatchedReservations
 * (transformer.go:252-278, updateNodeInfoRequested :280-293) or
 * restoreMatchedReservation (:227-250, NodeInfo.RemovePod of the reserve pod). */
void orc_resv_restore_delta(const orc_state *st, const koordhip_pod *pod, int32_t i, int64_t *dreq, int64_t *dnz,
                            int32_t *dpods) {
  const koordhip_node_soa *s = st->soa;
  int matched, unmatched;
  orc_resv_classify(st, pod, i, &matched, &unmatched);
  dreq[0] = dreq[1] = dnz[0] = dnz[1] = 0;
  *dpods = 0;
  if (!matched && !unmatched) return;
  const uint32_t rf = s->resv_flags[i];
  for (int r = 0; r < 2; r++) { /* the reserve pod leaves: Requested and NonZeroRequested */
    dreq[r] -= s->resv_alloc[r][i];
    dnz[r] -= s->resv_nz[r][i];
  }
  if (matched) {
    *dpods = -1; /* RemovePod */
    return;
  }
  /* unmatched: a pod requesting SubtractWithNonNegativeResult(Allocatable, Allocated) comes back unless IsZero */
  int64_t rem[2];
  for (int r = 0; r < 2; r++) rem[r] = has_key(rf, r) ? max0(s->resv_alloc[r][i] - st->resv_allocated[r][i]) : 0;
  if (rem[0] == 0 && rem[1] == 0) return;
  for (int r = 0; r < 2; r++) {
    dreq[r] += rem[r];
    /* GetNonzeroRequests of that pod: a key it lists counts as is, a missing one as the default */
    dnz[r] += has_key(rf, r) ? rem[r] : (r == 0 ? NZ_DEFAULT_CPU : NZ_DEFAULT_MEM);
  }
}

/* Apply (sign +1) / undo (-1) the restore of `pod` on every node holding a reservation. */
void orc_resv_restore(orc_state *st, const koordhip_pod *pod, int sign) {
  for (int32_t i = 0; i < st->n; i++) {
    if (!(st->soa->resv_flags[i] & KOORDHIP_RESV_PRESENT)) continue;
    int64_t dreq[2], dnz[2];
    int32_t dp;
    orc_resv_restore_delta(st, pod, i, dreq, dnz, &dp);
    st->requested[KOORDHIP_RES_CPU][i] += sign * dreq[0];
    st->requested[KOORDHIP_RES_MEM][i] += sign * dreq[1];
    st->nz_cpu_m[i] += sign * dnz[0];
    st->nz_mem[i] += sign * dnz[1];
    st->npods[i] += sign * dp;
  }
}

/* filterWithReservations (plugin.go:373-440) on the RESTORED node i, with
 * fitsNode (:445-494): podRequested = Requested after the unmatched restore
 * (= before the matched one), rAllocated = the matched reservations'
 * Allocated, rRemained = the reservation's Allocatable - Allocated.  1 = pass. */
int orc_resv_filter(const orc_state *st, const koordhip_pod *pod, int32_t i) {
  const koordhip_node_soa *s = st->soa;
  int matched, unmatched;
  orc_resv_classify(st, pod, i, &matched, &unmatched);
  if (!matched) return (pod->flags & KOORDHIP_POD_RESV_AFFINITY) ? 0 : 1; /* :378-392 (hasAffinity; nothing preemptible) */
  const uint32_t rf = s->resv_flags[i];
  const uint32_t policy = KOORDHIP_RESV_POLICY(rf);
  if (policy == 0) return 1; /* Default: insufficient only with preemptible resources (:405-412) */
  int64_t rem[2], podreq[2];
  for (int r = 0; r < 2; r++) {
    rem[r] = has_key(rf, r) ? max0(s->resv_alloc[r][i] - st->resv_allocated[r][i]) : 0;
    podreq[r] = st->requested[r][i] + s->resv_alloc[r][i]; /* undo the matched restore (:129) */
  }
  /* fitsNode */
  int fits = 1;
  if ((int64_t)st->npods[i] + 1 - 1 > (int64_t)s->alloc_pods[i]) fits = 0; /* len(Pods) - len(matched) + 1, restored Pods */
  if (fits && (pod->flags & KOORDHIP_POD_HAS_REQ)) {
    for (int r = 0; r < 2 && fits; r++)
      if (pod->req[r] > s->alloc[r][i] - (podreq[r] - rem[r] - st->resv_allocated[r][i])) fits = 0;
    if (fits && pod->req[KOORDHIP_RES_EPH] > s->alloc[KOORDHIP_RES_EPH][i] - st->requested[KOORDHIP_RES_EPH][i]) fits = 0;
    if (fits && (pod->flags & KOORDHIP_POD_REQ_BCPU) &&
        pod->req[KOORDHIP_RES_BCPU] > s->alloc[KOORDHIP_RES_BCPU][i] - st->requested[KOORDHIP_RES_BCPU][i])
      fits = 0;
    if (fits && (pod->flags & KOORDHIP_POD_REQ_BMEM) &&
        pod->req[KOORDHIP_RES_BMEM] > s->alloc[KOORDHIP_RES_BMEM][i] - st->requested[KOORDHIP_RES_BMEM][i])
      fits = 0;
  }
  if (policy == 1) return fits; /* Aligned :415-419 */
  /* Restricted :420-432: LessThanOrEqual(podRequests, rRemained) over rRemained's keys */
  int le = 1;
  for (int r = 0; r < 2; r++)
    if (has_key(rf, r) && pod_key(pod, r) && pod->req[r] > rem[r]) le = 0;
  return le && fits;
}

/* FilterReservation (plugin.go:504-535) of node i's matched reservation: the
 * nominated one when it passes (nominator.go:48-63, one candidate). */
int orc_resv_nominated(const orc_state *st, const koordhip_pod *pod, int32_t i) {
  int matched, unmatched;
  orc_resv_classify(st, pod, i, &matched, &unmatched);
  if (!matched) return 0;
  const uint32_t rf = st->soa->resv_flags[i];
  int inter = 0, nonzero = 0;
  for (int r = 0; r < 2; r++) {
    if (!(has_key(rf, r) && pod_key(pod, r))) continue; /* Intersection(ResourceNames, podRequests names) */
    inter = 1;
    if (max0(st->soa->resv_alloc[r][i] - st->resv_allocated[r][i]) != 0) nonzero = 1;
  }
  return inter && nonzero;
}

/* scoreReservation (scoring.go:177-200): MostAllocated over
 * RemoveZeros(Allocatable) of podRequests + Allocated. */
int64_t orc_resv_score(const orc_state *st, const koordhip_pod *pod, int32_t i) {
  const uint32_t rf = st->soa->resv_flags[i];
  int64_t s = 0, w = 0;
  for (int r = 0; r < 2; r++) {
    const int64_t cap = has_key(rf, r) ? st->soa->resv_alloc[r][i] : 0;
    if (cap == 0) continue;
    w++;
    const int64_t req = (pod_key(pod, r) ? pod->req[r] : 0) + st->resv_allocated[r][i];
    if (req <= cap) s += 100 * req / cap; /* MaxNodeScore * MilliValue / MilliValue */
  }
  return w ? s / w : 0;
}

/* Reserve: assumePod into the nominated reservation (Allocated += the pod's
 * requests masked to ResourceNames, one more assigned pod). */
void orc_resv_assume(orc_state *st, const koordhip_pod *pod, int32_t i) {
  if (!orc_resv_nominated(st, pod, i)) return;
  const uint32_t rf = st->soa->resv_flags[i];
  for (int r = 0; r < 2; r++)
    if (has_key(rf, r) && pod_key(pod, r)) st->resv_allocated[r][i] += pod->req[r];
  st->resv_assigned[i] += 1;
}

/* The Reservation plugin's contribution for one pod over its feasible nodes
 * (PreScore + Score + DefaultNormalizeScore): norm[j] for feasible[j].
 * preferredNode: the feasible node whose matched reservation has the smallest
 * order; the reference keeps the first such node of its (unordered) feasible
 * list, here the lowest node index (the selectHost tie rule, BASELINE.json). */
void orc_resv_normalized(const orc_state *st, const koordhip_pod *pod, const int32_t *feasible, int32_t nf,
                         int64_t *norm) {
  const koordhip_node_soa *s = st->soa;
  int32_t pref = -1, pref_rank = 0;
  for (int32_t j = 0; j < nf; j++) {
    const int32_t i = feasible[j];
    int matched, unmatched;
    orc_resv_classify(st, pod, i, &matched, &unmatched);
    if (!matched || !(s->resv_flags[i] & KOORDHIP_RESV_ORDERED)) continue;
    const int32_t rk = s->resv_order_rank[i];
    if (pref < 0 || rk < pref_rank || (rk == pref_rank && i < pref)) {
      pref = i;
      pref_rank = rk;
    }
  }
  int64_t mx = 0;
  for (int32_t j = 0; j < nf; j++) {
    const int32_t i = feasible[j];
    int64_t raw = 0;
    if (i == pref) raw = 1000; /* mostPreferredScore */
    else if (orc_resv_nominated(st, pod, i)) raw = orc_resv_score(st, pod, i);
    norm[j] = raw;
    if (raw > mx) mx = raw;
  }
  if (mx == 0) return;
  for (int32_t j = 0; j < nf; j++) norm[j] = 100 * norm[j] / mx;
}

/* The device's ranking total (Reservation key) of a feasible
 * (pod, node) with plugin total b: koordhip_eval's topk score. */
int64_t orc_resv_rank_total(const koordhip_config *cfg, const orc_state *st, const koordhip_pod *pod, int32_t i,
                            int64_t b) {
  int64_t bmax = 0;
  for (int p = 0; p < KOORDHIP_NPLUGINS; p++)
    if (cfg->score_plugins & orc_score_plugin_bit(p)) bmax += 100 * cfg->plugin_weight[p];
  if (!(cfg->score_plugins & KOORDHIP_PLUGIN_RESERVATION)) return b;
  int matched, unmatched;
  orc_resv_classify(st, pod, i, &matched, &unmatched);
  if (matched && (st->soa->resv_flags[i] & KOORDHIP_RESV_ORDERED))
    return 101 * (bmax + 1) + (KOORDHIP_RESV_MAX_ORDERS - 1 - st->soa->resv_order_rank[i]);
  const int64_t raw = orc_resv_nominated(st, pod, i) ? orc_resv_score(st, pod, i) : 0;
  return raw * (bmax + 1) + b;
}
