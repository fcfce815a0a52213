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
 * A node holds up to koordhip_node_soa.resv_slots Available reservations
 * (KOORDHIP_RESV_SLOTS, slot s of node i at [s n + i]); a reservation's state is
 * Allocated (cpu, memory; masked to ResourceNames) and len(AssignedPods).  The
 * reference iterates a node's reservations in Go map order
 * (forEachAvailableReservationOnNode, cache.go:236-252); the filter and the
 * restore do not depend on that order, the nomination's ties do
 * (findMostPreferredReservationByOrder keeps the first smallest order,
 * nominator.go:60; sort.Slice by score keeps an unspecified first,
 * nominator.go:69-71): here the lowest slot wins both.
 */
#include <string.h>

#include "koord_oracle.h"

#define NZ_DEFAULT_CPU 100                 /* (upstream) schedutil.DefaultMilliCPURequest */
#define NZ_DEFAULT_MEM (200ll * 1024 * 1024) /* (upstream) schedutil.DefaultMemoryRequest */

static int64_t max0(int64_t v) { return v > 0 ? v : 0; }

int orc_resv_on(const koordhip_config *cfg, const orc_state *st) {
  return ((cfg->filter_plugins | cfg->score_plugins) & KOORDHIP_PLUGIN_RESERVATION) && st->soa->resv_flags;
}

int orc_resv_slots(const orc_state *st) { return st->soa->resv_slots > 1 ? st->soa->resv_slots : 1; }
/* column index of slot s of node i */
static size_t at(const orc_state *st, int s, int32_t i) { return (size_t)s * (size_t)st->n + (size_t)i; }

static int has_key(uint32_t rf, int r) { return (rf & (r == 0 ? KOORDHIP_RESV_KEY_CPU : KOORDHIP_RESV_KEY_MEM)) != 0; }
static int pod_key(const koordhip_pod *p, int r) {
  return (p->flags & (r == 0 ? KOORDHIP_POD_KEY_CPU : KOORDHIP_POD_KEY_MEM)) != 0;
}
/* SubtractWithNonNegativeResult(Allocatable, Allocated) of slot x, resource r */
static int64_t rem_of(const orc_state *st, size_t x, int r) {
  return has_key(st->soa->resv_flags[x], r) ? max0(st->soa->resv_alloc[r][x] - st->resv_allocated[r][x]) : 0;
}

/* ---- ABI 14: the extended scalars of the node's reservation holding devices
 * (slot h = resv_dev_slot[i]): more keys of that reservation's Allocatable
 * (resv_xalloc; a listed key is > 0) and Allocated (st->resv_xallocated), so
 * every ResourceList rule of this file sees them as it sees cpu / memory.  The
 * pod's scalar requests are its koordhip_pod_ext record's (st->cur_ext; NULL:
 * none). */
static int xslot(const orc_state *st, int32_t i) {
  if (!st->soa->resv_xalloc || !st->soa->resv_dev_slot || !st->resv_xallocated) return -1;
  return st->soa->resv_dev_slot[i];
}
static int64_t xa(const orc_state *st, int j, int32_t i) { return st->soa->resv_xalloc[(size_t)j * st->n + i]; }
static int64_t xrem(const orc_state *st, int j, int32_t i) {
  return max0(xa(st, j, i) - st->resv_xallocated[(size_t)j * st->n + i]);
}
/* the pod requests scalar j (the key is in its request map) */
static int xkey(const orc_state *st, int j) { return st->cur_ext && ((st->cur_ext->xmask >> j) & 1u); }
static int64_t xreq(const orc_state *st, int j) { return xkey(st, j) ? st->cur_ext->xreq[j] : 0; }

/* transformer.go:86-103: 1 = matched, 2 = unmatched with assigned pods, 0 =
 * untouched, for slot x (isReservedPod is false: reserve pods are not streamed). */
static int slot_class(const orc_state *st, const koordhip_pod *pod, size_t x) {
  const uint32_t rf = st->soa->resv_flags[x];
  if (!(rf & KOORDHIP_RESV_PRESENT)) return 0;                                     /* :87-89 */
  const int32_t assigned = st->resv_assigned[x];
  if ((rf & KOORDHIP_RESV_ALLOCATE_ONCE) && assigned > 0) return 0;               /* :93-95 */
  const int match = (int)((pod->resv_match >> KOORDHIP_RESV_GROUP(rf)) & 1u);     /* matchReservation :335-359 */
  if (!(rf & KOORDHIP_RESV_UNSCHEDULABLE) && match) return 1;                     /* :97-98 */
  return assigned > 0 ? 2 : 0;                                                     /* :100-101 */
}

int orc_resv_slot_class(const orc_state *st, const koordhip_pod *pod, int s, int32_t i) {
  return st->soa->resv_flags ? slot_class(st, pod, at(st, s, i)) : 0;
}

void orc_resv_classify(const orc_state *st, const koordhip_pod *pod, int32_t i, int *matched, int *unmatched) {
  *matched = *unmatched = 0;
  if (!st->soa->resv_flags) return;
  for (int s = 0; s < orc_resv_slots(st); s++) {
    const int c = slot_class(st, pod, at(st, s, i));
    *matched += c == 1;
    *unmatched += c == 2;
  }
}

/* The NodeInfo delta the restore applies for `pod` on node i (requested cpu /
 * memory, non-zero cpu / memory, pod count), summed over its reservations:
 * restoreUnmatchedReservations (transformer.go:252-278, updateNodeInfoRequested
 * :280-293) or restoreMatchedReservation (:227-250, NodeInfo.RemovePod of the
 * reserve pod).  The sums do not depend on the reservations' order. */
void orc_resv_restore_delta(const orc_state *st, const koordhip_pod *pod, int32_t i, int64_t *dreq, int64_t *dnz,
                            int32_t *dpods) {
  const koordhip_node_soa *so = st->soa;
  dreq[0] = dreq[1] = dnz[0] = dnz[1] = 0;
  *dpods = 0;
  if (!so->resv_flags) return;
  for (int s = 0; s < orc_resv_slots(st); s++) {
    const size_t x = at(st, s, i);
    const int c = slot_class(st, pod, x);
    if (!c) continue;
    for (int r = 0; r < 2; r++) { /* the reserve pod leaves: Requested and NonZeroRequested */
      dreq[r] -= so->resv_alloc[r][x];
      dnz[r] -= so->resv_nz[r][x];
    }
    if (c == 1) {
      *dpods -= 1; /* RemovePod */
      continue;
    }
    /* unmatched: a pod requesting SubtractWithNonNegativeResult(Allocatable, Allocated) comes back unless IsZero
     * (its scalars too, on the device-holding reservation) */
    const uint32_t rf = so->resv_flags[x];
    const int64_t rem0 = rem_of(st, x, 0), rem1 = rem_of(st, x, 1);
    int xany = 0;
    if (s == xslot(st, i))
      for (int j = 0; j < KOORDHIP_NXRES; j++) xany |= xrem(st, j, i) != 0;
    if (rem0 == 0 && rem1 == 0 && !xany) continue;
    for (int r = 0; r < 2; r++) {
      const int64_t rem = r ? rem1 : rem0;
      dreq[r] += rem;
      /* GetNonzeroRequests of that pod: a key it lists counts as is, a missing one as the default */
      dnz[r] += has_key(rf, r) ? rem : (r == 0 ? NZ_DEFAULT_CPU : NZ_DEFAULT_MEM);
    }
  }
}

/* Apply (sign +1) / undo (-1) the restore of `pod` on every node holding a reservation. */
void orc_resv_restore(orc_state *st, const koordhip_pod *pod, int sign) {
  for (int32_t i = 0; i < st->n; i++) {
    int64_t dreq[2], dnz[2];
    int32_t dp;
    orc_resv_restore_delta(st, pod, i, dreq, dnz, &dp);
    st->requested[KOORDHIP_RES_CPU][i] += sign * dreq[0];
    st->requested[KOORDHIP_RES_MEM][i] += sign * dreq[1];
    st->nz_cpu_m[i] += sign * dnz[0];
    st->nz_mem[i] += sign * dnz[1];
    st->npods[i] += sign * dp;
    /* NodeResourcesFit's extended scalars (updateNodeInfoRequested's ScalarResources loop, :285-290, and
     * RemovePod): the device-holding reservation's Allocatable leaves, its remainder comes back when unmatched */
    const int h = xslot(st, i);
    const int c = h >= 0 ? slot_class(st, pod, at(st, h, i)) : 0;
    if (c)
      for (int j = 0; j < KOORDHIP_NXRES; j++)
        st->xrequested[(size_t)j * st->n + i] += sign * (-xa(st, j, i) + (c == 2 ? xrem(st, j, i) : 0));
  }
}

/* filterWithReservations (plugin.go:373-440) on the RESTORED node i, with
 * fitsNode (:445-494) per matched reservation: podRequested = Requested after
 * the unmatched restore (= before the matched one), rAllocated = the matched
 * reservations' Allocated, rRemained = the reservation's Allocatable -
 * Allocated.  Default-policy reservations are insufficient only with
 * preemptible resources (none in a stream, :405-412); an Aligned one that fits
 * or a Restricted one that fits and holds the pod's requests passes the node
 * (:414-431); otherwise it fails when it has Aligned or Restricted ones
 * (:434-438, all of them insufficient).  1 = pass. */
int orc_resv_filter(const orc_state *st, const koordhip_pod *pod, int32_t i) {
  const koordhip_node_soa *so = st->soa;
  int matched, unmatched;
  orc_resv_classify(st, pod, i, &matched, &unmatched);
  if (!matched) return (pod->flags & KOORDHIP_POD_RESV_AFFINITY) ? 0 : 1; /* :378-392 (hasAffinity; nothing preemptible) */
  const int S = orc_resv_slots(st);
  int64_t podreq[2] = {st->requested[0][i], st->requested[1][i]}, rall[2] = {0, 0};
  for (int s = 0; s < S; s++) {
    const size_t x = at(st, s, i);
    if (slot_class(st, pod, x) != 1) continue;
    for (int r = 0; r < 2; r++) {
      podreq[r] += so->resv_alloc[r][x]; /* undo the matched restore (:129) */
      rall[r] += st->resv_allocated[r][x];
    }
  }
  int n_ar = 0;
  for (int s = 0; s < S; s++) {
    const size_t x = at(st, s, i);
    if (slot_class(st, pod, x) != 1) continue;
    const uint32_t policy = KOORDHIP_RESV_POLICY(so->resv_flags[x]);
    if (policy == 0) continue;
    n_ar++;
    /* fitsNode: len(Pods) - len(matched) + 1 > allowed on the restored NodeInfo */
    int fits = !((int64_t)st->npods[i] - matched + 1 > (int64_t)so->alloc_pods[i]);
    if (fits && (pod->flags & KOORDHIP_POD_HAS_REQ)) {
      for (int r = 0; r < 2 && fits; r++)
        if (pod->req[r] > so->alloc[r][i] - (podreq[r] - rem_of(st, x, r) - rall[r])) fits = 0;
      if (fits && pod->req[KOORDHIP_RES_EPH] > so->alloc[KOORDHIP_RES_EPH][i] - st->requested[KOORDHIP_RES_EPH][i]) fits = 0;
      if (fits && (pod->flags & KOORDHIP_POD_REQ_BCPU) &&
          pod->req[KOORDHIP_RES_BCPU] > so->alloc[KOORDHIP_RES_BCPU][i] - st->requested[KOORDHIP_RES_BCPU][i])
        fits = 0;
      if (fits && (pod->flags & KOORDHIP_POD_REQ_BMEM) &&
          pod->req[KOORDHIP_RES_BMEM] > so->alloc[KOORDHIP_RES_BMEM][i] - st->requested[KOORDHIP_RES_BMEM][i])
        fits = 0;
    }
    /* fitsNode over the pod's scalars: Allocatable - (podRequested - rRemained - allRAllocated), podRequested
     * = the scalars' Requested after the unmatched restore (the matched one undone), on the device-holding
     * reservation h (rRemained: this reservation's, h's only when x is h; allRAllocated: h's when matched) */
    const int h = xslot(st, i);
    if (fits && (pod->flags & KOORDHIP_POD_HAS_REQ) && st->cur_ext)
      for (int j = 0; j < KOORDHIP_NXRES && fits; j++) {
        if (!xkey(st, j)) continue;
        const int hm = h >= 0 && slot_class(st, pod, at(st, h, i)) == 1;
        const int64_t alloc = so->xalloc ? so->xalloc[(size_t)j * st->n + i] : 0;
        const int64_t preq = st->xrequested[(size_t)j * st->n + i] + (hm ? xa(st, j, i) : 0);
        const int64_t rrem = (h >= 0 && s == h) ? xrem(st, j, i) : 0;
        const int64_t rall_x = hm ? st->resv_xallocated[(size_t)j * st->n + i] : 0;
        if (xreq(st, j) > alloc - (preq - rrem - rall_x)) fits = 0;
      }
    if (policy == 1 && fits) return 1; /* Aligned :415-419 */
    if (policy == 2) {                  /* Restricted :420-432: LessThanOrEqual(podRequests, rRemained) */
      int le = 1;
      for (int r = 0; r < 2; r++)
        if (has_key(so->resv_flags[x], r) && pod_key(pod, r) && pod->req[r] > rem_of(st, x, r)) le = 0;
      if (h >= 0 && s == h)
        for (int j = 0; j < KOORDHIP_NXRES; j++)
          if (xa(st, j, i) != 0 && xkey(st, j) && xreq(st, j) > xrem(st, j, i)) le = 0;
      if (le && fits) return 1;
    }
  }
  return n_ar == 0;
}

/* The Reservation Filter of a reserve pod (plugin.go:326-362): its
 * reservation's nodeName (x->reserve_node - 1, 0 / no record = none), then the
 * allocate-policy conflict with every Available reservation on the node
 * (:342-356: Default coexists only with Default); filterWithReservations is
 * not run for it (:365-367).  1 = pass. */
int orc_resv_reserve_pod_ok(const orc_state *st, const koordhip_pod *pod, const koordhip_pod_ext *x, int32_t i) {
  if (x && x->reserve_node > 0 && i != x->reserve_node - 1) return 0; /* ErrReasonNodeNotMatchReservation */
  if (!st->soa->resv_flags) return 1;
  const uint32_t pol = KOORDHIP_POD_RESERVE_POLICY(pod->flags);
  for (int s = 0; s < orc_resv_slots(st); s++) {
    const uint32_t rf = st->soa->resv_flags[at(st, s, i)];
    if (!(rf & KOORDHIP_RESV_PRESENT)) continue;
    const uint32_t rp = KOORDHIP_RESV_POLICY(rf);
    if ((pol == 0 || rp == 0) && pol != rp) return 0; /* ErrReasonReservationAllocatePolicyConflict */
  }
  return 1;
}

/* FilterReservation (plugin.go:504-535) of slot x, a matched reservation */
static int slot_passes(const orc_state *st, const koordhip_pod *pod, int s, int32_t i) {
  const size_t x = at(st, s, i);
  const uint32_t rf = st->soa->resv_flags[x];
  int inter = 0, nonzero = 0;
  for (int r = 0; r < 2; r++) {
    if (!(has_key(rf, r) && pod_key(pod, r))) continue; /* Intersection(ResourceNames, podRequests names) */
    inter = 1;
    if (rem_of(st, x, r) != 0) nonzero = 1;
  }
  if (s == xslot(st, i))
    for (int j = 0; j < KOORDHIP_NXRES; j++) {
      if (!(xa(st, j, i) != 0 && xkey(st, j))) continue;
      inter = 1;
      if (xrem(st, j, i) != 0) nonzero = 1;
    }
  return inter && nonzero;
}

/* scoreReservation (scoring.go:177-200) of slot x: MostAllocated over
 * RemoveZeros(Allocatable) of podRequests + Allocated. */
static int64_t slot_score(const orc_state *st, const koordhip_pod *pod, int slot, int32_t i) {
  const size_t x = at(st, slot, i);
  const uint32_t rf = st->soa->resv_flags[x];
  int64_t s = 0, w = 0;
  for (int r = 0; r < 2; r++) {
    const int64_t cap = has_key(rf, r) ? st->soa->resv_alloc[r][x] : 0;
    if (cap == 0) continue;
    w++;
    const int64_t req = (pod_key(pod, r) ? pod->req[r] : 0) + st->resv_allocated[r][x];
    if (req <= cap) s += 100 * req / cap; /* MaxNodeScore * MilliValue / MilliValue */
  }
  if (slot == xslot(st, i)) /* the scalars of RemoveZeros(Allocatable), requested = the pod's + Allocated */
    for (int j = 0; j < KOORDHIP_NXRES; j++) {
      const int64_t cap = xa(st, j, i);
      if (cap == 0) continue;
      w++;
      const int64_t req = xreq(st, j) + st->resv_xallocated[(size_t)j * st->n + i];
      if (req <= cap) s += 100 * req / cap;
    }
  return w ? s / w : 0;
}

/* NominateReservation (nominator.go:32-85) on node i: the slot of the
 * reservation nominated for `pod`, -1 for none.  Candidates: the matched
 * reservations passing RunReservationFilterPlugins (nominator.go:47-54); the
 * smallest order label among them (findMostPreferredReservationByOrder), else
 * the highest scoreReservation (prioritizeReservations); ties: the lowest slot.
 *
 * The reservation filter plugins are the Reservation plugin's FilterReservation
 * (slot_passes) and DeviceShare's (deviceshare/plugin.go:325-356): for a pod
 * requesting devices that one looks the reservation up among the node's
 * RestoreReservation state, which keeps only reservations holding devices
 * (reservation.go:134-161, `len(allocatable) == 0` -> skipped); a reservation
 * holding none fails it (allocIndex -1 -> an error status, :337-346), the
 * node's one reservation holding devices passes it when
 * tryAllocateFromReservation(requiredFromReservation) allocates
 * (orc_dev_filter_reservation).  With at most that one candidate left,
 * DeviceShare's ScoreReservation (normalized over the candidates) changes no
 * ranking. */
int orc_resv_nominate(const orc_state *st, const koordhip_pod *pod, int32_t i) {
  if (!st->soa->resv_flags) return -1;
  const int devshare = (pod->flags & ORC_POD_DEVSHARE) != 0;
  const int dslot = devshare ? orc_dev_resv_slot(st, i) : -1;
  if (devshare && (dslot < 0 || slot_class(st, pod, at(st, dslot, i)) != 1 ||
                   !orc_dev_filter_reservation(st, pod, st->cur_ext, i)))
    return -1;
  int best = -1, best_rank = 0, ord = 0;
  int64_t best_sc = -1;
  for (int s = 0; s < orc_resv_slots(st); s++) {
    const size_t x = at(st, s, i);
    if (slot_class(st, pod, x) != 1 || !slot_passes(st, pod, s, i)) continue;
    if (devshare && s != dslot) continue;
    const uint32_t rf = st->soa->resv_flags[x];
    if (rf & KOORDHIP_RESV_ORDERED) {
      const int rk = st->soa->resv_order_rank[x];
      if (!ord || rk < best_rank) {
        best = s;
        best_rank = rk;
        ord = 1;
      }
    } else if (!ord) {
      const int64_t sc = slot_score(st, pod, s, i);
      if (sc > best_sc) {
        best = s;
        best_sc = sc;
      }
    }
  }
  return best;
}

int orc_resv_nominated(const orc_state *st, const koordhip_pod *pod, int32_t i) {
  return orc_resv_nominate(st, pod, i) >= 0;
}

/* Score (scoring.go:105-121) of a node that is not the preferred one: the
 * nominated reservation's scoreReservation, 0 without one. */
int64_t orc_resv_score(const orc_state *st, const koordhip_pod *pod, int32_t i) {
  const int s = orc_resv_nominate(st, pod, i);
  return s < 0 ? 0 : slot_score(st, pod, s, i);
}

/* PreScore's node order (scoring.go:58-67): the smallest order label among the
 * node's matched reservations (before FilterReservation); -1 for none. */
static int node_order_rank(const orc_state *st, const koordhip_pod *pod, int32_t i) {
  int rk = -1;
  if (!st->soa->resv_flags) return -1;
  for (int s = 0; s < orc_resv_slots(st); s++) {
    const size_t x = at(st, s, i);
    if (slot_class(st, pod, x) != 1 || !(st->soa->resv_flags[x] & KOORDHIP_RESV_ORDERED)) continue;
    const int r = st->soa->resv_order_rank[x];
    if (rk < 0 || r < rk) rk = r;
  }
  return rk;
}

/* Reserve: assumePod into the nominated reservation (Allocated += the pod's
 * requests masked to ResourceNames, one more assigned pod).  The pod's CPUs
 * (cpus, NULL = none) join AssignedPods: the next RestoreReservation subtracts
 * them from the reservation's cpuset (nodenumaresource/reservation.go:90-97). */
void orc_resv_assume(orc_state *st, const koordhip_pod *pod, int32_t i, const uint64_t *cpus) {
  const int s = orc_resv_nominate(st, pod, i);
  if (s < 0) return;
  const size_t x = at(st, s, i);
  const uint32_t rf = st->soa->resv_flags[x];
  for (int r = 0; r < 2; r++)
    if (has_key(rf, r) && pod_key(pod, r)) st->resv_allocated[r][x] += pod->req[r];
  st->resv_assigned[x] += 1;
  if (s == xslot(st, i)) /* ... and the pod's scalars masked to its keys */
    for (int j = 0; j < KOORDHIP_NXRES; j++)
      if (xa(st, j, i) != 0 && xkey(st, j)) st->resv_xallocated[(size_t)j * st->n + i] += xreq(st, j);
  if (cpus && st->resv_cpus[0])
    for (int w = 0; w < KOORDHIP_NUMA_WORDS; w++) st->resv_cpus[w][x] &= ~cpus[w];
}

/* getReservationReservedCPUs (nodenumaresource/plugin.go:503-524): the
 * nominated reservation is PreScore's (scoring.go:42-89, so the Reservation
 * plugin must score), its reserved CPUs the RestoreReservation state
 * (reservation.go:76-113: the reservation's cpuset less its AssignedPods'),
 * restored only for pods AllowUseCPUSet admits (PreRestoreReservation :68-74)
 * and read only by cpuset pods (requestCPUBind).  Upstream skips PreScore when
 * exactly one node is feasible (schedule_one.go, v1.24.15: schedulePod returns
 * the only feasible node), so its NUMA Reserve then sees no nomination
 * (st->no_prescore). */
void orc_resv_pref(const koordhip_config *cfg, const orc_state *st, const koordhip_pod *pod, int32_t i, uint64_t *P) {
  for (int w = 0; w < KOORDHIP_NUMA_WORDS; w++) P[w] = 0;
  if (!st->resv_cpus[0] || !orc_resv_on(cfg, st) || !(cfg->score_plugins & KOORDHIP_PLUGIN_RESERVATION)) return;
  if (st->no_prescore) return;
  if (!(pod->flags & KOORDHIP_POD_CPUSET) || (pod->flags & KOORDHIP_POD_NUMA_SKIP)) return;
  const int s = orc_resv_nominate(st, pod, i);
  if (s < 0) return;
  const size_t x = at(st, s, i);
  for (int w = 0; w < KOORDHIP_NUMA_WORDS; w++) P[w] = st->resv_cpus[w][x];
}

/* The Reservation plugin's contribution for one pod over its feasible nodes
 * (PreScore + Score + DefaultNormalizeScore): norm[j] for feasible[j].
 * preferredNode: the feasible node whose matched reservations hold the smallest
 * order; the reference keeps the first such node of its (unordered) feasible
 * list, here the lowest node index (the selectHost tie rule, BASELINE.json). */
void orc_resv_normalized(const orc_state *st, const koordhip_pod *pod, const int32_t *feasible, int32_t nf,
                         int64_t *norm) {
  int32_t pref = -1, pref_rank = 0;
  for (int32_t j = 0; j < nf; j++) {
    const int32_t i = feasible[j];
    const int rk = node_order_rank(st, pod, i);
    if (rk < 0) continue;
    if (pref < 0 || rk < pref_rank || (rk == pref_rank && i < pref)) {
      pref = i;
      pref_rank = rk;
    }
  }
  int64_t mx = 0;
  for (int32_t j = 0; j < nf; j++) {
    const int32_t i = feasible[j];
    const int64_t raw = i == pref ? 1000 /* mostPreferredScore */ : orc_resv_score(st, pod, i);
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
  const int64_t bmax = orc_bmax(cfg);
  if (!(cfg->score_plugins & KOORDHIP_PLUGIN_RESERVATION)) return b;
  const int rk = node_order_rank(st, pod, i);
  if (rk >= 0) return 101 * (bmax + 1) + (KOORDHIP_RESV_MAX_ORDERS - 1 - rk);
  return orc_resv_score(st, pod, i) * (bmax + 1) + b;
}

/* node i holds an Available reservation; `pod` matches the owner group of one */
int orc_resv_node_present(const orc_state *st, int32_t i) {
  if (!st->soa->resv_flags) return 0;
  for (int s = 0; s < orc_resv_slots(st); s++)
    if (st->soa->resv_flags[at(st, s, i)] & KOORDHIP_RESV_PRESENT) return 1;
  return 0;
}
int orc_resv_node_matchable(const orc_state *st, const koordhip_pod *pod, int32_t i) {
  if (!st->soa->resv_flags) return 0;
  for (int s = 0; s < orc_resv_slots(st); s++) {
    const uint32_t rf = st->soa->resv_flags[at(st, s, i)];
    if ((rf & KOORDHIP_RESV_PRESENT) && ((pod->resv_match >> KOORDHIP_RESV_GROUP(rf)) & 1u)) return 1;
  }
  return 0;
}
