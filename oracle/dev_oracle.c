/*
 * dev_oracle.c -- TEST INFRASTRUCTURE (see koord_oracle.h).  Plain-C
 * restatement of koord-scheduler's DeviceShare plugin on the default
 * allocator, of NodeResourcesFit's extended scalar resources, of the
 * (upstream) NodeAffinity / TaintToleration Scores, and of DefaultNormalizeScore,
 * one function per reference rule with its file:line.  Paths are relative to
 * pkg/scheduler/plugins/deviceshare/ unless stated otherwise.
 *
 * Device model (nodeDevice, device_cache.go:44-50): per node and device type
 * the minors of the Device CR (dev_minor, ascending), their resources
 * (deviceTotal; all zero for an unhealthy device, buildDeviceResources
 * :550-568) and what pods hold (deviceUsed, advanced by Reserve through
 * updateCacheUsed :116-127).  deviceFree = SubtractWithNonNegativeResult(total,
 * used) per minor (resetDeviceFree :185-202).  A request key a pod does not
 * carry compares and adds as 0 (quotav1.LessThanOrEqual reads only the keys of
 * the free list that the request holds; a missing value is the zero Quantity).
 *
 * Reservations holding devices are outside the engine's envelope (the host
 * rejects them): RestoreReservation (reservation.go:119-170) then keeps no
 * reservation for DeviceShare, so Filter / Score / Reserve see the node alone.
 * No reservation is nominated for a device pod either: DeviceShare's
 * FilterReservation fails every reservation that holds no devices (see
 * orc_resv_nominate), so the `nominated` branches below (Score 0,
 * scoreWithNominatedReservation :409-431; Reserve failing,
 * allocateWithNominatedReservation :379-393) are not reached from a stream.
 */
#include <stdlib.h>
#include <string.h>

#include "koord_oracle.h"

#define T KOORDHIP_DEV_TYPES
#define R KOORDHIP_DEV_RES

static size_t dix(const orc_state *st, int32_t i, int t, int s) {
  return (((size_t)i * T + (size_t)t) * (size_t)st->soa->dev_slots + (size_t)s) * R;
}
static int32_t dminor(const orc_state *st, int32_t i, int t, int s) {
  return st->soa->dev_minor[((size_t)i * T + (size_t)t) * (size_t)st->soa->dev_slots + (size_t)s];
}

static int is_zero(const int64_t v[R]) { return v[0] == 0 && v[1] == 0 && v[2] == 0; }
static int has_type(const orc_state *st, int32_t i, int t) {
  for (int s = 0; s < st->soa->dev_slots; s++)
    if (dminor(st, i, t, s) >= 0) return 1;
  return 0;
}

koordhip_pod orc_devshare_pod(const koordhip_config *cfg, const koordhip_pod *pod, const koordhip_pod_ext *x) {
  koordhip_pod p = *pod;
  if (x && (x->flags & KOORDHIP_PODX_DEVICE) && ((cfg->filter_plugins | cfg->score_plugins) & KOORDHIP_PLUGIN_DEVICESHARE))
    p.flags |= ORC_POD_DEVSHARE;
  return p;
}

int orc_dev_node_present(const orc_state *st, int32_t i) {
  return st->soa->dev_slots > 0 && st->soa->dev_present && st->soa->dev_present[i];
}

/* the pod's request of device type t (quotav1.Mask over DeviceResourceNames[t],
 * device_resources.go:42-53; PreparePod removed zero keys, plugin.go:162-182) */
static int dev_requests(const koordhip_pod_ext *x, int t, int64_t q[R]) {
  int any = 0;
  for (int r = 0; r < R; r++) {
    q[r] = x->dev_req[t][r];
    if (q[r] > 0) any = 1;
  }
  return any;
}

/* fillGPUTotalMem, utils.go:211-233: the memory of the node's GPUs (the first
 * device with resources: one GPU model per node, host-checked) completes the
 * request -- gpu-memory present: ratio = int64(float64(bytes) / float64(total) *
 * 100) (memoryBytesToRatio :207-209); else bytes = ratio * total / 100
 * (memoryRatioToBytes :203-205).  0 = no device with resources (an error). */
static int dev_fill_gpu(const orc_state *st, int32_t i, int64_t q[R]) {
  const int64_t *tot = NULL;
  for (int s = 0; s < st->soa->dev_slots && !tot; s++) {
    if (dminor(st, i, KOORDHIP_DEV_GPU, s) < 0) continue;
    const int64_t *x = st->soa->dev_total + dix(st, i, KOORDHIP_DEV_GPU, s);
    if (!is_zero(x)) tot = x;
  }
  if (!tot) return 0;
  if (q[2] >= 0) {
    q[1] = (int64_t)((double)q[2] / (double)tot[2] * 100.0);
  } else {
    const int64_t ratio = q[1] > 0 ? q[1] : 0;
    q[2] = ratio * tot[2] / 100;
  }
  if (q[0] < 0) q[0] = 0;
  return 1;
}

/* calcDeviceWanted, device_cache.go:367-395 with isPodRequestsMultipleDevice
 * (utils.go:183-201): a gpu-memory-ratio (rdma, fpga) above 100 in whole
 * hundreds asks for that many devices, each with the request divided evenly. */
static int64_t dev_wanted(int t, const int64_t q[R], int64_t per[R]) {
  for (int r = 0; r < R; r++) per[r] = q[r] > 0 ? q[r] : 0;
  const int64_t key = t == KOORDHIP_DEV_GPU ? q[1] : q[0];
  if (!(key > 100 && key % 100 == 0)) return 1;
  const int64_t w = key / 100;
  for (int r = 0; r < R; r++) per[r] = (q[r] > 0 ? q[r] : 0) / w;
  return w;
}

/* quotav1.LessThanOrEqual(podRequestPerCard, free) */
static int dev_fits(const int64_t per[R], const int64_t f[R]) {
  for (int r = 0; r < R; r++)
    if (per[r] > f[r]) return 0;
  return 1;
}

/* the scorer's resources (resourcesToWeightMap, scoring.go:212-218): weight
 * map slot k -> (device type, resource) */
static const int k_dev_res_type[5] = {KOORDHIP_DEV_GPU, KOORDHIP_DEV_GPU, KOORDHIP_DEV_GPU, KOORDHIP_DEV_RDMA,
                                      KOORDHIP_DEV_FPGA};
static const int k_dev_res_idx[5] = {0, 1, 2, 0, 0};

/* leastRequestedScore / mostRequestedScore, scoring.go:236-245 / :263-274 */
static int64_t dev_least(int64_t req, int64_t cap) {
  if (cap == 0) return 0;
  if (req > cap) return 0;
  return (cap - req) * 100 / cap;
}
static int64_t dev_most(int64_t req, int64_t cap) {
  if (cap == 0) return 0;
  if (req > cap) req = cap;
  return req * 100 / cap;
}

/* the scorer over per-resource (total, free) pairs of type t: scoreDevice
 * (scoring.go:152-177) for one device, scoreNode (:179-209) for the sums over
 * the node's devices -- requested = total - free + the pod's request when
 * total >= free (else total); leastResourceScorer / mostResourceScorer
 * (:220-261): sum(score x weight) / sum(weight) over the resources with a
 * non-zero total, 0 without any */
static int64_t dev_scorer(const koordhip_config *cfg, int t, const int64_t tot[R], const int64_t fr[R],
                          const int64_t req[R]) {
  int64_t num = 0, wsum = 0;
  for (int k = 0; k < 5; k++) {
    const int64_t w = cfg->dev_res_weight[k];
    if (w <= 0 || k_dev_res_type[k] != t) continue;
    const int r = k_dev_res_idx[k];
    if (tot[r] == 0) continue;
    const int64_t rq = tot[r] >= fr[r] ? tot[r] - fr[r] + req[r] : tot[r];
    num += (cfg->dev_most_allocated ? dev_most(rq, tot[r]) : dev_least(rq, tot[r])) * w;
    wsum += w;
  }
  return wsum ? num / wsum : 0;
}

/* ---- the node's reservation holding devices (reservation.go:119-170) ----
 * At most one per node (host-checked): slot h = resv_dev_slot[i], its
 * allocatable A (the reserve pod's devices) and allocated D (its AssignedPods'
 * on A's minors), per type and dev slot.  For the pod being scheduled the
 * restore keeps it as matched (class 1) or as unmatched with assigned pods
 * (class 2, transformer.go:86-103); per minor:
 *   remained Rm = SubtractWithNonNegativeResult(A, D) (subtractAllocated :84-92)
 *   mergedUnmatchedUsed   = A - Rm           (class 2, :86-93)
 *   mergedMatchedAllocatable = A, mergedMatchedAllocated = D   (class 1, :95-105)
 * The free devices of a preemptible map P (calcFreeWithPreemptible,
 * device_cache.go:456-481): total - SubtractWithNonNegativeResult(used, P),
 * clamped at 0 -- with P = 0 the plain free. */
typedef struct dev_rc {
  int h;   /* slot of the reservation holding devices; -1: none (or no restore) */
  int cls; /* its class for the pod: 1 matched, 2 unmatched with assigned pods, 0 neither */
  int pol; /* its AllocatePolicy: 0 Default, 1 Aligned, 2 Restricted */
  const int64_t *A, *D; /* [TYPES][dev_slots][RES] */
} dev_rc;

enum { FREE_NODE = 0, FREE_ALIGNED = 1, FREE_REQUIRED = 2 };

int orc_dev_resv_slot(const orc_state *st, int32_t i) {
  if (!st->resv_dev || !st->soa->resv_dev_slot || !st->resv_restore) return -1;
  return st->soa->resv_dev_slot[i];
}

static size_t rdix(const orc_state *st, int32_t i, int half, int t, int s) {
  return ((((size_t)i * 2 + (size_t)half) * T + (size_t)t) * (size_t)st->soa->dev_slots + (size_t)s) * R;
}

static dev_rc dev_rc_of(const orc_state *st, const koordhip_pod *pod, int32_t i) {
  dev_rc rc = {-1, 0, 0, NULL, NULL};
  const int h = pod ? orc_dev_resv_slot(st, i) : -1;
  if (h < 0) return rc;
  rc.h = h;
  rc.cls = orc_resv_slot_class(st, pod, h, i);
  rc.pol = (int)KOORDHIP_RESV_POLICY(st->soa->resv_flags[(size_t)h * st->n + i]);
  rc.A = st->resv_dev + rdix(st, i, 0, 0, 0);
  rc.D = st->resv_dev + rdix(st, i, 1, 0, 0);
  return rc;
}

static const int64_t *rc_at(const orc_state *st, const int64_t *base, int t, int s) {
  return base + ((size_t)t * (size_t)st->soa->dev_slots + (size_t)s) * R;
}
/* the reservation's remained on (t, s) */
static void rc_remained(const orc_state *st, const dev_rc *rc, int t, int s, int64_t rm[R]) {
  const int64_t *a = rc_at(st, rc->A, t, s), *d = rc_at(st, rc->D, t, s);
  for (int r = 0; r < R; r++) rm[r] = a[r] - d[r] > 0 ? a[r] - d[r] : 0;
}
/* newDeviceMinorMap(allocatable): the reservation's minors of type t (dev slot bits) */
static uint32_t rc_hints(const orc_state *st, const dev_rc *rc, int t) {
  uint32_t m = 0;
  if (rc->h < 0) return 0;
  for (int s = 0; s < st->soa->dev_slots; s++)
    if (!is_zero(rc_at(st, rc->A, t, s))) m |= 1u << s;
  return m;
}
/* calcRequiredDeviceResources (reservation.go:344-363) for type t: 1 when it
 * names type t -- Rm has a minor of type t, or Rm is empty altogether and the
 * reservation holds type t (then every one of its minors with nothing left) */
static int rc_required(const orc_state *st, const dev_rc *rc, int t) {
  int any_t = 0, any = 0;
  for (int u = 0; u < T; u++)
    for (int s = 0; s < st->soa->dev_slots; s++) {
      int64_t rm[R];
      rc_remained(st, rc, u, s, rm);
      if (!is_zero(rm)) {
        any = 1;
        if (u == t) any_t = 1;
      }
    }
  return any_t || (!any && rc_hints(st, rc, t) != 0);
}

/* the preemptible amount on (t, s) of free mode `mode` (FREE_NODE: basic +
 * mergedMatchedAllocatable; FREE_ALIGNED: basic + mergedMatchedAllocated +
 * the reservation's remained, tryAllocateFromReservation :220-253) */
static void rc_preempt(const orc_state *st, const dev_rc *rc, int mode, int t, int s, int64_t p[R]) {
  for (int r = 0; r < R; r++) p[r] = 0;
  if (rc->h < 0) return;
  const int64_t *a = rc_at(st, rc->A, t, s), *d = rc_at(st, rc->D, t, s);
  int64_t rm[R];
  rc_remained(st, rc, t, s, rm);
  for (int r = 0; r < R; r++) {
    if (rc->cls == 2) p[r] += a[r] - rm[r]; /* mergedUnmatchedUsed */
    if (rc->cls == 1) p[r] += mode == FREE_NODE ? a[r] : d[r] + rm[r];
  }
}

/* the free resources of (t, s) in mode `mode` (FREE_REQUIRED: the remained
 * when calcRequiredDeviceResources names type t, tryAllocateByDeviceType
 * :330-335; else the aligned free) */
static void rc_free(const orc_state *st, const dev_rc *rc, int mode, int32_t i, int t, int s, int64_t f[R]) {
  if (mode == FREE_REQUIRED) {
    if (rc_required(st, rc, t)) {
      rc_remained(st, rc, t, s, f);
      return;
    }
    mode = FREE_ALIGNED;
  }
  int64_t p[R];
  rc_preempt(st, rc, mode, t, s, p);
  const int64_t *tot = st->soa->dev_total + dix(st, i, t, s);
  const int64_t *used = st->dev_used + dix(st, i, t, s);
  for (int r = 0; r < R; r++) {
    const int64_t u = used[r] - p[r] > 0 ? used[r] - p[r] : 0;
    f[r] = tot[r] - u > 0 ? tot[r] - u : 0;
  }
}

typedef struct dev_pick {
  int32_t s, minor, pref;
  int64_t score;
} dev_pick;

static int pick_cmp(const void *a, const void *b) {
  const dev_pick *x = (const dev_pick *)a, *y = (const dev_pick *)b;
  if (x->pref != y->pref) return x->pref ? -1 : 1;
  if (x->score != y->score) return x->score > y->score ? -1 : 1;
  return x->minor < y->minor ? -1 : (x->minor > y->minor ? 1 : 0);
}

/* tryAllocateDevice (device_cache.go:272-314) over the pod's requested types:
 * per type the node needs devices (:286-289), the GPU memory fill (:291-295),
 * `wanted` devices (calcDeviceWanted) among the free ones of `mode` ordered by
 * sortDeviceResourcesByMinor (device_resources.go:177-195: preferred minors --
 * the reservation's, `pref` -- first, then scoreDevices' score desc, minor
 * asc; no `scorer`: score 0), skipping minors outside the reservation's when
 * `req` (required, :337-339; a type the reservation holds none of is not
 * restricted) and zero ones (:341-343).  1 = allocated (slots[t], per_t[t]). */
static int dev_allocate(const koordhip_config *cfg, const orc_state *st, const koordhip_pod_ext *x, int32_t i,
                        const dev_rc *rc, int req, int pref, int mode, int scorer, uint32_t *slots,
                        int64_t per_t[T][R]) {
  for (int t = 0; t < T; t++) slots[t] = 0;
  for (int t = 0; t < T; t++) {
    int64_t q[R], per[R], f[R];
    if (!dev_requests(x, t, q)) continue;
    if (!has_type(st, i, t)) return 0;
    if (t == KOORDHIP_DEV_GPU && !dev_fill_gpu(st, i, q)) return 0;
    const int64_t w = dev_wanted(t, q, per);
    const uint32_t hm = rc_hints(st, rc, t);
    dev_pick pk[KOORDHIP_DEV_SLOTS];
    int np = 0;
    for (int s = 0; s < st->soa->dev_slots; s++) {
      const int32_t m = dminor(st, i, t, s);
      if (m < 0) continue;
      rc_free(st, rc, mode, i, t, s, f);
      pk[np].s = s;
      pk[np].minor = m;
      pk[np].pref = pref && ((hm >> s) & 1u);
      pk[np].score = scorer ? dev_scorer(cfg, t, st->soa->dev_total + dix(st, i, t, s), f, per) : 0;
      np++;
    }
    qsort(pk, (size_t)np, sizeof(dev_pick), pick_cmp);
    int64_t got = 0;
    for (int j = 0; j < np && got < w; j++) {
      if (req && hm && !((hm >> pk[j].s) & 1u)) continue;
      rc_free(st, rc, mode, i, t, pk[j].s, f);
      if (is_zero(f) || !dev_fits(per, f)) continue;
      slots[t] |= 1u << pk[j].s;
      got++;
    }
    if (got < w) return 0;
    if (per_t) memcpy(per_t[t], per, sizeof(per));
  }
  return 1;
}

/* tryAllocateFromReservation (reservation.go:181-283) over the node's matched
 * reservation holding devices: 1 allocated (slots), 0 none (the caller falls
 * back to the node), -1 Unschedulable (an Aligned / Restricted reservation
 * that cannot hold the pod, :278-281).  fromResv: requiredFromReservation
 * (FilterReservation): a Default reservation then also restricts to its minors. */
static int dev_from_reservation(const koordhip_config *cfg, const orc_state *st, const koordhip_pod_ext *x,
                                int32_t i, const dev_rc *rc, int fromResv, int scorer, uint32_t *slots,
                                int64_t per_t[T][R]) {
  if (rc->h < 0 || rc->cls != 1) return 0;
  if (rc->pol == 0) /* Default: preemptible = basic + mergedMatchedAllocatable, preferred its minors */
    return dev_allocate(cfg, st, x, i, rc, fromResv, 1, FREE_NODE, scorer, slots, per_t) ? 1 : 0;
  if (rc->pol == 1) /* Aligned: required = preferred = its minors */
    return dev_allocate(cfg, st, x, i, rc, 1, 1, FREE_ALIGNED, scorer, slots, per_t) ? 1 : -1;
  /* Restricted: the node fits (no scorer), then the reservation's remained holds it */
  if (!dev_allocate(cfg, st, x, i, rc, 1, 1, FREE_ALIGNED, 0, slots, per_t)) return -1;
  return dev_allocate(cfg, st, x, i, rc, 1, 1, FREE_REQUIRED, scorer, slots, per_t) ? 1 : -1;
}

/* tryAllocateFromReservation of the node's reservation holding devices for
 * `pod` (no scorer): 1 / 0 / -1 as dev_from_reservation (KAT entry point). */
int orc_dev_try_from_reservation(const orc_state *st, const koordhip_pod *pod, const koordhip_pod_ext *x, int32_t i,
                                 int fromResv, uint32_t *slots) {
  const dev_rc rc = dev_rc_of(st, pod, i);
  return dev_from_reservation(NULL, st, x, i, &rc, fromResv, 0, slots, NULL);
}

/* DeviceShare Filter, plugin.go:284-323: tryAllocateFromReservation over the
 * matched reservation holding devices, else the node with the matched
 * reservations' allocatable preemptible (no scorer).  1 = passes. */
int orc_dev_filter(const orc_state *st, const koordhip_pod *pod, const koordhip_pod_ext *x, int32_t i) {
  if (!x || !(x->flags & KOORDHIP_PODX_DEVICE)) return 1; /* state.skip */
  if (!orc_dev_node_present(st, i)) return 1;           /* nodeDeviceInfo == nil: :298-301 */
  const dev_rc rc = dev_rc_of(st, pod, i);
  uint32_t slots[T];
  const int r = dev_from_reservation(NULL, st, x, i, &rc, 0, 0, slots, NULL);
  if (r != 0) return r > 0;
  return dev_allocate(NULL, st, x, i, &rc, 0, 0, FREE_NODE, 0, slots, NULL);
}

/* DeviceShare FilterReservation (plugin.go:325-356) of the node's reservation
 * holding devices, for a matched one: tryAllocateFromReservation with
 * requiredFromReservation.  1 = passes. */
int orc_dev_filter_reservation(const orc_state *st, const koordhip_pod *pod, const koordhip_pod_ext *x, int32_t i) {
  if (!x || !(x->flags & KOORDHIP_PODX_DEVICE)) return 1;
  const dev_rc rc = dev_rc_of(st, pod, i);
  if (rc.h < 0 || rc.cls != 1) return 0; /* not in the restore's matched: allocIndex -1 */
  if (!orc_dev_node_present(st, i)) return 1; /* :349-352 */
  uint32_t slots[T];
  return dev_from_reservation(NULL, st, x, i, &rc, 1, 0, slots, NULL) > 0;
}

/* scoreNode of type t over the free devices of `mode` (scoring.go:179-209;
 * nodeDevice.scoreByDeviceType device_cache.go:425-452): sums of the node's
 * totals and of the frees, the (GPU-filled) pod request */
static int64_t dev_score_mode(const koordhip_config *cfg, const orc_state *st, const koordhip_pod_ext *x, int32_t i,
                              const dev_rc *rc, int mode) {
  int64_t sum = 0;
  for (int t = 0; t < T; t++) {
    int64_t q[R];
    if (!dev_requests(x, t, q)) continue;
    if (!has_type(st, i, t)) continue; /* scoreByDeviceType: no devices -> 0 */
    if (t == KOORDHIP_DEV_GPU && !dev_fill_gpu(st, i, q)) continue;
    int64_t tot[R] = {0, 0, 0}, fr[R] = {0, 0, 0}, f[R];
    for (int s = 0; s < st->soa->dev_slots; s++) {
      if (dminor(st, i, t, s) < 0) continue;
      const int64_t *tt = st->soa->dev_total + dix(st, i, t, s);
      rc_free(st, rc, mode, i, t, s, f);
      for (int r = 0; r < R; r++) {
        tot[r] += tt[r];
        fr[r] += f[r];
      }
    }
    for (int r = 0; r < R; r++)
      if (q[r] < 0) q[r] = 0;
    sum += dev_scorer(cfg, t, tot, fr, q);
  }
  return sum;
}

/* DeviceShare Score, scoring.go:33-72 -> nodeDevice.score (device_cache.go:
 * 397-452): per requested type, scoreNode; the types add up.  `nominated`: the
 * Reservation plugin's PreScore nominated a reservation on the node: the
 * device-holding one is scored by its policy (scoreWithReservation,
 * reservation.go:286-342), any other gives 0 (:409-431, allocIndex -1). */
int64_t orc_dev_score(const koordhip_config *cfg, const orc_state *st, const koordhip_pod *pod,
                      const koordhip_pod_ext *x, int32_t i, int nominated) {
  if (!x || !(x->flags & KOORDHIP_PODX_DEVICE)) return 0;
  if (!orc_dev_node_present(st, i)) return 0;
  const dev_rc rc = dev_rc_of(st, pod, i);
  if (nominated) {
    const int q = pod ? orc_resv_nominate(st, pod, i) : -1;
    if (q < 0 || q != rc.h || rc.cls != 1) return 0;
    return dev_score_mode(cfg, st, x, i, &rc, rc.pol == 0 ? FREE_NODE : (rc.pol == 1 ? FREE_ALIGNED : FREE_REQUIRED));
  }
  return dev_score_mode(cfg, st, x, i, &rc, FREE_NODE);
}

/* DeviceShare Reserve, plugin.go:368-405: the nominated reservation's
 * allocation (allocateWithNominatedReservation :365-407 -> tryAllocateFrom-
 * Reservation with the scorer), else the node's (the default allocator's
 * Allocate with the plugin's scorer, allocator.go:91-102); Reserve adds it to
 * deviceUsed (updateCacheUsed, allocator.go:116-118).  With the pod assumed
 * into the device-holding reservation (the Reservation Reserve, `assumed`
 * below) the next cycle's restore counts the allocation on its minors as its
 * allocated (appendAllocatedByHints, reservation.go:145-151).  Returns 0
 * (allocation in slots[t], bit s = dev slot s) or -1 (nothing committed). */
int orc_dev_reserve(const koordhip_config *cfg, orc_state *st, const koordhip_pod *pod, const koordhip_pod_ext *x,
                    int32_t i, int nominated, uint32_t *slots, int apply) {
  for (int t = 0; t < T; t++) slots[t] = 0;
  if (!x || !(x->flags & KOORDHIP_PODX_DEVICE)) return 0;
  if (!orc_dev_node_present(st, i)) return 0; /* :377-380 */
  const dev_rc rc = dev_rc_of(st, pod, i);
  int64_t per_t[T][R];
  memset(per_t, 0, sizeof(per_t));
  int r = 0;
  if (nominated) {
    const int q = pod ? orc_resv_nominate(st, pod, i) : -1;
    if (q < 0 || q != rc.h || rc.cls != 1) return -1; /* missing nominated reservation :391-393 */
    r = dev_from_reservation(cfg, st, x, i, &rc, 0, 1, slots, per_t);
    if (r < 0) return -1;
  }
  if (r == 0 && !dev_allocate(cfg, st, x, i, &rc, 0, 0, FREE_NODE, 1, slots, per_t)) return -1;
  if (apply) orc_dev_apply(st, x, i, slots, -1);
  return 0;
}

/* updateCacheUsed of an allocation (slots from orc_dev_reserve): deviceUsed
 * += the per-device request; `assumed` = the slot of the reservation the
 * Reservation Reserve assumed the pod into (-1 none): when it is the node's
 * device-holding one, its allocated grows on its minors. */
void orc_dev_apply(orc_state *st, const koordhip_pod_ext *x, int32_t i, const uint32_t *slots, int assumed) {
  const int h = orc_dev_resv_slot(st, i);
  for (int t = 0; t < T; t++) {
    if (!slots[t]) continue;
    int64_t q[R], per[R];
    (void)dev_requests(x, t, q);
    if (t == KOORDHIP_DEV_GPU) (void)dev_fill_gpu(st, i, q);
    (void)dev_wanted(t, q, per);
    uint32_t hm = 0u;
    if (h >= 0 && assumed == h)
      for (int s = 0; s < st->soa->dev_slots; s++)
        if (!is_zero(st->resv_dev + rdix(st, i, 0, t, s))) hm |= 1u << s;
    for (int s = 0; s < st->soa->dev_slots; s++)
      if ((slots[t] >> s) & 1u) {
        int64_t *u = st->dev_used + dix(st, i, t, s);
        for (int r = 0; r < R; r++) u[r] += per[r];
        if ((hm >> s) & 1u) {
          int64_t *d = st->resv_dev + rdix(st, i, 1, t, s);
          for (int r = 0; r < R; r++) d[r] += per[r];
        }
      }
  }
}

/* (upstream, UPSTREAM-ASSUMED) noderesources fitsRequest over the pod's
 * extended scalar resources: each requested key needs request <=
 * Allocatable - Requested.  1 = fits. */
int orc_xfit_filter(const orc_state *st, const koordhip_pod_ext *x, int32_t i) {
  if (!x || !x->xmask) return 1;
  const int32_t n = st->n;
  for (int j = 0; j < KOORDHIP_NXRES; j++) {
    if (!((x->xmask >> j) & 1u)) continue;
    const int64_t a = st->soa->xalloc ? st->soa->xalloc[(size_t)j * n + i] : 0;
    if (x->xreq[j] > a - st->xrequested[(size_t)j * n + i]) return 0;
  }
  return 1;
}

/* (upstream, UPSTREAM-ASSUMED) NodeAffinity Score (preferred terms' weights,
 * host-resolved per static class) and TaintToleration Score (intolerable
 * PreferNoSchedule taints) */
int64_t orc_static_score(const orc_state *st, const koordhip_pod *pod, int32_t i, int which) {
  const uint16_t *s = st->soa->static_score[which];
  return s ? (int64_t)s[(size_t)pod->static_class * (size_t)st->n + (size_t)i] : 0;
}

/* (upstream) framework/plugins/helper/normalize_score.go DefaultNormalizeScore:
 * score = maxPriority * score / max over the list (reverse: maxPriority -
 * that); all zero: unchanged, or maxPriority for every node when reversed. */
void orc_default_normalize(int64_t *scores, int32_t nf, int reverse) {
  int64_t mx = 0;
  for (int32_t j = 0; j < nf; j++)
    if (scores[j] > mx) mx = scores[j];
  if (mx == 0) {
    if (reverse)
      for (int32_t j = 0; j < nf; j++) scores[j] = 100;
    return;
  }
  for (int32_t j = 0; j < nf; j++) {
    int64_t s = 100 * scores[j] / mx;
    scores[j] = reverse ? 100 - s : s;
  }
}
