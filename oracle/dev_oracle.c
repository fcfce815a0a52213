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

/* resetDeviceFree, device_cache.go:185-202 (SubtractWithNonNegativeResult) */
static void dev_free(const orc_state *st, int32_t i, int t, int s, int64_t f[R]) {
  const int64_t *tot = st->soa->dev_total + dix(st, i, t, s);
  const int64_t *used = st->dev_used + dix(st, i, t, s);
  for (int r = 0; r < R; r++) {
    const int64_t x = tot[r] - used[r];
    f[r] = x > 0 ? x : 0;
  }
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

/* DeviceShare Filter, plugin.go:284-323 -> tryAllocateDevice (device_cache.go:
 * 272-314) with no scorer: per requested type, the node needs its devices
 * (:286-289), the GPU memory fill (:291-295) and `wanted` devices whose free
 * resources hold the per-device request, unhealthy (zero) ones skipped
 * (tryAllocateByDeviceType :316-365).  1 = passes. */
int orc_dev_filter(const orc_state *st, const koordhip_pod_ext *x, int32_t i) {
  if (!x || !(x->flags & KOORDHIP_PODX_DEVICE)) return 1; /* state.skip */
  if (!orc_dev_node_present(st, i)) return 1;           /* nodeDeviceInfo == nil: :298-301 */
  for (int t = 0; t < T; t++) {
    int64_t q[R], per[R], f[R];
    if (!dev_requests(x, t, q)) continue;
    if (!has_type(st, i, t)) return 0;
    if (t == KOORDHIP_DEV_GPU && !dev_fill_gpu(st, i, q)) return 0;
    const int64_t w = dev_wanted(t, q, per);
    int64_t cnt = 0;
    for (int s = 0; s < st->soa->dev_slots; s++) {
      if (dminor(st, i, t, s) < 0) continue;
      dev_free(st, i, t, s, f);
      if (is_zero(f)) continue;
      if (dev_fits(per, f)) cnt++;
    }
    if (cnt < w) return 0;
  }
  return 1;
}

/* DeviceShare Score, scoring.go:33-72 -> nodeDevice.score (device_cache.go:
 * 397-452): per requested type, scoreNode over the sums of the node's device
 * totals and frees with the (GPU-filled) pod request; the types add up.
 * `nominated`: the Reservation plugin nominated a reservation on the node
 * (no DeviceShare reservation state: the score is 0, :54-59 / reservation.go:
 * 409-431). */
int64_t orc_dev_score(const koordhip_config *cfg, const orc_state *st, const koordhip_pod_ext *x, int32_t i,
                      int nominated) {
  if (!x || !(x->flags & KOORDHIP_PODX_DEVICE)) return 0;
  if (!orc_dev_node_present(st, i) || nominated) return 0;
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
      dev_free(st, i, t, s, f);
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

typedef struct dev_pick {
  int32_t s, minor;
  int64_t score;
} dev_pick;

static int pick_cmp(const void *a, const void *b) {
  const dev_pick *x = (const dev_pick *)a, *y = (const dev_pick *)b;
  if (x->score != y->score) return x->score > y->score ? -1 : 1;
  return x->minor < y->minor ? -1 : (x->minor > y->minor ? 1 : 0);
}

/* DeviceShare Reserve, plugin.go:368-405 -> the default allocator's Allocate
 * with the plugin's scorer (allocator.go:91-102) and Reserve (:116-118): per
 * requested type the devices ordered by scoreDevices (device_resources.go:
 * 161-175) and sortDeviceResourcesByMinor (:177-195: score desc, minor asc; no
 * preferred minors), the first `wanted` that hold the per-device request;
 * updateCacheUsed adds it to each.  Returns 0 (allocation in slots[t], bit s =
 * dev slot s) or -1 (insufficient devices / a nominated reservation: the
 * Reserve fails and nothing is committed).  apply = 0: nothing changes. */
int orc_dev_reserve(const koordhip_config *cfg, orc_state *st, const koordhip_pod_ext *x, int32_t i, int nominated,
                    uint32_t *slots, int apply) {
  for (int t = 0; t < T; t++) slots[t] = 0;
  if (!x || !(x->flags & KOORDHIP_PODX_DEVICE)) return 0;
  if (!orc_dev_node_present(st, i)) return 0; /* :377-380 */
  if (nominated) return -1;                   /* allocateWithNominatedReservation: missing nominated reservation */
  int64_t per_t[T][R];
  for (int t = 0; t < T; t++) {
    int64_t q[R], per[R], f[R];
    if (!dev_requests(x, t, q)) continue;
    if (!has_type(st, i, t)) return -1;
    if (t == KOORDHIP_DEV_GPU && !dev_fill_gpu(st, i, q)) return -1;
    const int64_t w = dev_wanted(t, q, per);
    dev_pick pk[KOORDHIP_DEV_SLOTS];
    int np = 0;
    for (int s = 0; s < st->soa->dev_slots; s++) {
      const int32_t m = dminor(st, i, t, s);
      if (m < 0) continue;
      dev_free(st, i, t, s, f);
      pk[np].s = s;
      pk[np].minor = m;
      pk[np].score = dev_scorer(cfg, t, st->soa->dev_total + dix(st, i, t, s), f, per);
      np++;
    }
    qsort(pk, (size_t)np, sizeof(dev_pick), pick_cmp);
    int64_t got = 0;
    for (int j = 0; j < np && got < w; j++) {
      dev_free(st, i, t, pk[j].s, f);
      if (is_zero(f) || !dev_fits(per, f)) continue;
      slots[t] |= 1u << pk[j].s;
      got++;
    }
    if (got < w) return -1;
    memcpy(per_t[t], per, sizeof(per));
  }
  if (!apply) return 0;
  for (int t = 0; t < T; t++)
    for (int s = 0; s < st->soa->dev_slots; s++)
      if ((slots[t] >> s) & 1u) {
        int64_t *u = st->dev_used + dix(st, i, t, s);
        for (int r = 0; r < R; r++) u[r] += per_t[t][r];
      }
  return 0;
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
