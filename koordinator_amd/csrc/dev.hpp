// dev.hpp -- DeviceShare (pkg/scheduler/plugins/deviceshare) on CDNA4 for the
// sequential cycle: Filter (plugin.go:284-323), Score (scoring.go:33-72) and
// the default allocator's Reserve (allocator.go:91-122), over the node's
// device columns; plus NodeResourcesFit's extended scalars and the upstream
// static Score columns.  Integer arithmetic as in the reference (int64; the
// only float step is memoryBytesToRatio's float64 divide and multiply,
// utils.go:207-209, built with -ffp-contract=off like the rest).
//
// Device model: per node and type up to `slots` minors (ascending), their Device
// CR resources and the amounts pods hold; free = total - used clamped at 0 per
// resource (resetDeviceFree, device_cache.go:185-202).  A request key the pod
// does not carry compares and adds as 0.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "eval.hpp"

namespace kh {

constexpr int DT = KOORDHIP_DEV_TYPES, DR = KOORDHIP_DEV_RES, DS = KOORDHIP_DEV_SLOTS;

// Device copy of koordhip_pod_ext (same layout).
struct DevPodX {
  int64_t req[DT][DR];
  int64_t xreq[KOORDHIP_NXRES];
  uint32_t flags;
  uint32_t xmask;
};
static_assert(sizeof(DevPodX) == sizeof(koordhip_pod_ext), "DevPodX mirrors koordhip_pod_ext");

__device__ __forceinline__ size_t dev_at(const DevDev &dv, int32_t i, int t, int s) {
  return ((size_t)i * DT + (size_t)t) * (size_t)dv.slots + (size_t)s;
}

// one minor of type t: its total and free resources; false = empty slot
__device__ __forceinline__ bool dev_slot(const DevDev &dv, int32_t i, int t, int s, int64_t tot[DR], int64_t fr[DR]) {
  const size_t a = dev_at(dv, i, t, s);
  if (dv.minor[a] < 0) return false;
#pragma unroll
  for (int r = 0; r < DR; r++) {
    tot[r] = dv.total[a * DR + r];
    const int64_t x = tot[r] - dv.used[a * DR + r];
    fr[r] = x > 0 ? x : 0;
  }
  return true;
}

__device__ __forceinline__ bool dev_zero(const int64_t v[DR]) { return v[0] == 0 && v[1] == 0 && v[2] == 0; }

__device__ __forceinline__ bool dev_requests(const DevPodX &x, int t, int64_t q[DR]) {
  bool any = false;
#pragma unroll
  for (int r = 0; r < DR; r++) {
    q[r] = x.req[t][r];
    any |= q[r] > 0;
  }
  return any;
}

__device__ __forceinline__ bool dev_has_type(const DevDev &dv, int32_t i, int t) {
  for (int s = 0; s < dv.slots; s++)
    if (dv.minor[dev_at(dv, i, t, s)] >= 0) return true;
  return false;
}

// fillGPUTotalMem (utils.go:211-233): memory <-> ratio from the node's GPU
// memory (the first GPU with resources; one model per node, host-checked)
__device__ __forceinline__ bool dev_fill_gpu(const DevDev &dv, int32_t i, int64_t q[DR]) {
  int64_t mem = -1;
  for (int s = 0; s < dv.slots && mem < 0; s++) {
    const size_t a = dev_at(dv, i, KOORDHIP_DEV_GPU, s);
    if (dv.minor[a] < 0) continue;
    const int64_t *t = dv.total + a * DR;
    if (t[0] != 0 || t[1] != 0 || t[2] != 0) mem = t[2];
  }
  if (mem < 0) return false;
  if (q[2] >= 0) {
    const double f = (double)q[2] / (double)mem;  // memoryBytesToRatio, float64
    q[1] = (int64_t)(f * 100.0);
  } else {
    q[2] = (q[1] > 0 ? q[1] : 0) * mem / 100;  // memoryRatioToBytes
  }
  if (q[0] < 0) q[0] = 0;
  return true;
}

// calcDeviceWanted (device_cache.go:367-395): the devices wanted and the request per device
__device__ __forceinline__ int64_t dev_wanted(int t, const int64_t q[DR], int64_t per[DR]) {
#pragma unroll
  for (int r = 0; r < DR; r++) per[r] = q[r] > 0 ? q[r] : 0;
  const int64_t key = t == KOORDHIP_DEV_GPU ? q[1] : q[0];
  if (!(key > 100 && key % 100 == 0)) return 1;
  const int64_t w = key / 100;
#pragma unroll
  for (int r = 0; r < DR; r++) per[r] = per[r] / w;
  return w;
}

__device__ __forceinline__ bool dev_fits(const int64_t per[DR], const int64_t f[DR]) {
  return per[0] <= f[0] && per[1] <= f[1] && per[2] <= f[2];
}

// leastResourceScorer / mostResourceScorer over (total, free, request) of
// type t's weighted resources (scoring.go:152-274)
__device__ __forceinline__ int64_t dev_scorer(const DevCfg &c, int t, const int64_t tot[DR], const int64_t fr[DR],
                                              const int64_t req[DR]) {
  int64_t num = 0, ws = 0;
#pragma unroll
  for (int k = 0; k < 5; k++) {
    const int kt = k < 3 ? KOORDHIP_DEV_GPU : (k == 3 ? KOORDHIP_DEV_RDMA : KOORDHIP_DEV_FPGA);
    const int r = k < 3 ? k : 0;
    const int64_t w = c.dev_w[k];
    if (w <= 0 || kt != t || tot[r] == 0) continue;
    int64_t rq = tot[r] >= fr[r] ? tot[r] - fr[r] + req[r] : tot[r];
    int64_t sc;
    if (c.dev_most) {
      if (rq > tot[r]) rq = tot[r];
      sc = rq * 100 / tot[r];
    } else {
      sc = rq > tot[r] ? 0 : (tot[r] - rq) * 100 / tot[r];
    }
    num += sc * w;
    ws += w;
  }
  return ws ? num / ws : 0;
}

__device__ __forceinline__ bool dev_present(const DevDev &dv, int32_t i) {
  return dv.slots > 0 && dv.present && dv.present[i];
}

// DeviceShare Filter: per requested type, `wanted` devices hold the per-device request
__device__ __forceinline__ bool dev_filter(const DevDev &dv, const DevPodX &x, int32_t i) {
  if (!(x.flags & KOORDHIP_PODX_DEVICE) || !dev_present(dv, i)) return true;
  for (int t = 0; t < DT; t++) {
    int64_t q[DR], per[DR], tot[DR], f[DR];
    if (!dev_requests(x, t, q)) continue;
    if (!dev_has_type(dv, i, t)) return false;
    if (t == KOORDHIP_DEV_GPU && !dev_fill_gpu(dv, i, q)) return false;
    const int64_t w = dev_wanted(t, q, per);
    int64_t cnt = 0;
    for (int s = 0; s < dv.slots; s++) {
      if (!dev_slot(dv, i, t, s, tot, f) || dev_zero(f)) continue;
      cnt += dev_fits(per, f) ? 1 : 0;
    }
    if (cnt < w) return false;
  }
  return true;
}

// DeviceShare Score (raw, before NormalizeScore); `nominated`: a reservation
// PreScore nominated on the node (no device reservation state: 0)
__device__ __forceinline__ int32_t dev_score(const DevCfg &c, const DevDev &dv, const DevPodX &x, int32_t i,
                                             bool nominated) {
  if (!(x.flags & KOORDHIP_PODX_DEVICE) || !dev_present(dv, i) || nominated) return 0;
  int64_t sum = 0;
  for (int t = 0; t < DT; t++) {
    int64_t q[DR], tot[DR], f[DR];
    if (!dev_requests(x, t, q) || !dev_has_type(dv, i, t)) continue;
    if (t == KOORDHIP_DEV_GPU && !dev_fill_gpu(dv, i, q)) continue;
    int64_t st[DR] = {0, 0, 0}, sf[DR] = {0, 0, 0};
    for (int s = 0; s < dv.slots; s++) {
      if (!dev_slot(dv, i, t, s, tot, f)) continue;
#pragma unroll
      for (int r = 0; r < DR; r++) {
        st[r] += tot[r];
        sf[r] += f[r];
      }
    }
#pragma unroll
    for (int r = 0; r < DR; r++) q[r] = q[r] > 0 ? q[r] : 0;
    sum += dev_scorer(c, t, st, sf, q);
  }
  return (int32_t)sum;
}

// DeviceShare Reserve: per requested type the devices by (device score desc,
// minor asc), the first `wanted` that hold the per-device request.  slots[t]:
// bit s = dev slot s.  apply: add the per-device request to each one's used.
// false: the Reserve fails (insufficient devices, or a nominated reservation
// DeviceShare holds no state for).
__device__ __forceinline__ bool dev_reserve(const DevCfg &c, const DevDev &dv, const DevPodX &x, int32_t i,
                                            bool nominated, uint32_t slots[DT], bool apply) {
#pragma unroll
  for (int t = 0; t < DT; t++) slots[t] = 0u;
  if (!(x.flags & KOORDHIP_PODX_DEVICE) || !dev_present(dv, i)) return true;
  if (nominated) return false;
  int64_t per_t[DT][DR];
  for (int t = 0; t < DT; t++) {
    int64_t q[DR], per[DR], tot[DR], f[DR];
#pragma unroll
    for (int r = 0; r < DR; r++) per_t[t][r] = 0;
    if (!dev_requests(x, t, q)) continue;
    if (!dev_has_type(dv, i, t)) return false;
    if (t == KOORDHIP_DEV_GPU && !dev_fill_gpu(dv, i, q)) return false;
    const int64_t w = dev_wanted(t, q, per);
    // selection: repeatedly the best unpicked fitting device (score desc, minor asc)
    int64_t got = 0;
    uint32_t taken = 0u;
    while (got < w) {
      int bs = -1;
      int64_t bsc = -1;
      int32_t bmin = 0;
      for (int s = 0; s < dv.slots; s++) {
        if ((taken >> s) & 1u) continue;
        if (!dev_slot(dv, i, t, s, tot, f) || dev_zero(f) || !dev_fits(per, f)) continue;
        const int64_t sc = dev_scorer(c, t, tot, f, per);
        const int32_t m = dv.minor[dev_at(dv, i, t, s)];
        if (bs < 0 || sc > bsc || (sc == bsc && m < bmin)) {
          bs = s;
          bsc = sc;
          bmin = m;
        }
      }
      if (bs < 0) return false;
      taken |= 1u << bs;
      got++;
    }
    slots[t] = taken;
#pragma unroll
    for (int r = 0; r < DR; r++) per_t[t][r] = per[r];
  }
  if (apply)
    for (int t = 0; t < DT; t++)
      for (int s = 0; s < dv.slots; s++)
        if ((slots[t] >> s) & 1u) {
          const size_t a = dev_at(dv, i, t, s) * DR;
#pragma unroll
          for (int r = 0; r < DR; r++) dv.used[a + r] += per_t[t][r];
        }
  return true;
}

// NodeResourcesFit over the extended scalars the pod requests (upstream fitsRequest)
__device__ __forceinline__ bool xfit_filter(const DevDev &dv, const DevPodX &x, int32_t i, int32_t n) {
  if (!x.xmask) return true;
  for (int j = 0; j < KOORDHIP_NXRES; j++) {
    if (!((x.xmask >> j) & 1u)) continue;
    const int64_t a = dv.xalloc ? dv.xalloc[(size_t)j * n + i] : 0;
    if (x.xreq[j] > a - dv.xreq[(size_t)j * n + i]) return false;
  }
  return true;
}

__device__ __forceinline__ int32_t static_raw(const DevDev &dv, int which, int32_t cls, int32_t i, int32_t n) {
  const uint16_t *s = dv.sscore[which];
  return s ? (int32_t)s[(size_t)cls * n + i] : 0;
}

}  // namespace kh
