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
  uint8_t pts_n, pts_class, pts_match, pts_pad;
  uint8_t pts_c[KOORDHIP_PTS_POD];
  uint8_t pts_fl[KOORDHIP_PTS_POD];
  int32_t pts_skew[KOORDHIP_PTS_POD];
  int32_t reserve_node;  // KOORDHIP_POD_RESERVE: 1 + the node its reservation names, 0 = any
  uint32_t ipa_inc, ipa_aff, ipa_anti, ipa_score, ipa_flags;
  int32_t ipa_reserved;
  int32_t ipa_w[KOORDHIP_IPA_ENTRIES];
};
static_assert(sizeof(DevPodX) == sizeof(koordhip_pod_ext), "DevPodX mirrors koordhip_pod_ext");

__device__ __forceinline__ size_t dev_at(const DevDev &dv, int32_t i, int t, int s) {
  return ((size_t)i * DT + (size_t)t) * (size_t)dv.slots + (size_t)s;
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

// A node's minors of one type, loaded once: every slot's minor, total and
// free issue back to back (unrolled over KOORDHIP_DEV_SLOTS) instead of one
// dependent round trip per slot and per plugin.
struct DevRow {
  int32_t minor[DS];
  int64_t tot[DS][DR];
  int64_t fr[DS][DR];
};

__device__ __forceinline__ void dev_load(const DevDev &dv, int32_t i, int t, DevRow &w) {
  const size_t a0 = dev_at(dv, i, t, 0);
#pragma unroll
  for (int s = 0; s < DS; s++) {
    const bool on = s < dv.slots;
    w.minor[s] = on ? dv.minor[a0 + s] : -1;
#pragma unroll
    for (int r = 0; r < DR; r++) {
      const int64_t tt = on ? dv.total[(a0 + s) * DR + r] : 0;
      const int64_t x = tt - (on ? dv.used[(a0 + s) * DR + r] : 0);
      w.tot[s][r] = tt;
      w.fr[s][r] = x > 0 ? x : 0;
    }
  }
}

__device__ __forceinline__ bool dev_has_type(const DevRow &w) {
  bool any = false;
#pragma unroll
  for (int s = 0; s < DS; s++) any |= w.minor[s] >= 0;
  return any;
}

// fillGPUTotalMem (utils.go:211-233): memory <-> ratio from the node's GPU
// memory (the first GPU with resources; one model per node, host-checked)
__device__ __forceinline__ bool dev_fill_gpu(const DevRow &w, int64_t q[DR]) {
  int64_t mem = -1;
#pragma unroll
  for (int s = DS - 1; s >= 0; s--)
    if (w.minor[s] >= 0 && (w.tot[s][0] != 0 || w.tot[s][1] != 0 || w.tot[s][2] != 0)) mem = w.tot[s][2];
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

// floor(a / b) for 0 <= a <= 100 b, 0 < b < 2^45: the quotient is at most 100,
// so the f64 reciprocal estimate is within one of it and one exact fix-up step
// (the remainder by fma) settles it -- int64 division without the 64-bit
// software divide (the same device as eval.hpp lrs / mrs)
__device__ __forceinline__ int64_t dev_pct_div(int64_t a, int64_t b) {
  const double fa = (double)a, fb = (double)b;
  int64_t q = (int64_t)(fa * __builtin_amdgcn_rcp(fb));
  const double r = __builtin_fma(-(double)q, fb, fa);
  q -= (r < 0.0);
  q += (r >= fb);
  return q;
}

// leastResourceScorer / mostResourceScorer over (total, free, request) of
// type t's weighted resources (scoring.go:152-274)
__device__ __forceinline__ int64_t dev_scorer(const DevCfg &c, int t, const int64_t tot[DR], const int64_t fr[DR],
                                              const int64_t req[DR]) {
  int32_t num = 0, ws = 0;
#pragma unroll
  for (int k = 0; k < 5; k++) {
    const int kt = k < 3 ? KOORDHIP_DEV_GPU : (k == 3 ? KOORDHIP_DEV_RDMA : KOORDHIP_DEV_FPGA);
    const int r = k < 3 ? k : 0;
    const int32_t w = c.dev_w[k];
    if (w <= 0 || kt != t || tot[r] == 0) continue;
    int64_t rq = tot[r] >= fr[r] ? tot[r] - fr[r] + req[r] : tot[r];
    int64_t sc;
    if (c.dev_most) {
      if (rq > tot[r]) rq = tot[r];
      sc = dev_pct_div(rq * 100, tot[r]);
    } else {
      sc = rq > tot[r] ? 0 : dev_pct_div((tot[r] - rq) * 100, tot[r]);
    }
    num += (int32_t)sc * w;
    ws += w;
  }
  return ws ? num / ws : 0;
}

__device__ __forceinline__ bool dev_present(const DevDev &dv, int32_t i) {
  return dv.slots > 0 && dv.present && dv.present[i];
}

// DeviceShare Filter (plugin.go:284-323: per requested type, `wanted`
// devices hold the per-device request) and the raw Score (scoring.go:33-72,
// before NormalizeScore; computed on infeasible nodes too, like the
// reference's planes) in one pass over the node's device rows.  `nominated`:
// a reservation PreScore nominated on the node (no device reservation state:
// Score 0).  Returns the Filter verdict.
__device__ __forceinline__ bool dev_eval(const DevCfg &c, const DevDev &dv, const DevPodX &x, int32_t i,
                                         bool nominated, bool filter, bool score, int32_t *raw) {
  *raw = 0;
  if (!(x.flags & KOORDHIP_PODX_DEVICE) || dv.slots <= 0 || !dv.present) return true;
  // the nodeDevice entry and the first requested type's rows in one round trip
  const bool present = dv.present[i] != 0;
  bool ok = true;
  int64_t sum = 0;
#pragma unroll 1
  for (int t = 0; t < DT; t++) {
    int64_t q[DR];
    if (!dev_requests(x, t, q)) continue;
    DevRow w;
    dev_load(dv, i, t, w);
    if (!present) return true;
    if (!dev_has_type(w) || (t == KOORDHIP_DEV_GPU && !dev_fill_gpu(w, q))) {
      ok = false;
      continue;
    }
    if (filter) {
      int64_t per[DR];
      const int64_t want = dev_wanted(t, q, per);
      int64_t cnt = 0;
#pragma unroll
      for (int s = 0; s < DS; s++)
        cnt += (w.minor[s] >= 0 && !dev_zero(w.fr[s]) && dev_fits(per, w.fr[s])) ? 1 : 0;
      ok &= cnt >= want;
    }
    if (score && !nominated) {
      int64_t st[DR] = {0, 0, 0}, sf[DR] = {0, 0, 0};
#pragma unroll
      for (int s = 0; s < DS; s++)
        if (w.minor[s] >= 0)
#pragma unroll
          for (int r = 0; r < DR; r++) {
            st[r] += w.tot[s][r];
            sf[r] += w.fr[s][r];
          }
#pragma unroll
      for (int r = 0; r < DR; r++) q[r] = q[r] > 0 ? q[r] : 0;
      sum += dev_scorer(c, t, st, sf, q);
    }
  }
  *raw = (int32_t)sum;
  return ok || !filter;
}

// DeviceShare Reserve (allocator.go:91-122): per requested type the devices
// by (device score desc, minor asc), the first `wanted` that hold the
// per-device request.  slots[t]: bit s = dev slot s; per[t]: the per-device
// request dev_apply adds.  false: the Reserve fails (insufficient devices, or
// a nominated reservation DeviceShare holds no state for).
__device__ __forceinline__ bool dev_reserve(const DevCfg &c, const DevDev &dv, const DevPodX &x, int32_t i,
                                            bool nominated, uint32_t slots[DT], int64_t per_t[DT][DR]) {
#pragma unroll
  for (int t = 0; t < DT; t++) {
    slots[t] = 0u;
#pragma unroll
    for (int r = 0; r < DR; r++) per_t[t][r] = 0;
  }
  if (!(x.flags & KOORDHIP_PODX_DEVICE) || dv.slots <= 0 || !dv.present) return true;
  const bool present = dv.present[i] != 0;  // (issued with the first type's rows)
  bool any = false;
  for (int t = 0; t < DT; t++) {
    int64_t q[DR], per[DR];
    if (!dev_requests(x, t, q)) continue;
    any = true;
    DevRow w;
    dev_load(dv, i, t, w);
    if (!present) return true;
    if (nominated) return false;
    if (!dev_has_type(w)) return false;
    if (t == KOORDHIP_DEV_GPU && !dev_fill_gpu(w, q)) return false;
    const int64_t want = dev_wanted(t, q, per);
    // every fitting device's score once, then the best `want` by (score desc, minor asc)
    int64_t sc[DS];
#pragma unroll
    for (int s = 0; s < DS; s++)
      sc[s] = (w.minor[s] >= 0 && !dev_zero(w.fr[s]) && dev_fits(per, w.fr[s])) ? dev_scorer(c, t, w.tot[s], w.fr[s], per)
                                                                               : -1;
    uint32_t taken = 0u;
    for (int64_t got = 0; got < want; got++) {
      // the best untaken slot by (score desc, minor asc); the running best's
      // score and minor in registers (sc[bs] with a dynamic bs would live in scratch)
      int bs = -1;
      int64_t bsc = -1;
      int32_t bmi = 0;
#pragma unroll
      for (int s = 0; s < DS; s++) {
        if (sc[s] < 0 || ((taken >> s) & 1u)) continue;
        if (bs < 0 || sc[s] > bsc || (sc[s] == bsc && w.minor[s] < bmi)) {
          bs = s;
          bsc = sc[s];
          bmi = w.minor[s];
        }
      }
      if (bs < 0) return false;
      taken |= 1u << bs;
    }
    slots[t] = taken;
#pragma unroll
    for (int r = 0; r < DR; r++) per_t[t][r] = per[r];
  }
  return any || !present || !nominated;
}

// WT: write-through stores (k_ext_final: read next on other XCDs after a
// relaxed hand-off, no L2 write-back fence)
template <bool WT = false>
__device__ __forceinline__ void dev_apply(const DevDev &dv, int32_t i, const uint32_t slots[DT],
                                          const int64_t per_t[DT][DR]) {
  for (int t = 0; t < DT; t++) {
    if (!slots[t]) continue;
    // every taken slot's used values loaded before any store (one round trip)
    int64_t u[DS][DR];
    const size_t a0 = dev_at(dv, i, t, 0) * DR;
#pragma unroll
    for (int s = 0; s < DS; s++)
#pragma unroll
      for (int r = 0; r < DR; r++) u[s][r] = ((slots[t] >> s) & 1u) ? dv.used[a0 + (size_t)s * DR + r] : 0;
#pragma unroll
    for (int s = 0; s < DS; s++)
      if ((slots[t] >> s) & 1u)
#pragma unroll
        for (int r = 0; r < DR; r++) {
          if constexpr (WT)
            st_wt(&dv.used[a0 + (size_t)s * DR + r], (int64_t)(u[s][r] + per_t[t][r]));
          else
            dv.used[a0 + (size_t)s * DR + r] = u[s][r] + per_t[t][r];
        }
  }
}

// ---- DeviceShare with the node's reservation holding devices ------------
// (deviceshare/reservation.go:119-443; oracle/dev_oracle.c restates the same
// rules).  One such reservation per node (host-checked), slot h; for the pod
// its restore class (1 matched, 2 unmatched with assigned pods) and
// AllocatePolicy.  Per minor: remained Rm = max0(A - D); the preemptible amount
// P of a free mode -- RC_NODE: (class 2) A - Rm, (class 1) A; RC_ALIGNED:
// (class 1) D + Rm -- and the free resources max0(total - max0(used - P));
// RC_REQUIRED: Rm itself on a type calcRequiredDeviceResources names.  Rare
// (a device pod on a node whose reservation holds devices), so these run out
// of line: the common device path keeps its registers.
struct DevRC {
  int32_t h;    // reservation slot holding devices, -1 none
  int32_t cls;  // its class for the pod
  int32_t pol;  // its AllocatePolicy
  uint32_t rq;  // bit t: calcRequiredDeviceResources names type t
};
enum { RC_NODE = 0, RC_ALIGNED = 1, RC_REQUIRED = 2 };

__device__ __forceinline__ size_t rdev_at(const DevDev &dv, int32_t i, int half, int t, int s) {
  return ((((size_t)i * 2 + (size_t)half) * DT + (size_t)t) * (size_t)dv.slots + (size_t)s) * DR;
}

// calcRequiredDeviceResources (reservation.go:344-363): the types it names --
// those with a minor left in Rm, or (Rm empty) every type the reservation holds
__device__ __noinline__ uint32_t rc_required_types(const DevDev &dv, int32_t i) {
  uint32_t left = 0u, held = 0u;
  for (int t = 0; t < DT; t++)
    for (int s = 0; s < dv.slots; s++) {
      const size_t a = rdev_at(dv, i, 0, t, s), d = rdev_at(dv, i, 1, t, s);
      for (int r = 0; r < DR; r++) {
        const int64_t av = dv.rdev[a + r], dd = dv.rdev[d + r];
        held |= (av != 0 ? 1u : 0u) << t;
        left |= (av - dd > 0 ? 1u : 0u) << t;
      }
    }
  return left ? left : held;
}

// the free resources of dev slot s of type t in `mode`; *hint: the slot is one
// of the reservation's minors (A nonzero)
__device__ __forceinline__ void rc_free_slot(const DevDev &dv, int32_t i, const DevRC &rc, int mode, int t, int s,
                                             int64_t f[DR], bool *hint) {
  const size_t a = rdev_at(dv, i, 0, t, s), d = rdev_at(dv, i, 1, t, s), u = dev_at(dv, i, t, s) * DR;
  int64_t A[DR], D[DR], Rm[DR];
  bool h = false;
#pragma unroll
  for (int r = 0; r < DR; r++) {
    A[r] = dv.rdev[a + r];
    D[r] = dv.rdev[d + r];
    Rm[r] = A[r] - D[r] > 0 ? A[r] - D[r] : 0;
    h |= A[r] != 0;
  }
  *hint = h;
  if (mode == RC_REQUIRED && ((rc.rq >> t) & 1u)) {
#pragma unroll
    for (int r = 0; r < DR; r++) f[r] = Rm[r];
    return;
  }
  if (mode == RC_REQUIRED) mode = RC_ALIGNED;
#pragma unroll
  for (int r = 0; r < DR; r++) {
    int64_t p = 0;
    if (rc.cls == 2) p += A[r] - Rm[r];
    if (rc.cls == 1) p += mode == RC_NODE ? A[r] : D[r] + Rm[r];
    const int64_t uu = dv.used[u + r] - p > 0 ? dv.used[u + r] - p : 0;
    const int64_t tt = dv.total[u + r];
    f[r] = tt - uu > 0 ? tt - uu : 0;
  }
}

// tryAllocateDevice over the pod's types with the reservation's hints
// (device_cache.go:272-365): `req` keeps to its minors (a type it holds none of
// is not restricted), `pref` orders them first, then the scorer's score
// (`scorer`; else 0) desc, minor asc; `want` fitting non-zero devices per type.
__device__ __noinline__ bool rc_allocate(const DevCfg &c, const DevDev &dv, const DevPodX &x, int32_t i,
                                         const DevRC &rc, bool req, bool pref, int mode, bool scorer,
                                         uint32_t slots[DT], int64_t per_t[DT][DR]) {
  for (int t = 0; t < DT; t++) {
    slots[t] = 0u;
    for (int r = 0; r < DR; r++) per_t[t][r] = 0;
  }
  for (int t = 0; t < DT; t++) {
    int64_t q[DR], per[DR];
    if (!dev_requests(x, t, q)) continue;
    DevRow w;
    dev_load(dv, i, t, w);
    if (!dev_has_type(w)) return false;
    if (t == KOORDHIP_DEV_GPU && !dev_fill_gpu(w, q)) return false;
    const int64_t want = dev_wanted(t, q, per);
    uint32_t hm = 0u;
    int64_t sc[DS];
    for (int s = 0; s < DS; s++) {
      sc[s] = -1;
      if (s >= dv.slots || w.minor[s] < 0) continue;
      int64_t f[DR];
      bool h;
      rc_free_slot(dv, i, rc, mode, t, s, f, &h);
      hm |= (h ? 1u : 0u) << s;
      if (!dev_zero(f) && dev_fits(per, f)) sc[s] = scorer ? dev_scorer(c, t, w.tot[s], f, per) : 0;
    }
    uint32_t taken = 0u;
    for (int64_t got = 0; got < want; got++) {
      int bs = -1;
      int64_t bsc = -1;
      int32_t bmi = 0;
      bool bpf = false;
      for (int s = 0; s < DS; s++) {
        if (sc[s] < 0 || ((taken >> s) & 1u)) continue;
        if (req && hm && !((hm >> s) & 1u)) continue;
        const bool pf = pref && ((hm >> s) & 1u);
        if (bs < 0 || (pf && !bpf) || (pf == bpf && (sc[s] > bsc || (sc[s] == bsc && w.minor[s] < bmi)))) {
          bs = s;
          bsc = sc[s];
          bmi = w.minor[s];
          bpf = pf;
        }
      }
      if (bs < 0) return false;
      taken |= 1u << bs;
    }
    slots[t] = taken;
    for (int r = 0; r < DR; r++) per_t[t][r] = per[r];
  }
  return true;
}

// tryAllocateFromReservation (reservation.go:181-283) over the matched
// reservation holding devices: 1 allocated, 0 none (fall back to the node),
// -1 Unschedulable (Aligned / Restricted that cannot hold the pod).
// fromResv: requiredFromReservation (FilterReservation).
__device__ __forceinline__ int rc_from_reservation(const DevCfg &c, const DevDev &dv, const DevPodX &x, int32_t i,
                                                   const DevRC &rc, bool fromResv, bool scorer, uint32_t slots[DT],
                                                   int64_t per_t[DT][DR]) {
  if (rc.h < 0 || rc.cls != 1) return 0;
  if (rc.pol == 0) return rc_allocate(c, dv, x, i, rc, fromResv, true, RC_NODE, scorer, slots, per_t) ? 1 : 0;
  if (rc.pol == 1) return rc_allocate(c, dv, x, i, rc, true, true, RC_ALIGNED, scorer, slots, per_t) ? 1 : -1;
  if (!rc_allocate(c, dv, x, i, rc, true, true, RC_ALIGNED, false, slots, per_t)) return -1;
  return rc_allocate(c, dv, x, i, rc, true, true, RC_REQUIRED, scorer, slots, per_t) ? 1 : -1;
}

// the node's reservation holding devices for a device pod (rc.h -1: none or
// no restore).  `klass`: the restore class of slot q (resv_class).
__device__ __forceinline__ DevRC rc_of(const DevCfg &c, const DevDev &dv, int32_t i, int32_t h, int32_t klass,
                                       uint32_t rf) {
  DevRC rc{-1, 0, 0, 0u};
  if (!dv.rslot || !c.resv || h < 0) return rc;
  rc.h = h;
  rc.cls = klass;
  rc.pol = (int32_t)KOORDHIP_RESV_POLICY(rf);
  rc.rq = (rc.cls == 1 && rc.pol == 2) ? rc_required_types(dv, i) : 0u;
  return rc;
}

// DeviceShare FilterReservation (plugin.go:325-356) of the matched reservation holding devices
__device__ __noinline__ bool rc_filter_reservation(const DevCfg &c, const DevDev &dv, const DevPodX &x, int32_t i,
                                                   const DevRC &rc) {
  if (!dev_present(dv, i)) return true;
  uint32_t slots[DT];
  int64_t per[DT][DR];
  return rc_from_reservation(c, dv, x, i, rc, true, false, slots, per) > 0;
}

// scoreNode per requested type over the free devices of `mode`
__device__ __noinline__ int64_t rc_score(const DevCfg &c, const DevDev &dv, const DevPodX &x, int32_t i,
                                         const DevRC &rc, int mode) {
  int64_t sum = 0;
  for (int t = 0; t < DT; t++) {
    int64_t q[DR];
    if (!dev_requests(x, t, q)) continue;
    DevRow w;
    dev_load(dv, i, t, w);
    if (!dev_has_type(w) || (t == KOORDHIP_DEV_GPU && !dev_fill_gpu(w, q))) continue;
    int64_t st[DR] = {0, 0, 0}, sf[DR] = {0, 0, 0};
    for (int s = 0; s < DS; s++) {
      if (s >= dv.slots || w.minor[s] < 0) continue;
      int64_t f[DR];
      bool h;
      rc_free_slot(dv, i, rc, mode, t, s, f, &h);
      for (int r = 0; r < DR; r++) {
        st[r] += w.tot[s][r];
        sf[r] += f[r];
      }
    }
    for (int r = 0; r < DR; r++) q[r] = q[r] > 0 ? q[r] : 0;
    sum += dev_scorer(c, t, st, sf, q);
  }
  return sum;
}

// DeviceShare Filter and raw Score on a node whose reservation holds devices
// (plugin.go:284-323, scoring.go:33-72 with scoreWithNominatedReservation);
// `nomq`: the reservation slot PreScore nominated (-1 none)
__device__ __noinline__ bool rc_eval(const DevCfg &c, const DevDev &dv, const DevPodX &x, int32_t i, const DevRC &rc,
                                     int32_t nomq, bool filter, bool score, int32_t *raw) {
  *raw = 0;
  if (!dev_present(dv, i)) return true;
  bool ok = true;
  if (filter) {
    uint32_t slots[DT];
    int64_t per[DT][DR];
    const int r = rc_from_reservation(c, dv, x, i, rc, false, false, slots, per);
    ok = r != 0 ? r > 0 : rc_allocate(c, dv, x, i, rc, false, false, RC_NODE, false, slots, per);
  }
  if (score) {
    if (nomq >= 0)
      *raw = (nomq == rc.h && rc.cls == 1)
                 ? (int32_t)rc_score(c, dv, x, i, rc, rc.pol == 0 ? RC_NODE : (rc.pol == 1 ? RC_ALIGNED : RC_REQUIRED))
                 : 0;
    else
      *raw = (int32_t)rc_score(c, dv, x, i, rc, RC_NODE);
  }
  return ok || !filter;
}

// DeviceShare Reserve on such a node (plugin.go:368-405): the nominated
// reservation's allocation (`nomq`, -1 none), else the node's
__device__ __noinline__ bool rc_reserve(const DevCfg &c, const DevDev &dv, const DevPodX &x, int32_t i,
                                        const DevRC &rc, int32_t nomq, uint32_t slots[DT], int64_t per_t[DT][DR]) {
  for (int t = 0; t < DT; t++) {
    slots[t] = 0u;
    for (int r = 0; r < DR; r++) per_t[t][r] = 0;
  }
  if (!(x.flags & KOORDHIP_PODX_DEVICE) || !dev_present(dv, i)) return true;
  int r = 0;
  if (nomq >= 0) {
    if (nomq != rc.h || rc.cls != 1) return false;
    r = rc_from_reservation(c, dv, x, i, rc, false, true, slots, per_t);
    if (r < 0) return false;
  }
  return r > 0 || rc_allocate(c, dv, x, i, rc, false, false, RC_NODE, true, slots, per_t);
}

// the assumed pod's allocation on the reservation's minors joins its allocated
template <bool WT = false>
__device__ __noinline__ void rc_apply_allocated(const DevDev &dv, int32_t i, const uint32_t slots[DT],
                                                const int64_t per_t[DT][DR]) {
  for (int t = 0; t < DT; t++)
    for (int s = 0; s < dv.slots; s++) {
      if (!((slots[t] >> s) & 1u)) continue;
      const size_t a = rdev_at(dv, i, 0, t, s), d = rdev_at(dv, i, 1, t, s);
      if (dv.rdev[a] == 0 && dv.rdev[a + 1] == 0 && dv.rdev[a + 2] == 0) continue;  // not its minor
      for (int r = 0; r < DR; r++) {
        if constexpr (WT)
          st_wt(&dv.rdev[d + r], (int64_t)(dv.rdev[d + r] + per_t[t][r]));
        else
          dv.rdev[d + r] += per_t[t][r];
      }
    }
}

// NodeResourcesFit over the extended scalars the pod requests (upstream fitsRequest)
__device__ __forceinline__ bool xfit_filter(const DevDev &dv, const DevPodX &x, int32_t i, int32_t n) {
  if (!x.xmask) return true;
  // no early exit: every requested scalar's loads in flight together
  bool ok = true;
#pragma unroll
  for (int j = 0; j < KOORDHIP_NXRES; j++) {
    if (!((x.xmask >> j) & 1u)) continue;
    const int64_t a = dv.xalloc ? dv.xalloc[(size_t)j * n + i] : 0;
    ok &= x.xreq[j] <= a - dv.xreq[(size_t)j * n + i];
  }
  return ok;
}

__device__ __forceinline__ int32_t static_raw(const DevDev &dv, int which, int32_t cls, int32_t i, int32_t n) {
  const uint16_t *s = dv.sscore[which];
  return s ? (int32_t)s[(size_t)cls * n + i] : 0;
}

}  // namespace kh
