// resv.hpp -- the Reservation plugin's per-(pod, node) part on CDNA4: the
// BeforePreFilter restore of the node's reservation (reservation/
// transformer.go:48-293), filterWithReservations (plugin.go:373-494), the
// nomination filter (plugin.go:504-535), scoreReservation (scoring.go:177-200)
// and the Reserve into the nominated reservation (reservation_info.go:297-306).
//
// The reference normalises the Reservation score over the pod's feasible
// nodes (DefaultNormalizeScore) and weighs it 5000.  With a weight above 100 x
// the other plugins' weights (host-checked) one normalised unit outweighs any
// other total, so the argmax -- and the order of any two nodes while no node
// is "preferred" -- equals the lexicographic order of (raw score, other
// plugins' total); a preferred node (smallest reservation order) wins
// outright.  The ranking total below encodes exactly that per node, so the
// top-k / resolve machinery keeps working on independent per-node keys:
//   ordered matched reservation:  T2 + (MAX_ORDERS - 1 - rank)
//   nominated, raw score s > 0:   s * (B + 1) + b
//   otherwise:                    b
// with b the other plugins' total, B its maximum and T2 = 101 (B + 1).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/koordhip.h"

namespace kh {

// A NUMA side row with the node's reservation (NM == 3 builds).
struct NumaRowR : NumaRow {
  double ra[2], rd[2], rz[2];
  int32_t rn;
  uint32_t rf;  // KOORDHIP_RESV_* (0: none)
  int32_t rk;
  int32_t rpad;
};

constexpr double RESV_NZ_CPU = 100.0;                         // (upstream) DefaultMilliCPURequest
constexpr double RESV_NZ_MEM = 200.0 * 1024.0 * 1024.0;       // (upstream) DefaultMemoryRequest

__device__ __forceinline__ void load_resv(NumaRowR &r, const DevResv &d, int32_t i) {
  r.rf = d.flags[i];
  r.rn = 0;
  r.rk = 0;
#pragma unroll
  for (int k = 0; k < 2; k++) r.ra[k] = r.rd[k] = r.rz[k] = 0.0;
  if (r.rf & KOORDHIP_RESV_PRESENT) {
    r.rn = d.rn[i];
    r.rk = d.rank[i];
#pragma unroll
    for (int k = 0; k < 2; k++) {
      r.ra[k] = d.ra[k][i];
      r.rd[k] = d.rd[k][i];
      r.rz[k] = d.rz[k][i];
    }
  }
}

__device__ __forceinline__ void store_resv(const NumaRowR &r, const DevResv &d, int32_t i) {
  if (!(r.rf & KOORDHIP_RESV_PRESENT)) return;
  d.rd[0][i] = r.rd[0];
  d.rd[1][i] = r.rd[1];
  d.rn[i] = r.rn;
}
__device__ __forceinline__ void store_resv_wt(const NumaRowR &r, const DevResv &d, int32_t i) {  // write-through
  if (!(r.rf & KOORDHIP_RESV_PRESENT)) return;
  st_wt(&d.rd[0][i], r.rd[0]);
  st_wt(&d.rd[1][i], r.rd[1]);
  st_wt(&d.rn[i], r.rn);
}

__device__ __forceinline__ bool rkey(uint32_t rf, int k) {
  return (rf & (k == 0 ? KOORDHIP_RESV_KEY_CPU : KOORDHIP_RESV_KEY_MEM)) != 0;
}
__device__ __forceinline__ bool pkey(const DevPod &p, int k) {
  return (p.flags & (k == 0 ? KOORDHIP_POD_KEY_CPU : KOORDHIP_POD_KEY_MEM)) != 0;
}
__device__ __forceinline__ double rem_of(const NumaRowR &r, int k) {
  const double x = r.ra[k] - r.rd[k];
  return rkey(r.rf, k) && x > 0.0 ? x : 0.0;  // SubtractWithNonNegativeResult(Allocatable, Allocated)
}

// transformer.go:86-103: 1 = matched, 2 = unmatched with assigned pods, 0 = untouched
__device__ __forceinline__ int resv_class(const NumaRowR &r, const DevPod &p) {
  if (!(r.rf & KOORDHIP_RESV_PRESENT)) return 0;
  if ((r.rf & KOORDHIP_RESV_ALLOCATE_ONCE) && r.rn > 0) return 0;
  const bool match = (p.resv_match >> KOORDHIP_RESV_GROUP(r.rf)) & 1ull;
  if (!(r.rf & KOORDHIP_RESV_UNSCHEDULABLE) && match) return 1;
  return r.rn > 0 ? 2 : 0;
}

// The restore on the node's values (restoreMatchedReservation /
// restoreUnmatchedReservations), then the Fit over-commit bits of the result.
__device__ __forceinline__ void resv_restore(NV &v, const NumaRowR &r, int cls) {
  if (cls == 0) return;
  v.r[KOORDHIP_RES_CPU] -= r.ra[0];
  v.r[KOORDHIP_RES_MEM] -= r.ra[1];
  v.nz_cpu -= r.rz[0];
  v.nz_mem -= r.rz[1];
  if (cls == 1) {
    v.npods -= 1;  // NodeInfo.RemovePod(reservePod)
  } else {
    const double rc = rem_of(r, 0), rm = rem_of(r, 1);
    if (rc > 0.0 || rm > 0.0) {  // a pod requesting the remainder comes back
      v.r[KOORDHIP_RES_CPU] += rc;
      v.r[KOORDHIP_RES_MEM] += rm;
      v.nz_cpu += rkey(r.rf, 0) ? rc : RESV_NZ_CPU;
      v.nz_mem += rkey(r.rf, 1) ? rm : RESV_NZ_MEM;
    }
  }
  uint32_t f = v.flags & ~(uint32_t)(NF_OVER_CPU | NF_OVER_MEM);
  if (v.r[KOORDHIP_RES_CPU] > v.a[KOORDHIP_RES_CPU]) f |= NF_OVER_CPU;
  if (v.r[KOORDHIP_RES_MEM] > v.a[KOORDHIP_RES_MEM]) f |= NF_OVER_MEM;
  v.flags = f;
}

// filterWithReservations for a matched reservation on the restored values v
// (podRequested = v.r + Allocatable: the matched restore undone).
__device__ __forceinline__ bool resv_filter(const DevPod &p, const NV &v, const NumaRowR &r) {
  const uint32_t pol = KOORDHIP_RESV_POLICY(r.rf);
  if (pol == 0) return true;  // Default: only preemptible resources can make it insufficient
  bool fits = !(v.npods > v.a_pods);  // len(Pods) - len(matched) + 1 > allowed, on the restored NodeInfo
  if (p.flags & KOORDHIP_POD_HAS_REQ) {
#pragma unroll
    for (int k = 0; k < 2; k++)
      fits &= !(p.req[k] > v.a[k] - ((v.r[k] + r.ra[k]) - rem_of(r, k) - r.rd[k]));
    fits &= !(p.req[KOORDHIP_RES_EPH] > v.a[KOORDHIP_RES_EPH] - v.r[KOORDHIP_RES_EPH]);
    if (p.flags & KOORDHIP_POD_REQ_BCPU)
      fits &= !(p.req[KOORDHIP_RES_BCPU] > v.a[KOORDHIP_RES_BCPU] - v.r[KOORDHIP_RES_BCPU]);
    if (p.flags & KOORDHIP_POD_REQ_BMEM)
      fits &= !(p.req[KOORDHIP_RES_BMEM] > v.a[KOORDHIP_RES_BMEM] - v.r[KOORDHIP_RES_BMEM]);
  }
  if (pol == 1) return fits;  // Aligned
  bool le = true;             // Restricted: LessThanOrEqual(podRequests, rRemained)
#pragma unroll
  for (int k = 0; k < 2; k++) le &= !(rkey(r.rf, k) && pkey(p, k) && p.req[k] > rem_of(r, k));
  return le && fits;
}

// FilterReservation of a matched reservation: it is the nominated one
__device__ __forceinline__ bool resv_nominated(const DevPod &p, const NumaRowR &r) {
  bool inter = false, nonzero = false;
#pragma unroll
  for (int k = 0; k < 2; k++) {
    const bool both = rkey(r.rf, k) && pkey(p, k);
    inter |= both;
    nonzero |= both && rem_of(r, k) != 0.0;
  }
  return inter && nonzero;
}

// scoreReservation: MostAllocated (weights 1) over the non-zero Allocatable
__device__ __forceinline__ int32_t resv_score(const DevPod &p, const NumaRowR &r) {
  int32_t s = 0, w = 0;
#pragma unroll
  for (int k = 0; k < 2; k++) {
    const double cap = rkey(r.rf, k) ? r.ra[k] : 0.0;
    const double req = (pkey(p, k) ? p.req[k] : 0.0) + r.rd[k];
    const bool on = cap != 0.0;
    w += on ? 1 : 0;
    s += (on && req <= cap) ? mrs(req, cap) : 0;  // 100 * req / cap, req <= cap
  }
  return w == 2 ? (s >> 1) : s;
}

// Reserve: AddAssignedPod to the nominated reservation (Allocated += the
// pod's requests masked to ResourceNames).
__device__ __forceinline__ void resv_assume(NumaRowR &r, const DevPod &p) {
  if (resv_class(r, p) != 1 || !resv_nominated(p, r)) return;
#pragma unroll
  for (int k = 0; k < 2; k++)
    if (rkey(r.rf, k) && pkey(p, k)) r.rd[k] += p.req[k];
  r.rn += 1;
}

}  // namespace kh
