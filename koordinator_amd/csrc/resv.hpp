// resv.hpp -- the Reservation plugin's per-(pod, node) part on CDNA4: the
// BeforePreFilter restore of the node's reservations (reservation/
// transformer.go:48-293), filterWithReservations (plugin.go:373-494), the
// nomination (FilterReservation plugin.go:504-535, NominateReservation
// nominator.go:32-85), scoreReservation (scoring.go:177-200) and the Reserve
// into the nominated reservation (reservation_info.go:297-306).
//
// A node holds up to S reservations (slots; the reference's map order is
// replaced by the slot order, include/koordhip.h): NumaRowRS<1> for the
// common one-per-node snapshot (NM 3 builds), NumaRowRS<KOORDHIP_RESV_SLOTS>
// otherwise (NM 4).
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

// One reservation of a node (64 B).
struct ResvSlot {
  double ra[2], rd[2], rz[2];  // Allocatable, Allocated, the reserve pod's non-zero request (cpu milli, memory)
  int32_t rn;                  // len(AssignedPods)
  uint32_t rf;                 // KOORDHIP_RESV_* (0: empty slot)
  int32_t rk;                  // order rank
  int32_t rdev;                // (per pod) DeviceShare's FilterReservation passes: the slot can be a device pod's
                               // nomination (set by the caller after load_resv; 0 = not)
};
static_assert(sizeof(ResvSlot) == 64, "reservation slot = 64 B");

// A NUMA side row with the node's reservations (NM >= 3 builds).  The
// several-slot rows (NM 4, which every snapshot with CPU-holding reservations
// runs) keep each slot's reserved CPUs in NumaRow::rcm; the sequential cycle's
// rows (KOORDHIP_RESV_SLOTS_MAX slots) keep those of the slots past
// KOORDHIP_RESV_SLOTS in rcx (rcm_of).
template <int S, bool X = (S > KOORDHIP_RESV_SLOTS)>
struct NumaRowRS;
template <int S>
struct NumaRowRS<S, false> : NumaRow {
  static constexpr int kSlots = S;
  ResvSlot rs[S];
};
template <int S>
struct NumaRowRS<S, true> : NumaRow {
  static constexpr int kSlots = S;
  ResvSlot rs[S];
  uint64_t rcx[S - KOORDHIP_RESV_SLOTS][NW];
};
using NumaRowR = NumaRowRS<1>;
using NumaRowR4 = NumaRowRS<KOORDHIP_RESV_SLOTS>;
using NumaRowR8 = NumaRowRS<KOORDHIP_RESV_SLOTS_MAX>;

// slot q's reserved CPUs (q: an unrolled, compile-time index)
template <int S>
__device__ __forceinline__ uint64_t *rcm_of(NumaRowRS<S> &r, int q) {
  if constexpr (S > KOORDHIP_RESV_SLOTS) {
    return q < KOORDHIP_RESV_SLOTS ? r.rcm[q] : r.rcx[q - KOORDHIP_RESV_SLOTS];
  } else {
    return r.rcm[q];
  }
}
template <int S>
__device__ __forceinline__ const uint64_t *rcm_of(const NumaRowRS<S> &r, int q) {
  if constexpr (S > KOORDHIP_RESV_SLOTS) {
    return q < KOORDHIP_RESV_SLOTS ? r.rcm[q] : r.rcx[q - KOORDHIP_RESV_SLOTS];
  } else {
    return r.rcm[q];
  }
}

constexpr double RESV_NZ_CPU = 100.0;                         // (upstream) DefaultMilliCPURequest
constexpr double RESV_NZ_MEM = 200.0 * 1024.0 * 1024.0;       // (upstream) DefaultMemoryRequest

template <int S>
__device__ __forceinline__ void load_resv(NumaRowRS<S> &r, const DevResv &d, int32_t i) {
#pragma unroll
  for (int q = 0; q < S; q++) {
    ResvSlot &x = r.rs[q];
    const size_t at = (size_t)q * (size_t)d.stride + (size_t)i;
    x.rf = q < d.slots ? d.flags[at] : 0u;
    x.rn = 0;
    x.rk = 0;
    x.rdev = 0;
#pragma unroll
    for (int k = 0; k < 2; k++) x.ra[k] = x.rd[k] = x.rz[k] = 0.0;
    if (x.rf & KOORDHIP_RESV_PRESENT) {
      x.rn = d.rn[at];
      x.rk = d.rank[at];
#pragma unroll
      for (int k = 0; k < 2; k++) {
        x.ra[k] = d.ra[k][at];
        x.rd[k] = d.rd[k][at];
        x.rz[k] = d.rz[k][at];
      }
    }
    if constexpr (S > 1) {
      const bool on = d.rc[0] != nullptr && (x.rf & KOORDHIP_RESV_PRESENT);
#pragma unroll
      for (int w = 0; w < NW; w++) rcm_of(r, q)[w] = on ? d.rc[w][at] : 0ull;
    }
  }
}

template <int S>
__device__ __forceinline__ void store_resv(const NumaRowRS<S> &r, const DevResv &d, int32_t i) {
#pragma unroll
  for (int q = 0; q < S; q++) {
    const ResvSlot &x = r.rs[q];
    if (!(x.rf & KOORDHIP_RESV_PRESENT)) continue;
    const size_t at = (size_t)q * (size_t)d.stride + (size_t)i;
    d.rd[0][at] = x.rd[0];
    d.rd[1][at] = x.rd[1];
    d.rn[at] = x.rn;
    if constexpr (S > 1) {
      if (d.rc[0])
#pragma unroll
        for (int w = 0; w < NW; w++) d.rc[w][at] = rcm_of(r, q)[w];
    }
  }
}
template <int S>
__device__ __forceinline__ void store_resv_wt(const NumaRowRS<S> &r, const DevResv &d, int32_t i) {  // write-through
#pragma unroll
  for (int q = 0; q < S; q++) {
    const ResvSlot &x = r.rs[q];
    if (!(x.rf & KOORDHIP_RESV_PRESENT)) continue;
    const size_t at = (size_t)q * (size_t)d.stride + (size_t)i;
    st_wt(&d.rd[0][at], x.rd[0]);
    st_wt(&d.rd[1][at], x.rd[1]);
    st_wt(&d.rn[at], x.rn);
    if constexpr (S > 1) {
      if (d.rc[0])
#pragma unroll
        for (int w = 0; w < NW; w++) st_wt(&d.rc[w][at], rcm_of(r, q)[w]);
    }
  }
}

__device__ __forceinline__ bool rkey(uint32_t rf, int k) {
  return (rf & (k == 0 ? KOORDHIP_RESV_KEY_CPU : KOORDHIP_RESV_KEY_MEM)) != 0;
}
__device__ __forceinline__ bool pkey(const DevPod &p, int k) {
  return (p.flags & (k == 0 ? KOORDHIP_POD_KEY_CPU : KOORDHIP_POD_KEY_MEM)) != 0;
}
__device__ __forceinline__ double rem_of(const ResvSlot &r, int k) {
  const double x = r.ra[k] - r.rd[k];
  return rkey(r.rf, k) && x > 0.0 ? x : 0.0;  // SubtractWithNonNegativeResult(Allocatable, Allocated)
}

// ABI 14 (the sequential cycle): the node's reservation holding devices
// (slot h) may list NodeResourcesFit extended scalars in its Allocatable.  They
// are more keys of that reservation's ResourceLists, so every rule below sees
// them -- as the facts one out-of-line pass over the scalars (seq.hip
// resv_scalars) derives for the (pod, node):
//   RX_REM    SubtractWithNonNegativeResult(Allocatable, Allocated) has a
//             non-zero scalar (an unmatched reservation's remainder pod comes
//             back even when its cpu / memory remainder is zero, transformer.go:262-276)
//   RX_FIT_H  fitsNode's scalar part with rInfo = h (rRemained = h's remainder)
//   RX_FIT_O  ... with any other matched rInfo (rRemained 0); both with
//             podRequested = the scalars after the unmatched restore and
//             allRAllocated = h's Allocated when h is matched (plugin.go:445-494)
//   RX_LE     Restricted's LessThanOrEqual(podRequests, rRemained) over the scalars (:420-432)
//   RX_INTER  FilterReservation's intersection holds a scalar; RX_NZ: one with a remainder (:504-535)
//   RX_XFIT   NodeResourcesFit over the pod's scalars on the restored Requested
//   xs / xw   scoreReservation's scalar terms: the sum of 100 (request + Allocated) /
//             Allocatable over RemoveZeros(Allocatable)'s scalars and their count (scoring.go:177-200)
// h = -1: no such reservation (every hook is a no-op: the pipelined builds
// never see one -- such snapshots run in the sequential cycle).
enum : uint32_t { RX_REM = 1u, RX_FIT_H = 2u, RX_FIT_O = 4u, RX_LE = 8u, RX_INTER = 16u, RX_NZ = 32u, RX_XFIT = 64u };
struct ResvXS {
  int32_t h;
  uint32_t f;
  int32_t xs, xw;
};
__device__ __forceinline__ ResvXS no_rx() { return ResvXS{-1, 0u, 0, 0}; }

// transformer.go:86-103: 1 = matched, 2 = unmatched with assigned pods, 0 = untouched
__device__ __forceinline__ int resv_class(const ResvSlot &r, const DevPod &p) {
  if (!(r.rf & KOORDHIP_RESV_PRESENT)) return 0;
  if ((r.rf & KOORDHIP_RESV_ALLOCATE_ONCE) && r.rn > 0) return 0;
  const bool match = (p.resv_match >> KOORDHIP_RESV_GROUP(r.rf)) & 1ull;
  if (!(r.rf & KOORDHIP_RESV_UNSCHEDULABLE) && match) return 1;
  return r.rn > 0 ? 2 : 0;
}

// The restore of every reservation of the node on its values
// (restoreMatchedReservation / restoreUnmatchedReservations; the sums do not
// depend on the order), then the Fit over-commit bits of the result.  Returns
// the matched count; mm: the matched slots.
template <int S>
__device__ __forceinline__ int resv_restore(NV &v, const NumaRowRS<S> &r, const DevPod &p, uint32_t &mm,
                                            ResvXS rx = no_rx()) {
  int nmatch = 0;
  bool touched = false;
  mm = 0;
#pragma unroll
  for (int q = 0; q < S; q++) {
    const ResvSlot &x = r.rs[q];
    const int cls = resv_class(x, p);
    if (cls == 0) continue;
    touched = true;
    v.r[KOORDHIP_RES_CPU] -= x.ra[0];
    v.r[KOORDHIP_RES_MEM] -= x.ra[1];
    v.nz_cpu -= x.rz[0];
    v.nz_mem -= x.rz[1];
    if (cls == 1) {
      v.npods -= 1;  // NodeInfo.RemovePod(reservePod)
      nmatch++;
      mm |= 1u << q;
    } else {
      const double rc = rem_of(x, 0), rm = rem_of(x, 1);
      if (rc > 0.0 || rm > 0.0 || (q == rx.h && (rx.f & RX_REM))) {  // a pod requesting the remainder comes back
        v.r[KOORDHIP_RES_CPU] += rc;
        v.r[KOORDHIP_RES_MEM] += rm;
        v.nz_cpu += rkey(x.rf, 0) ? rc : RESV_NZ_CPU;
        v.nz_mem += rkey(x.rf, 1) ? rm : RESV_NZ_MEM;
      }
    }
  }
  if (touched) {
    uint32_t f = v.flags & ~(uint32_t)(NF_OVER_CPU | NF_OVER_MEM);
    if (v.r[KOORDHIP_RES_CPU] > v.a[KOORDHIP_RES_CPU]) f |= NF_OVER_CPU;
    if (v.r[KOORDHIP_RES_MEM] > v.a[KOORDHIP_RES_MEM]) f |= NF_OVER_MEM;
    v.flags = f;
  }
  return nmatch;
}

// filterWithReservations on the restored values v, fitsNode per matched
// reservation (podRequested = v.r + the matched Allocatable: their restore
// undone; rAllocated = the matched Allocated): an Aligned reservation that
// fits, or a Restricted one that fits and holds the pod's requests, passes the
// node; without any the node fails if it has Aligned / Restricted ones
// (Default ones are insufficient only with preemptible resources).
template <int S>
__device__ __forceinline__ bool resv_filter(const DevPod &p, const NV &v, const NumaRowRS<S> &r, uint32_t mm,
                                            int nmatch, ResvXS rx = no_rx()) {
  double podreq[2] = {v.r[KOORDHIP_RES_CPU], v.r[KOORDHIP_RES_MEM]}, rall[2] = {0.0, 0.0};
#pragma unroll
  for (int q = 0; q < S; q++)
    if ((mm >> q) & 1u)
#pragma unroll
      for (int k = 0; k < 2; k++) {
        podreq[k] += r.rs[q].ra[k];
        rall[k] += r.rs[q].rd[k];
      }
  bool pass = false;
  int nar = 0;
#pragma unroll
  for (int q = 0; q < S; q++) {
    if (!((mm >> q) & 1u)) continue;
    const ResvSlot &x = r.rs[q];
    const uint32_t pol = KOORDHIP_RESV_POLICY(x.rf);
    if (pol == 0) continue;
    nar++;
    bool fits = !(v.npods - nmatch + 1 > v.a_pods);  // len(Pods) - len(matched) + 1 > allowed, restored NodeInfo
    if (p.flags & KOORDHIP_POD_HAS_REQ) {
#pragma unroll
      for (int k = 0; k < 2; k++) fits &= !(p.req[k] > v.a[k] - (podreq[k] - rem_of(x, k) - rall[k]));
      fits &= !(p.req[KOORDHIP_RES_EPH] > v.a[KOORDHIP_RES_EPH] - v.r[KOORDHIP_RES_EPH]);
      if (p.flags & KOORDHIP_POD_REQ_BCPU)
        fits &= !(p.req[KOORDHIP_RES_BCPU] > v.a[KOORDHIP_RES_BCPU] - v.r[KOORDHIP_RES_BCPU]);
      if (p.flags & KOORDHIP_POD_REQ_BMEM)
        fits &= !(p.req[KOORDHIP_RES_BMEM] > v.a[KOORDHIP_RES_BMEM] - v.r[KOORDHIP_RES_BMEM]);
      if (rx.h >= 0) fits &= (rx.f & (q == rx.h ? RX_FIT_H : RX_FIT_O)) != 0u;  // the extended scalars
    }
    if (pol == 1) {  // Aligned
      pass |= fits;
    } else {  // Restricted: LessThanOrEqual(podRequests, rRemained)
      bool le = !(q == rx.h && !(rx.f & RX_LE));
#pragma unroll
      for (int k = 0; k < 2; k++) le &= !(rkey(x.rf, k) && pkey(p, k) && p.req[k] > rem_of(x, k));
      pass |= le && fits;
    }
  }
  return pass || nar == 0;
}

// FilterReservation of a matched reservation: a nomination candidate
__device__ __forceinline__ bool resv_candidate(const DevPod &p, const ResvSlot &r, bool xh = false, uint32_t xf = 0u) {
  bool inter = xh && (xf & RX_INTER), nonzero = xh && (xf & RX_NZ);
#pragma unroll
  for (int k = 0; k < 2; k++) {
    const bool both = rkey(r.rf, k) && pkey(p, k);
    inter |= both;
    nonzero |= both && rem_of(r, k) != 0.0;
  }
  return inter && nonzero;
}

// scoreReservation: MostAllocated (weights 1) over the non-zero Allocatable
__device__ __forceinline__ int32_t resv_score(const DevPod &p, const ResvSlot &r, bool xh = false, ResvXS rx = no_rx()) {
  int32_t s = 0, w = 0;
#pragma unroll
  for (int k = 0; k < 2; k++) {
    const double cap = rkey(r.rf, k) ? r.ra[k] : 0.0;
    const double req = (pkey(p, k) ? p.req[k] : 0.0) + r.rd[k];
    const bool on = cap != 0.0;
    w += on ? 1 : 0;
    s += (on && req <= cap) ? mrs(req, cap) : 0;  // 100 * req / cap, req <= cap
  }
  if (xh && rx.xw > 0) return (s + rx.xs) / (w + rx.xw);  // (the extended scalars of RemoveZeros(Allocatable))
  return w == 2 ? (s >> 1) : s;
}

// NominateReservation: among the matched candidates the smallest order label,
// else the highest scoreReservation; ties -> the lowest slot.  -1: none.  A
// device pod under DeviceShare (KH_POD_DEVSHARE) must also pass DeviceShare's
// FilterReservation (deviceshare/plugin.go:325-356): only the node's
// reservation holding devices can (ResvSlot::rdev, set by the caller); a
// reservation holding none has no restore entry and fails it (:337-346).
template <int S>
__device__ __forceinline__ int resv_nominate(const DevPod &p, const NumaRowRS<S> &r, uint32_t mm, ResvXS rx = no_rx()) {
  const bool devshare = (p.flags & KH_POD_DEVSHARE) != 0;
  int best = -1, brk = 0;
  bool ord = false;
  int32_t bsc = -1;
#pragma unroll
  for (int q = 0; q < S; q++) {
    if (!((mm >> q) & 1u) || !resv_candidate(p, r.rs[q], q == rx.h, rx.f)) continue;
    if (devshare && !r.rs[q].rdev) continue;
    const ResvSlot &x = r.rs[q];
    if (x.rf & KOORDHIP_RESV_ORDERED) {
      if (!ord || x.rk < brk) {
        best = q;
        brk = x.rk;
        ord = true;
      }
    } else if (!ord) {
      const int32_t sc = resv_score(p, x, q == rx.h, rx);
      if (sc > bsc) {
        best = q;
        bsc = sc;
      }
    }
  }
  return best;
}

// the matched slots of the pod (their classes only)
template <int S>
__device__ __forceinline__ uint32_t resv_matched(const NumaRowRS<S> &r, const DevPod &p) {
  uint32_t mm = 0;
#pragma unroll
  for (int q = 0; q < S; q++) mm |= (resv_class(r.rs[q], p) == 1 ? 1u : 0u) << q;
  return mm;
}

// PreScore's node order: the smallest order rank among the matched slots, -1 none
template <int S>
__device__ __forceinline__ int resv_node_rank(const NumaRowRS<S> &r, uint32_t mm) {
  int rk = -1;
#pragma unroll
  for (int q = 0; q < S; q++)
    if (((mm >> q) & 1u) && (r.rs[q].rf & KOORDHIP_RESV_ORDERED) && (rk < 0 || r.rs[q].rk < rk)) rk = r.rs[q].rk;
  return rk;
}

// Reserve: AddAssignedPod to the nominated reservation (Allocated += the
// pod's requests masked to ResourceNames); the pod's CPUs leave the slot's
// reserved CPUs (the next cycle's RestoreReservation subtracts the assigned
// pods' cpusets, reservation.go:90-97).
template <int S>
__device__ __forceinline__ int resv_assume(NumaRowRS<S> &r, const DevPod &p, const uint64_t *cpus, ResvXS rx = no_rx()) {
  const int q = resv_nominate(p, r, resv_matched(r, p), rx);
  if (q < 0) return q;
  ResvSlot &x = r.rs[q];
#pragma unroll
  for (int k = 0; k < 2; k++)
    if (rkey(x.rf, k) && pkey(p, k)) x.rd[k] += p.req[k];
  x.rn += 1;
  if constexpr (S > 1) {
#pragma unroll
    for (int w = 0; w < NW; w++) rcm_of(r, q)[w] &= ~cpus[w];
  } else {
    (void)cpus;
  }
  return q;
}

// The reservation-preferred CPUs of a pod on the node (getReservationReservedCPUs,
// nodenumaresource/plugin.go:503-524): the reserved CPUs left in the nominated
// reservation, for a pod AllowUseCPUSet lets restore them (PreRestoreReservation
// :68-74; only cpuset pods -- requestCPUBind -- read them).  Zero: none.
template <int S>
__device__ __forceinline__ void resv_pref_cpus(const NumaRowRS<S> &r, const DevPod &p, uint32_t mm, uint64_t *P,
                                               ResvXS rx = no_rx()) {
#pragma unroll
  for (int w = 0; w < NW; w++) P[w] = 0ull;
  if constexpr (S > 1) {
    if (!(p.flags & KOORDHIP_POD_CPUSET) || (p.flags & KOORDHIP_POD_NUMA_SKIP) || mm == 0u) return;
    const int q = resv_nominate(p, r, mm, rx);
    if (q < 0) return;
#pragma unroll
    for (int w = 0; w < NW; w++) P[w] = rcm_of(r, q)[w];
  } else {
    (void)r;
    (void)p;
    (void)mm;
    (void)rx;
  }
}

// The Reservation Filter of a reserve pod (plugin.go:326-362): its
// reservation's nodeName (reserve_node - 1; 0 = none), and its AllocatePolicy
// against every Available reservation of the node -- Default coexists only
// with Default.
template <int S>
__device__ __forceinline__ bool reserve_pod_ok(const DevPod &p, int32_t reserve_node, const NumaRowRS<S> &r,
                                               int32_t i) {
  if (reserve_node > 0 && i != reserve_node - 1) return false;
  const uint32_t pol = KOORDHIP_POD_RESERVE_POLICY(p.flags);
  bool ok = true;
#pragma unroll
  for (int q = 0; q < S; q++) {
    const uint32_t rf = r.rs[q].rf;
    const uint32_t rp = KOORDHIP_RESV_POLICY(rf);
    ok &= !((rf & KOORDHIP_RESV_PRESENT) && (pol == 0u || rp == 0u) && pol != rp);
  }
  return ok;
}

// a slot of the node holds an Available reservation whose owner group `p` matches
template <int S>
__device__ __forceinline__ bool resv_matchable(const NumaRowRS<S> &r, const DevPod &p) {
  bool m = false;
#pragma unroll
  for (int q = 0; q < S; q++)
    m |= (r.rs[q].rf & KOORDHIP_RESV_PRESENT) && ((p.resv_match >> KOORDHIP_RESV_GROUP(r.rs[q].rf)) & 1ull);
  return m;
}

}  // namespace kh
