// seq.hip -- the exact sequential cycle (koordhip_place_stream_ext) for
// profiles whose Scores are normalized over the pod's feasible nodes
// (DeviceShare, NodeAffinity / TaintToleration Score: DefaultNormalizeScore,
// upstream helper/normalize_score.go; deviceshare/scoring.go:78-80).  The
// normalization couples every node of a pod -- the maximum over the feasible
// set moves when any node's feasibility or raw score does -- so the pipelined
// top-k + resolve of kernels.hip, whose keys are per node, does not apply.
// Instead ONE persistent launch over every CU runs the reference cycle pod by
// pod on the state all earlier commits left:
//
//   phase A  every block evaluates its node slices (Filter of every plugin,
//            the weighted sum of the per-node plugins, the raw normalized
//            scores) into LDS; per block: feasible count, the raw maxima over
//            its feasible nodes and its best (total, lowest index) key as if
//            every maximum were 0, published as tagged granules (the data is
//            the flag: cdna_hip_programming.md Guideline 16 R2, no barrier)
//   phase B  only when some maximum is not 0 (a pod requesting devices, or
//            with preferred terms / intolerable soft taints somewhere): every
//            block normalizes its nodes' raw scores by the global maxima and
//            publishes its best key the same way.  With all maxima 0 every
//            normalized score is the same constant, so phase A's keys already
//            rank the nodes: one hand-off per pod instead of two.
//   commit   every block reads all keys: the winner w; the block owning w
//            runs the Reserve of every plugin on w (DeviceShare's device
//            choice, NodeNUMAResource's cpuset, Reservation's assume, the
//            Fit / LoadAware delta) before it evaluates its nodes for the
//            next pod.  Node w is only ever read by its owner block, so no
//            other block waits for the commit.
//
// Granule ring: 2 parities x G blocks x SEQ_GRAN words; a block overwrites parity
// q's granules only after it has read every block's granules of the next
// phase, which every block writes after it finished reading parity q.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "dev.hpp"
#include "ipa.hpp"
#include "pipe.hpp"
#include "pts.hpp"
#include "seq.h"

namespace kh {

constexpr int SEQ_THREADS = 256;
constexpr int SEQ_NPT = 8;  // nodes per thread held across the pod's phases (grid 256 x 256 x 8 >= 400k nodes)
constexpr uint32_t SEQ_SPIN_LIMIT = 1u << 24;

struct SeqArgs {
  const DevPod *pods;
  const DevPodX *podx;  // NULL: no pod has a device / extended request
  int32_t n_pods;
  int32_t npt;          // node slices per thread
  uint64_t *ga, *gb;    // granules [2][G][SEQ_GRAN]
  uint32_t *tmo;        // spin timeout word (0 = ok)
  int32_t *out_node;
  uint64_t *out_cpus;   // [n_pods][NW] (NULL: no NodeNUMAResource)
  uint32_t *out_dev;    // [n_pods][DT] (NULL: no DeviceShare)
  uint32_t ext;         // bit e: normalized plugin e scores (DeviceShare, NodeAffinity, TaintToleration)
  int32_t rs;           // the Reservation plugin scores (its PreScore nominates)
  uint64_t *dbg;        // KOORDHIP_STAMPS: block 0's per-phase cycle sums [0..4], owner commits [5] (NULL: off)
  const DevCfg *gc;     // global copies of the kernel's config and column descriptors (the commit's)
  const DevNodes *gd;
  // PodTopologySpread: the columns and the per-pod phases' granules: g0 the
  // hostname minimum, gp the raw Score's min / max, gr the commit result
  PtsArgs pts;
  uint64_t *g0, *gp, *gr;
  IpaArgs ipa;  // InterPodAffinity: the count entries (ents 0: off)
};

__device__ __forceinline__ uint64_t seq_stamp() {
  uint64_t v;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory");
  return v;
}

__device__ __forceinline__ uint64_t seq_wave_max(uint64_t v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    const uint64_t o = __shfl_xor(v, m);
    v = o > v ? o : v;
  }
  return v;
}

__device__ __forceinline__ uint32_t ext_bits(const DevCfg &c) {
  return ((c.score & KOORDHIP_PLUGIN_DEVICESHARE) ? 1u : 0u) | ((c.score & KOORDHIP_PLUGIN_AFFINITY_SCORE) ? 2u : 0u) |
         ((c.score & KOORDHIP_PLUGIN_TAINT_SCORE) ? 4u : 0u);
}

// SM: the compiled side-row mode -- 0 none (Fit / LoadAware / static /
// balanced), 1 + NodeNUMAResource (with the zone code), 2 + Reservation (the
// 4-slot rows, with NUMA when enabled), 3 the same with the 8-slot rows
// (more than KOORDHIP_RESV_SLOTS reservations on a node).  The plain build
// keeps no side row at all: a zero-initialised ~0.5 KB row per lane would live
// in scratch.
__host__ __device__ constexpr int seq_mode(const DevCfg &c) {
  return c.resv ? (c.resv_slots > KOORDHIP_RESV_SLOTS ? 3 : 2) : (((c.filt | c.score) & KOORDHIP_PLUGIN_NUMA) ? 1 : 0);
}
template <int SM>
using SeqResvRow = NumaRowRS<SM == 3 ? KOORDHIP_RESV_SLOTS_MAX : KOORDHIP_RESV_SLOTS>;

// The node's reservation holding devices, for a device pod under DeviceShare
// (KH_POD_DEVSHARE): its DevRC (dev.hpp; h -1: none) and DeviceShare's
// FilterReservation of it, recorded in its slot's rdev -- the nomination's only
// possible candidate for the pod (resv_nominate).
template <int S>
__device__ __forceinline__ DevRC seq_dev_resv(const DevCfg &c, const DevDev &dv, const DevPod &p, const DevPodX &x,
                                              NumaRowRS<S> &r, int32_t i) {
  DevRC rc{-1, 0, 0, 0u};
  if (!dv.rslot || !c.resv || !(p.flags & KH_POD_DEVSHARE)) return rc;
  const int32_t h = dv.rslot[i];
  if (h < 0 || h >= S) return rc;
  int32_t cls = 0;
  uint32_t rf = 0u;
#pragma unroll
  for (int q = 0; q < S; q++)
    if (q == h) {
      cls = resv_class(r.rs[q], p);
      rf = r.rs[q].rf;
    }
  rc = rc_of(c, dv, i, h, cls, rf);
  if (rc.h >= 0 && rc.cls == 1 && rc_filter_reservation(c, dv, x, i, rc))
#pragma unroll
    for (int q = 0; q < S; q++)
      if (q == h) r.rs[q].rdev = 1;
  return rc;
}

// ABI 14: resv.hpp's ResvXS for pod (p, x) on node i, whose reservation
// holding devices is slot h with restore class `cls` (1 matched, 2 unmatched
// with assigned pods, 0 neither), from its extended scalars (Allocatable A,
// Allocated D, remainder max0(A - D); a listed key has A > 0) and the node's
// scalar Allocatable / Requested.  Rare (a node whose reservation lists
// extended scalars), so out of line: the common path keeps its registers.
__device__ __noinline__ ResvXS resv_scalars(const DevDev &dv, const DevPodX &x, int32_t i, int32_t n, int32_t h,
                                            int cls) {
  ResvXS rx{h, RX_FIT_H | RX_FIT_O | RX_LE | RX_XFIT, 0, 0};
  for (int j = 0; j < KOORDHIP_NXRES; j++) {
    const size_t at = (size_t)j * n + i;
    const int64_t A = dv.rxa[at], D = dv.rxd[at];
    const int64_t rem = A - D > 0 ? A - D : 0;
    const bool key = (x.xmask >> j) & 1u;
    const int64_t px = key ? x.xreq[j] : 0;
    if (rem > 0) rx.f |= RX_REM;
    if (A != 0) {  // RemoveZeros(Allocatable) / ResourceNames
      rx.xw++;
      const int64_t req = px + D;  // scoreReservation: PodRequestsAndLimits + Allocated
      if (req <= A) rx.xs += (int32_t)(100 * req / A);
      if (key) {
        rx.f |= RX_INTER | (rem > 0 ? RX_NZ : 0u);
        if (px > rem) rx.f &= ~RX_LE;
      }
    }
    if (!key) continue;
    const int64_t alloc = dv.xalloc ? dv.xalloc[at] : 0, xr = dv.xreq[at];
    // NodeResourcesFit on the restored NodeInfo: the reserve pod leaves, an
    // unmatched reservation's remainder comes back (transformer.go:227-293)
    if (px > alloc - (xr - (cls != 0 ? A : 0) + (cls == 2 ? rem : 0))) rx.f &= ~RX_XFIT;
    // fitsNode: podRequested after the unmatched restore, allRAllocated = D when matched
    const int64_t preq = xr + (cls == 2 ? rem - A : 0), rall = cls == 1 ? D : 0;
    if (px > alloc - (preq - rem - rall)) rx.f &= ~RX_FIT_H;
    if (px > alloc - (preq - rall)) rx.f &= ~RX_FIT_O;
  }
  return rx;
}

// the ResvXS of node i's reservation holding devices for the pod (h -1: none)
template <int S>
__device__ __forceinline__ ResvXS seq_resv_x(const DevNodes &d, const DevPod &p, const DevPodX &x,
                                             const NumaRowRS<S> &r, int32_t i) {
  if (!d.dv.rxa) return no_rx();
  const int32_t h = d.dv.rslot[i];
  if (h < 0 || h >= S) return no_rx();
  int cls = 0;
#pragma unroll
  for (int q = 0; q < S; q++)
    if (q == h) cls = resv_class(r.rs[q], p);
  return resv_scalars(d.dv, x, i, d.n, h, cls);
}

// One node for one pod: the total of the per-node plugins (-1: some Filter
// fails; with the Reservation plugin the ranking total of resv.hpp) and the
// raw normalized scores.  Every column is read (the parity evaluator's rows,
// like k_eval_full).  Inlined once per kernel: a call keeps its frame (the
// config and column descriptors, the NV row) in scratch, kilobytes per lane.
// EARLY (k_ext_worker: no status, no raw planes of infeasible nodes): a node
// whose extended scalars do not fit returns -1 before any other load.
template <int SM, bool EARLY = false>
__device__ __forceinline__ int32_t seq_eval(const DevCfg &c, const DevNodes &d, const DevPod &p, const DevPodX &x,
                                            int32_t i, bool rs, int32_t raw[KOORDHIP_NEXT_PLUGINS],
                                            uint8_t *status) {
  if constexpr (EARLY)
    if ((c.filt & KOORDHIP_PLUGIN_FIT) && !xfit_filter(d.dv, x, i, d.n)) return -1;
  NV v{};
  const Need all = need_all(c);
  load_node(v, d, i, all, c);
  // the reads that do not depend on the node row next, so their round trips
  // overlap the row's: the extended scalars, the static Scores and (without
  // the Reservation build, whose nomination needs the reservation rows) the
  // device rows
  bool xfr = EARLY || !(c.filt & KOORDHIP_PLUGIN_FIT) || xfit_filter(d.dv, x, i, d.n);
  raw[1] = (c.score & KOORDHIP_PLUGIN_AFFINITY_SCORE) ? static_raw(d.dv, 0, p.sclass, i, d.n) : 0;
  raw[2] = (c.score & KOORDHIP_PLUGIN_TAINT_SCORE) ? static_raw(d.dv, 1, p.sclass, i, d.n) : 0;
  int32_t t;
  bool df = true, rfail = false;
  if constexpr (SM >= 2) {
    constexpr int S = SM == 3 ? KOORDHIP_RESV_SLOTS_MAX : KOORDHIP_RESV_SLOTS;
    SeqResvRow<SM> nr{};
    load_numa<false>(nr, d, i, all);  // (the zone row shares the reserved CPUs' bytes: eval_total_resv<.., Z> reads it)
    load_resv(nr, d.rv, i);
    const DevRC rc = seq_dev_resv(c, d.dv, p, x, nr, i);
    const ResvXS rx = seq_resv_x(d, p, x, nr, i);
    if (rx.h >= 0 && (c.filt & KOORDHIP_PLUGIN_FIT)) xfr = (rx.f & RX_XFIT) != 0u;  // on the restored scalars
    t = c.zones       ? eval_total_resv<S, true, true>(p, v, nr, d.nu.cls, c, &d, i, rx)
        : c.resv_cpus ? eval_total_resv<S, true>(p, v, nr, d.nu.cls, c, nullptr, 0, rx)
                      : eval_total_resv<S, false>(p, v, nr, d.nu.cls, c, nullptr, 0, rx);
    const int32_t nq = (rs && (x.flags & KOORDHIP_PODX_DEVICE)) ? resv_nominate(p, nr, resv_matched(nr, p), rx) : -1;
    if (rc.h >= 0)
      df = rc_eval(c, d.dv, x, i, rc, nq, (c.filt & KOORDHIP_PLUGIN_DEVICESHARE) != 0,
                   (c.score & KOORDHIP_PLUGIN_DEVICESHARE) != 0, &raw[0]);
    else
      df = dev_eval(c, d.dv, x, i, nq >= 0, (c.filt & KOORDHIP_PLUGIN_DEVICESHARE) != 0,
                    (c.score & KOORDHIP_PLUGIN_DEVICESHARE) != 0, &raw[0]);
    if ((p.flags & (KOORDHIP_POD_RESERVE | KOORDHIP_POD_RESV_OPERATING)) && (c.filt & KOORDHIP_PLUGIN_RESERVATION) &&
        !reserve_pod_ok(p, (p.flags & KOORDHIP_POD_RESERVE) ? x.reserve_node : 0, nr, i))
      rfail = true;
  } else {
    df = dev_eval(c, d.dv, x, i, false, (c.filt & KOORDHIP_PLUGIN_DEVICESHARE) != 0,
                  (c.score & KOORDHIP_PLUGIN_DEVICESHARE) != 0, &raw[0]);
    if constexpr (SM == 1) {
      NumaRow nr{};
      load_numa<true>(nr, d, i, all);
      t = eval_total_numa<true>(p, v, nr, d.nu.cls, c);
    } else {
      t = eval_total(p, v, c);
    }
  }
  const bool xf = xfr;
  if (status)
    *status = (xf ? 0 : KOORDHIP_ST_XFIT_FAIL) | (df ? 0 : KOORDHIP_ST_DEVICE_FAIL) | (rfail ? KOORDHIP_ST_RESV_FAIL : 0);
  if (!xf || !df || rfail) t = -1;
  raw[3] = 0;  // PodTopologySpread: its own phases (pts.hpp)
  raw[4] = 0;  // InterPodAffinity: ipa.hpp
  return t;
}

// DefaultNormalizeScore(MaxNodeScore, reverse) of one raw score given the
// maximum over the feasible nodes
__device__ __forceinline__ int32_t norm_score(int32_t raw, int32_t mx, bool reverse) {
  if (mx == 0) return reverse ? 100 : raw;
  const int32_t s = (int32_t)((int64_t)100 * raw / mx);
  return reverse ? 100 - s : s;
}

// the max-normalized plugins (DeviceShare, NodeAffinity, TaintToleration reversed)
__device__ __forceinline__ int32_t ext_total(const DevCfg &c, uint32_t ext, const int32_t raw[KOORDHIP_NEXT_PLUGINS],
                                             const int32_t mx[KOORDHIP_NEXT_PLUGINS]) {
  int32_t t = 0;
#pragma unroll
  for (int e = 0; e < 3; e++)
    if ((ext >> e) & 1u) t += c.w_ext[e] * norm_score(raw[e], mx[e], e == 2);
  return t;
}

// tk plus the normalized plugins' `extra`, except in the Reservation ranking
// total's preferred tier (a node whose matched reservations carry an order
// label, resv.hpp): the reference's preferred node takes the normalized
// Reservation score 100 x its weight and wins outright, the tier ranks by the
// order alone -- extra added there would reorder two ordered nodes
// (orc_resv_rank_total ignores it the same way)
__device__ __forceinline__ int32_t rank_add(const DevCfg &c, int32_t tk, int32_t extra) {
  return (c.resv && (c.score & KOORDHIP_PLUGIN_RESERVATION) && tk >= 101 * c.resv_b1) ? tk : tk + extra;
}

// The record of a pod without koordhip_pod_ext (no device request: gpu -1 =
// key absent).  Pods read their record in place (global, wave-uniform: scalar
// loads) -- a register copy of the 328-B record spills.
__device__ const DevPodX kNoPodX = {{{-1, -1, -1}, {0, 0, 0}, {0, 0, 0}}};

// R2 granules: {epoch, value}; one aligned 8-byte write-through store
__device__ __forceinline__ void put_granule(uint64_t *g, uint32_t epoch, uint32_t v) {
  __hip_atomic_store(g, ((uint64_t)epoch << 32) | v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// thread t < G waits for block t's NW granules of `epoch`; false on timeout
template <int NG>
__device__ __forceinline__ bool sweep(const uint64_t *g, uint32_t epoch, uint32_t (&v)[NG], uint32_t *tmo) {
  for (uint32_t spins = 0;; spins++) {
    bool ok = true;
#pragma unroll
    for (int k = 0; k < NG; k++) {
      const uint64_t x = __hip_atomic_load(const_cast<uint64_t *>(g) + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      v[k] = (uint32_t)x;
      ok &= (uint32_t)(x >> 32) == epoch;
    }
    if (ok) return true;
    if (spins > SEQ_SPIN_LIMIT || __hip_atomic_load(tmo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
      __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// The Reserve of every plugin on node w (k_commit's order and rules, plus
// DeviceShare and the extended scalars); rc: 0, or KOORDHIP_RESERVE_FAILED
// (nothing committed).  nf: the feasible node count (one: no PreScore, so no
// reservation is nominated before the NodeNUMAResource / DeviceShare Reserve).
// ROW false (k_ext_worker): the Fit / LoadAware row is the pipelined
// resolve's, which applies that delta itself -- everything else here.
template <int SM, bool ROW = true>
__device__ __forceinline__ int32_t seq_commit_body(const DevCfg &c, const DevNodes &d, const DevPod &p,
                                                   const DevPodX &x, int32_t w, int32_t nf, bool rs,
                                                   uint64_t *cpus_out, uint32_t *dev_out) {
  using RV = typename std::conditional<SM >= 2, SeqResvRow<SM>, NumaRow>::type;
  RV rv;
  uint32_t mm = 0u;
  DevRC rc{-1, 0, 0, 0u};
  ResvXS rx = no_rx();
  if constexpr (SM >= 2) {
    load_resv(rv, d.rv, w);
    mm = resv_matched(rv, p);
    rc = seq_dev_resv(c, d.dv, p, x, rv, w);
    rx = seq_resv_x(d, p, x, rv, w);
  }
  const bool prescore = rs && nf > 1;
  // the reservation PreScore nominated (DeviceShare Reserve reads it) and the
  // one the Reservation Reserve assumes the pod into, both on the state
  // before any Reserve
  int32_t nq = -1, qa = -1;
  if constexpr (SM >= 2) {
    qa = resv_nominate(p, rv, mm, rx);
    nq = prescore ? qa : -1;
  }
  uint32_t slots[DT] = {0u, 0u, 0u};
  int64_t per[DT][DR];
  const bool dev = ((c.filt | c.score) & KOORDHIP_PLUGIN_DEVICESHARE) != 0;
  // the loads of every row the Reserve changes go out first (one round trip
  // with the device rows' instead of one per structure): the Fit / LoadAware
  // row and the extended scalars' Requested
  NV v;
  if constexpr (ROW) load_row(v, d, w);
  int64_t xr[KOORDHIP_NXRES];
#pragma unroll
  for (int j = 0; j < KOORDHIP_NXRES; j++) xr[j] = ((x.xmask >> j) & 1u) ? d.dv.xreq[(size_t)j * d.n + w] : 0;
  if (dev && !(rc.h >= 0 ? rc_reserve(c, d.dv, x, w, rc, nq, slots, per) : dev_reserve(c, d.dv, x, w, nq >= 0, slots, per)))
    return KOORDHIP_RESERVE_FAILED;
  uint64_t m[NW] = {0, 0, 0, 0};
  if constexpr (SM >= 1) {
    if (numa_on(c) && numa_active(p, c)) {
      NumaRow r;
      load_numa_row(r, d, w);
      uint64_t pref[NW] = {0, 0, 0, 0};
      if constexpr (SM >= 2) resv_pref_cpus(rv, p, prescore ? mm : 0u, pref, rx);
      if (!numa_reserve<true>(d.nu.cls, r, p, m, pref)) return KOORDHIP_RESERVE_FAILED;
      store_numa_row(r, d, w);
    }
  }
  if (dev) {
    dev_apply<!ROW>(d.dv, w, slots, per);
    if (rc.h >= 0 && qa == rc.h) rc_apply_allocated<!ROW>(d.dv, w, slots, per);
  }
  if constexpr (SM >= 2) {  // Reservation Reserve: assumePod into the nominated reservation
    const int qz = resv_assume(rv, p, m, rx);
    store_resv(rv, d.rv, w);
    if (qz >= 0 && qz == rx.h && x.xmask)  // ... its extended scalars' Allocated (masked to its keys)
      for (int j = 0; j < KOORDHIP_NXRES; j++) {
        const size_t at = (size_t)j * d.n + w;
        if (((x.xmask >> j) & 1u) && d.dv.rxa[at] != 0) d.dv.rxd[at] += x.xreq[j];
      }
  }
  if constexpr (ROW) {
    apply_delta(v, p, +1);
    store_row(v, d, w);
  }
  if (x.xmask)
#pragma unroll
    for (int j = 0; j < KOORDHIP_NXRES; j++)
      if ((x.xmask >> j) & 1u) {
        if constexpr (ROW)
          d.dv.xreq[(size_t)j * d.n + w] = xr[j] + x.xreq[j];
        else
          st_wt(&d.dv.xreq[(size_t)j * d.n + w], (int64_t)(xr[j] + x.xreq[j]));
      }
  if (cpus_out)
    for (int q = 0; q < NW; q++) cpus_out[q] = m[q];
  if (dev_out)
    for (int t = 0; t < DT; t++) dev_out[t] = slots[t];
  return 0;
}

// The owner's commit of pod p (out_node / out_cpus / out_dev written here).
// Not inlined: one lane per pod runs it, and inlined its Reserve code (the
// device choice, the cpuset replay) would push the per-pod loop out of the
// instruction cache.  The config, the column descriptors and the pod come
// through global pointers (reference arguments to kernel parameters make the
// caller copy them into scratch).
template <int SM>
__device__ __noinline__ void seq_commit(const DevCfg *cp, const DevNodes *dp, const DevPod *pp, const DevPodX *px,
                                        int32_t w, int32_t nf, bool rs, int32_t *out_node, uint64_t *out_cpus,
                                        uint32_t *out_dev) {
  const DevPodX &x = px ? *px : kNoPodX;
  uint64_t cpus[NW] = {0, 0, 0, 0};
  uint32_t dv[DT] = {0u, 0u, 0u};
  int32_t res = KOORDHIP_UNSCHEDULABLE;
  if (w >= 0) {
    const int32_t rc = seq_commit_body<SM>(*cp, *dp, *pp, x, w, nf, rs, cpus, dv);
    res = rc ? KOORDHIP_RESERVE_FAILED : w;
    if (rc) {
      for (int q = 0; q < NW; q++) cpus[q] = 0;
      for (int q = 0; q < DT; q++) dv[q] = 0u;
    }
  }
  *out_node = res;
  if (out_cpus)
    for (int q = 0; q < NW; q++) out_cpus[q] = cpus[q];
  if (out_dev)
    for (int q = 0; q < DT; q++) out_dev[q] = dv[q];
}

// Reserve (sign > 0) / Unreserve (sign < 0) of ONE pod with its
// koordhip_pod_ext record on node w, from the host (koordhip_commit_ext /
// koordhip_uncommit_ext): what the Go shim calls after it chose a node itself,
// or when Permit / PreBind fails after Reserve.  Reserve is the sequential
// cycle's commit (seq_commit_body: DeviceShare's device choice and deviceUsed,
// plugin.go:368-405; NodeNUMAResource's cpuset; Reservation's assume; the Fit /
// LoadAware delta; the extended scalars), with PreScore assumed to have run
// (nf > 1), plus the PodTopologySpread / InterPodAffinity counts the placed pod
// adds (upstream AddPod).  Unreserve undoes each of them from what Reserve
// returned: the device slots (deviceshare plugin.go:407-426 -> allocator
// Unreserve: each slot's per-device request, recomputed from the node's GPU
// memory as Reserve computed it), the cpuset, the counts (RemovePod).  rc: 0,
// KOORDHIP_ERESERVE (Reserve failed, nothing applied) or KOORDHIP_EINVAL
// (an Unreserve the returned values cannot undo: see k_commit).
template <int SM>
__global__ void k_commit_ext(DevCfg c, DevNodes d, const DevPod *__restrict__ pod, const DevPodX *__restrict__ px,
                             int32_t w, int32_t sign, int32_t rs, uint64_t *__restrict__ cpus, uint32_t *__restrict__ dev,
                             int32_t *__restrict__ rc, PtsArgs pa, IpaArgs ia) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const DevPod p = *pod;
  const DevPodX &x = *px;
  *rc = 0;
  const uint32_t pm = pa.cnt ? (uint32_t)x.pts_match : 0u;
  const uint32_t im = ia.cnt ? x.ipa_inc : 0u;
  if (sign > 0) {
    const int32_t r = seq_commit_body<SM>(c, d, p, x, w, 2, rs != 0, cpus, dev);
    if (r) {
      *rc = KOORDHIP_ERESERVE;
      return;
    }
    for (int cc = 0; cc < pa.cons; cc++)
      if ((pm >> cc) & 1u) pa.cnt[(size_t)cc * d.n + w] += 1;
    ipa_commit_cols(ia, im, d.n, w);
    return;
  }
  // ---- Unreserve: refuse what the returned values cannot undo (k_commit's rules)
  if constexpr (SM >= 2) {
    SeqResvRow<SM> rv;
    load_resv(rv, d.rv, w);
    if (c.resv && resv_matchable(rv, p)) {
      *rc = KOORDHIP_EINVAL;
      return;
    }
  }
  if constexpr (SM >= 1) {
    if (numa_on(c) && numa_active(p, c)) {
      NumaRow r;
      load_numa_row(r, d, w);
      if (topo_policy(r.nflags) != 0) {
        *rc = KOORDHIP_EINVAL;
        return;
      }
      if (is_cpuset(p)) {
        uint64_t m[NW];
        for (int q = 0; q < NW; q++) m[q] = cpus[q];
        numa_apply(r, p, m, -1);
        store_numa_row(r, d, w);
      }
    }
  }
  if (((c.filt | c.score) & KOORDHIP_PLUGIN_DEVICESHARE) && (x.flags & KOORDHIP_PODX_DEVICE) && d.dv.slots > 0) {
    for (int t = 0; t < DT; t++) {
      int64_t q[DR], per[DR];
      if (!dev[t] || !dev_requests(x, t, q)) continue;
      DevRow dr;
      dev_load(d.dv, w, t, dr);
      if (t == KOORDHIP_DEV_GPU && !dev_fill_gpu(dr, q)) continue;
      (void)dev_wanted(t, q, per);
      const size_t a0 = dev_at(d.dv, w, t, 0) * DR;
      for (int s = 0; s < d.dv.slots; s++)
        if ((dev[t] >> s) & 1u)
          for (int r = 0; r < DR; r++) d.dv.used[a0 + (size_t)s * DR + r] -= per[r];
    }
  }
  if (x.xmask)
    for (int j = 0; j < KOORDHIP_NXRES; j++)
      if ((x.xmask >> j) & 1u) d.dv.xreq[(size_t)j * d.n + w] -= x.xreq[j];
  NV v;
  load_row(v, d, w);
  apply_delta(v, p, -1);
  store_row(v, d, w);
  for (int cc = 0; cc < pa.cons; cc++)
    if ((pm >> cc) & 1u) pa.cnt[(size_t)cc * d.n + w] -= 1;
  for (uint32_t inc = im; inc;) {
    const int e = ipa_next(inc);
    ia.cnt[(size_t)e * d.n + w] -= 1;
  }
}

hipError_t launch_commit_ext(const DevCfg &c, const DevNodes &d, const DevPod *pod, const DevPodX *px, int32_t node,
                             int32_t sign, int32_t rs, uint64_t *cpus, uint32_t *dev, int32_t *rc, const PtsArgs &pts,
                             const IpaArgs &ipa, hipStream_t s) {
  switch (seq_mode(c)) {
    case 3: hipLaunchKernelGGL(k_commit_ext<3>, dim3(1), dim3(64), 0, s, c, d, pod, px, node, sign, rs, cpus, dev, rc, pts, ipa); break;
    case 2: hipLaunchKernelGGL(k_commit_ext<2>, dim3(1), dim3(64), 0, s, c, d, pod, px, node, sign, rs, cpus, dev, rc, pts, ipa); break;
    case 1: hipLaunchKernelGGL(k_commit_ext<1>, dim3(1), dim3(64), 0, s, c, d, pod, px, node, sign, rs, cpus, dev, rc, pts, ipa); break;
    default: hipLaunchKernelGGL(k_commit_ext<0>, dim3(1), dim3(64), 0, s, c, d, pod, px, node, sign, rs, cpus, dev, rc, pts, ipa);
  }
  return hipGetLastError();
}

// Block-wide reduction of (sum, max, max, max) and a u64 max over the block's
// threads; every thread gets the result.
__device__ __forceinline__ void seq_block_reduce(int32_t v4[4], uint64_t &key, int32_t (*s_red)[8], uint64_t *s_key,
                                                 int t) {
  const int lane = t & 63, wv = t >> 6;
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    v4[0] += __shfl_xor(v4[0], m);
#pragma unroll
    for (int e = 1; e < 4; e++) v4[e] = max(v4[e], __shfl_xor(v4[e], m));
  }
  key = seq_wave_max(key);
  __syncthreads();  // the previous use of s_red / s_key is finished
  if (lane == 0) {
#pragma unroll
    for (int e = 0; e < 4; e++) s_red[wv][e] = v4[e];
    s_key[wv] = key;
  }
  __syncthreads();
  v4[0] = 0;
  v4[1] = v4[2] = v4[3] = 0;
  key = 0;
#pragma unroll
  for (int w = 0; w < SEQ_THREADS / 64; w++) {
    v4[0] += s_red[w][0];
#pragma unroll
    for (int e = 1; e < 4; e++) v4[e] = max(v4[e], s_red[w][e]);
    key = s_key[w] > key ? s_key[w] : key;
  }
}

// ---- device pods inside the pipelined greedy (koordhip_place_staged, a
// DeviceShare profile whose staged batch holds a few device pods among pods
// without ext content).  The pipelined resolve places every other pod; at a
// device pod (KH_POD_EXT) it writes every commit so far back, exports its X
// set (the nodes committed since the state the round's lists were evaluated
// on: M' and this round's M, pipe_xlist) and stores sync->ext_req = pod + 1.
// This persistent grid runs that pod's reference cycle: every node's Filter
// and per-node total, DeviceShare's raw Score (0 .. 100 per requested type,
// scoring.go:33-72) and the normalization over the feasible nodes
// (DefaultNormalizeScore, scoring.go:78-80).
//   pre-evaluation, off the critical path: as soon as the pod's round u may
//     be evaluated (res_round >= u - lag, and the device commits of the device
//     pods of the rounds before that are published), every node's key
//     make_key(total, i) (0: infeasible) and raw score into pk / pr;
//   final, at the hand-off: only the X nodes are evaluated again (every other
//     node's row is the pre-evaluation's); the normalized total of a node is
//     its total + w * norm(raw), so the winner is among the best (total,
//     lowest index) node of each raw value: every workgroup folds its chunk
//     into a [EXT_RAW] table of such keys in LDS and merges it into the global
//     one with agent-scope atomic max; the workgroup finishing the last chunk
//     takes the maximum raw value, ranks the <= EXT_RAW candidates, stores
//     out_node write-through and ext_done = pod + 1, and only then runs
//     DeviceShare's Reserve (device choice + deviceUsed, the extended scalars;
//     not the Fit / LoadAware row, which the resolve commits in its own copy)
//     and publishes it (cdone) for the next device pod.
// Node chunks are claimed from per-pod counters, not assigned: whichever
// workgroups are resident share the work (none waits for a workgroup the GPU
// has not started -- its CUs may be held by persistent kernels that wait on
// this pod).
constexpr int EXT_RAW = 320;  // raw DeviceShare scores 0 .. 300 (three device types x 100)
constexpr int EXT_THREADS = 256;
constexpr int32_t EXT_PCHUNK = EXT_THREADS;      // pre-evaluation chunk: one node per thread
constexpr int EXT_FNPT = 4;                      // final chunk: four nodes per thread (two loads each)
constexpr int32_t EXT_FCHUNK = EXT_THREADS * EXT_FNPT;
constexpr int EXT_CW = 8;     // counter words per device pod: claimed / finished chunks of both phases
constexpr int EXT_RING = 4;   // pre-evaluation buffers: device pods evaluated ahead of their hand-off

// Workgroups [0, gf) run the final phases, [gf, grid) the pre-evaluations,
// which run up to EXT_RING device pods ahead.
template <int SM>
__global__ __launch_bounds__(EXT_THREADS) void k_ext_worker(DevCfg c, DevNodes d, const DevPod *__restrict__ pods,
                                                            const DevPodX *__restrict__ podx,
                                                            const int32_t *__restrict__ ext_idx,
                                                            const int32_t *__restrict__ needc, int32_t n_ext, int32_t P,
                                                            int32_t lag, int32_t lead, int32_t gf,
                                                            uint64_t *__restrict__ tab,
                                                            uint32_t *__restrict__ cnt, uint64_t *__restrict__ pk,
                                                            int32_t *__restrict__ pr, const int32_t *__restrict__ perm,
                                                            int32_t *__restrict__ out_node,
                                                            uint32_t *__restrict__ out_dev, PipeSync *sy, uint64_t *dbg) {
  __shared__ uint64_t lt[EXT_RAW];
  __shared__ uint32_t xm[EXT_FCHUNK / 32];  // the chunk's X nodes
  __shared__ int32_t s_red[SEQ_THREADS / 64][8];
  __shared__ uint64_t s_key[SEQ_THREADS / 64];
  __shared__ int32_t s_go, s_last, s_ch;
  const int t = threadIdx.x;
  const int32_t b = blockIdx.x;
  const int32_t ncp = (d.n + EXT_PCHUNK - 1) / EXT_PCHUNK, ncf = (d.n + EXT_FCHUNK - 1) / EXT_FCHUNK;
  int32_t *cdone = reinterpret_cast<int32_t *>(cnt + (size_t)EXT_CW * n_ext);  // device commits published
  const int32_t *xl = pipe_xlist(sy);
  const int32_t wdev = (c.score & KOORDHIP_PLUGIN_DEVICESHARE) ? c.w_ext[0] : 0;
  const bool dev = ((c.filt | c.score) & KOORDHIP_PLUGIN_DEVICESHARE) != 0;
  const size_t nn = (size_t)max(d.n, 1);
  if (t == 0) atomicAdd(cdone + 4, 1);  // workgroups started (diagnostics: api.hip pipe_status)
  // dbg (KOORDHIP_STAMPS): final workgroup 0's cycles waiting for the hand-off,
  // final phase, merge + arrival [80..82], its final chunks [87]; pre-evaluation
  // workgroup gf's cycles waiting [89] and evaluating [88]; the last final
  // workgroup's reduce, device commit (after the hand-off), publish [83..85],
  // pods [86]
  uint64_t c_w = 0, c_e = 0, c_m = 0, c_r = 0, c_c = 0, c_p = 0, n_l = 0, n_ch = 0, c_pre = 0, c_pw = 0, c_dc = 0,
           c_pe = 0;
  // claim chunks of a phase until none is left; f(chunk) per claimed chunk
  auto claim_all = [&](uint32_t *claim, int32_t nch, auto f) -> int32_t {
    int32_t done = 0;
    for (;;) {
      if (t == 0) s_ch = (int32_t)__hip_atomic_fetch_add(claim, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __syncthreads();
      const int32_t ch = s_ch;
      __syncthreads();
      if (ch >= nch) return done;  // block-uniform
      done++;
      f(ch);
    }
  };
  // the pre-evaluation chunks of device pod e this workgroup can claim: every
  // node's key (0: infeasible) and raw score into the pod's ring buffer, then
  // the chunks counted as finished
  auto pre_eval = [&](int32_t e) {
    const int32_t gp = ext_idx[e];
    uint32_t *cw = cnt + (size_t)EXT_CW * e;
    const DevPod &p = pods[gp];
    const DevPodX &x = podx[gp];
    uint64_t *bk = pk + (size_t)(e % EXT_RING) * nn;
    int32_t *br = pr + (size_t)(e % EXT_RING) * nn;
    const int32_t pdone = claim_all(cw, ncp, [&](int32_t ch) {
      const int32_t j = ch * EXT_PCHUNK + t;
      if (j < d.n) {
        const int32_t i = perm[j];
        int32_t raw[KOORDHIP_NEXT_PLUGINS] = {0, 0, 0, 0, 0};
        const int32_t tk = seq_eval<SM, true>(c, d, p, x, i, false, raw, nullptr);
        st_wt(&bk[i], (uint64_t)(tk >= 0 ? make_key(tk, i) : 0ull));
        st_wt(&br[i], (int32_t)min(max(raw[0], 0), EXT_RAW - 1));
      }
    });
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0 && pdone) __hip_atomic_fetch_add(cw + 1, (uint32_t)pdone, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  if (b >= gf) {
    // ---- pre-evaluations: device pod e on the state round u's lists see, as
    //      soon as that state is written back (X covers everything later), the
    //      device commits of the device pods before it are published, and its
    //      ring buffer's previous pod has had its final phase
    for (int32_t e = 0; e < n_ext; e++) {
      const int32_t gp = ext_idx[e], u = gp / P;
      uint32_t *cw = cnt + (size_t)EXT_CW * e;  // {pre claimed, pre finished, final claimed, final finished}
      const uint64_t tp0 = dbg ? stamp() : 0;
      if (t == 0)
        s_go = ((u <= lead || wait_at_least_idle(&sy->res_round, u - lead, sy)) && wait_at_least_idle(cdone, needc[e], sy) &&
                (e < EXT_RING || wait_at_least_idle(&sy->ext_done, ext_idx[e - EXT_RING] + 1, sy)))
                   ? 1
                   : 0;
      __syncthreads();
      if (!s_go) {  // the pipeline gave up (block-uniform); the host reports where
        if (t == 0) atomicMax(cdone + 1, (e << 4) | 1);
        break;
      }
      const uint64_t tp1 = dbg ? stamp() : 0;
      pre_eval(e);
      if (dbg && b == gf) {
        c_pw += tp1 - tp0;
        c_pre += stamp() - tp1;
      }
    }
    if (dbg && t == 0 && b == gf) {
      atomicAdd((unsigned long long *)&dbg[88], (unsigned long long)c_pre);
      atomicAdd((unsigned long long *)&dbg[89], (unsigned long long)c_pw);
    }
    return;
  }
  __builtin_amdgcn_s_setprio(2);  // the resolve waits on the final phases: ahead of the evaluation side's waves
  for (int32_t e = 0; e < n_ext; e++) {
    const int32_t gp = ext_idx[e];
    uint32_t *cw = cnt + (size_t)EXT_CW * e;
    const DevPod &p = pods[gp];
    const DevPodX &x = podx[gp];
    const uint64_t *bk = pk + (size_t)(e % EXT_RING) * nn;
    const int32_t *br = pr + (size_t)(e % EXT_RING) * nn;
    // ---- final: at the hand-off, the previous device pod's device commit and
    //      this pod's pre-evaluation published
    for (int r = t; r < EXT_RAW; r += EXT_THREADS) lt[r] = 0ull;
    const uint64_t t0 = dbg ? stamp() : 0;
    uint64_t tw1 = 0, tw2 = 0;
    if (t == 0) {
      s_go = wait_at_least(&sy->ext_req, gp + 1, sy) ? 1 : 0;
      tw1 = dbg ? stamp() : 0;
      s_go = s_go && wait_at_least(cdone, e, sy);
      tw2 = dbg ? stamp() : 0;
    }
    __syncthreads();
    // the pre-evaluation chunks nobody has claimed yet (every condition of the
    // pre-evaluation holds at the hand-off): the final workgroups never wait
    // for a pre-evaluation workgroup the GPU has not started
    if (s_go) pre_eval(e);
    if (t == 0 && s_go) s_go = wait_at_least(reinterpret_cast<const int32_t *>(cw + 1), ncp, sy) ? 1 : 0;
    __syncthreads();
    if (dbg && b == 0 && t == 0) {  // after the hand-off: the previous device commit, then the pre-evaluation
      c_dc += tw2 - tw1;
      c_pe += stamp() - tw2;
    }
    if (!s_go) {
      if (t == 0) atomicMax(cdone + 1, (e << 4) | 2);
      break;
    }
    const uint64_t t1 = dbg ? stamp() : 0;
    const int32_t nx = xl[0];
    // the pre-evaluation saw the state after round u - lead - 1: the nodes
    // committed since are the resolve's X (rounds u - lag .. u) and the commit
    // log of rounds u - lead .. u - lag - 1 (out_node, written through, complete)
    const int32_t u = gp / P;
    const int32_t xlo = max(0, u - lead) * P, xhi = max(0, u - lag) * P;
    const int32_t done = claim_all(cw + 2, ncf, [&](int32_t ch) {
      const int32_t c0 = ch * EXT_FCHUNK;
      for (int32_t w = t; w < EXT_FCHUNK / 32; w += EXT_THREADS) xm[w] = 0u;
      __syncthreads();
      for (int32_t q = t; q < nx; q += EXT_THREADS) {
        const int32_t y = xl[1 + q] - c0;
        if (y >= 0 && y < EXT_FCHUNK) atomicOr(&xm[y >> 5], 1u << (y & 31));
      }
      for (int32_t q = xlo + t; q < xhi; q += EXT_THREADS) {
        const int32_t y = __hip_atomic_load(&out_node[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - c0;
        if (y >= 0 && y < EXT_FCHUNK) atomicOr(&xm[y >> 5], 1u << (y & 31));
      }
      __syncthreads();
      uint64_t kv[EXT_FNPT];
      int32_t rv[EXT_FNPT];
#pragma unroll
      for (int k = 0; k < EXT_FNPT; k++) {  // the pre-evaluated values, all loads in flight
        const int32_t i = c0 + k * EXT_THREADS + t;
        kv[k] = i < d.n ? __hip_atomic_load(&bk[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
        rv[k] = i < d.n ? __hip_atomic_load(&br[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
      }
#pragma unroll 1
      for (int k = 0; k < EXT_FNPT; k++) {
        const int32_t y = k * EXT_THREADS + t, i = c0 + y;
        if (i < d.n && ((xm[y >> 5] >> (y & 31)) & 1u)) {  // committed since the pre-evaluation: evaluate again
          int32_t raw[KOORDHIP_NEXT_PLUGINS] = {0, 0, 0, 0, 0};
          const int32_t tk = seq_eval<SM, true>(c, d, p, x, i, false, raw, nullptr);
          kv[k] = tk >= 0 ? make_key(tk, i) : 0ull;
          rv[k] = min(max(raw[0], 0), EXT_RAW - 1);
        }
      }
#pragma unroll
      for (int k = 0; k < EXT_FNPT; k++)
        if (kv[k]) atomicMax(&lt[rv[k]], kv[k]);
      __syncthreads();  // (xm reused by the next chunk)
    });
    const uint64_t t2 = dbg ? stamp() : 0;
    if (done) {
      for (int r = t; r < EXT_RAW; r += EXT_THREADS)
        if (lt[r]) __hip_atomic_fetch_max(&tab[r], lt[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (t == 0) {
        const uint32_t old = __hip_atomic_fetch_add(cw + 3, (uint32_t)done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = old + (uint32_t)done == (uint32_t)ncf;
        if (s_last) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      }
    } else if (t == 0) {
      s_last = 0;
    }
    __syncthreads();
    const uint64_t t3 = dbg ? stamp() : 0;
    if (dbg && b == 0) {
      c_w += t1 - t0;
      c_e += t2 - t1;
      c_m += t3 - t2;
      n_ch += done;
    }
    if (!s_last) continue;  // block-uniform
    uint64_t v[2];
    int32_t v4[4] = {0, -1, 0, 0};
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const int r = t + h * EXT_THREADS;
      v[h] = r < EXT_RAW ? __hip_atomic_load(&tab[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
      if (v[h]) v4[1] = r;
      if (r < EXT_RAW) __hip_atomic_store(&tab[r], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // the next pod's
    }
    uint64_t kk = 0;
    seq_block_reduce(v4, kk, s_red, s_key, t);
    const int32_t mx = max(v4[1], 0);
    uint64_t best = 0;
#pragma unroll
    for (int h = 0; h < 2; h++)
      if (v[h]) {
        const uint64_t k2 = v[h] + ((uint64_t)(uint32_t)(wdev * norm_score(t + h * EXT_THREADS, mx, false)) << 32);
        best = k2 > best ? k2 : best;
      }
    v4[0] = v4[1] = v4[2] = v4[3] = 0;
    seq_block_reduce(v4, best, s_red, s_key, t);
    const uint64_t t4 = dbg ? stamp() : 0;
    // The node goes back to the resolve first: in the plain build the Reserve
    // cannot fail where the Filter passed on the same state (the same device
    // rows: dev_reserve takes the best `wanted` of the devices dev_eval counted,
    // the extended scalars only add), so the resolve continues while this
    // workgroup commits the devices; the next device pod's workgroups wait for
    // that commit (cdone).  A Reserve that fails anyway stops the pipeline
    // (sync->err = 4) instead of diverging.
    if (t == 0) st_wt(&out_node[gp], best ? key_node(best) : (int32_t)KOORDHIP_UNSCHEDULABLE);
    // every lane's table reset and out_node, drained, then the relaxed hand-off
    // (Guideline 16 R1: no L2 write-back fence)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const uint64_t t5 = dbg ? stamp() : 0;
    if (t == 0) {
      __hip_atomic_store(&sy->ext_done, gp + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      uint32_t slots[DT] = {0u, 0u, 0u};
      if (best) {
        // (nf 2: SM 0 has no Reservation PreScore to skip)
        if (seq_commit_body<SM, false>(c, d, p, x, key_node(best), 2, false, nullptr, dev ? slots : nullptr))
          __hip_atomic_store(&sy->err, 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (out_dev)
        for (int q = 0; q < DT; q++) st_wt(&out_dev[(size_t)gp * DT + q], slots[q]);
      // the device rows and extended scalars (write-through: read next by the
      // next device pod's workgroups on other XCDs), drained, then cdone
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(cdone, e + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (dbg && t == 0) {
      c_r += t4 - t3;
      c_p += t5 - t4;
      c_c += stamp() - t5;
      n_l++;
    }
  }
  if (dbg && t == 0) {
    if (b == 0) {
      atomicAdd((unsigned long long *)&dbg[80], (unsigned long long)c_w);
      atomicAdd((unsigned long long *)&dbg[81], (unsigned long long)c_e);
      atomicAdd((unsigned long long *)&dbg[82], (unsigned long long)c_m);
      atomicAdd((unsigned long long *)&dbg[87], (unsigned long long)n_ch);
      atomicAdd((unsigned long long *)&dbg[94], (unsigned long long)c_dc);
      atomicAdd((unsigned long long *)&dbg[95], (unsigned long long)c_pe);
    }
    atomicAdd((unsigned long long *)&dbg[83], (unsigned long long)c_r);
    atomicAdd((unsigned long long *)&dbg[84], (unsigned long long)c_c);
    atomicAdd((unsigned long long *)&dbg[85], (unsigned long long)c_p);
    atomicAdd((unsigned long long *)&dbg[86], (unsigned long long)n_l);
  }
}

// The pre-evaluation's node order: nodes holding device scalars (any xalloc
// > 0) first, the rest after (their extended-scalar Fit fails for a pod
// requesting one: seq_eval<.., true> returns before their other loads, so
// whole waves of them finish at once).  Order inside each part is free: the
// pre-evaluation writes by node index.  cnt2: two zeroed counters.
__global__ void k_ext_perm(DevDev dv, int32_t n, int32_t *__restrict__ perm, uint32_t *__restrict__ cnt2) {
  const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  bool has = false;
  if (i < n && dv.xalloc)
#pragma unroll
    for (int j = 0; j < KOORDHIP_NXRES; j++) has = has || dv.xalloc[(size_t)j * n + i] > 0;
  const uint64_t bh = __ballot(i < n && has), bo = __ballot(i < n && !has);
  const int lane = threadIdx.x & 63;
  uint32_t ah = 0, ao = 0;
  if (lane == 0) {
    if (bh) ah = atomicAdd(&cnt2[0], (uint32_t)__popcll(bh));
    if (bo) ao = atomicAdd(&cnt2[1], (uint32_t)__popcll(bo));
  }
  ah = __shfl(ah, 0, 64);
  ao = __shfl(ao, 0, 64);
  const uint64_t below = (1ull << lane) - 1ull;
  if (i < n) {
    if (has)
      perm[ah + __popcll(bh & below)] = i;
    else
      perm[n - 1 - (int32_t)(ao + __popcll(bo & below))] = i;
  }
}

// pods[idx[j]].flags |= KH_POD_EXT
__global__ void k_mark_ext(DevPod *pods, const int32_t *__restrict__ idx, int32_t n) {
  const int32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j < n) pods[idx[j]].flags |= KH_POD_EXT;
}

hipError_t launch_mark_ext(DevPod *pods, const int32_t *idx, int32_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_mark_ext, dim3((n + 255) / 256), dim3(256), 0, s, pods, idx, n);
  return hipGetLastError();
}

// The worker's stream holds a quarter of the CUs (api.hip), two workgroups of
// this kernel per CU (its VGPRs): final-phase workgroups about one chunk each,
// at most half the slots; pre-evaluation workgroups on the rest (any subset
// of either group makes progress: chunks are claimed)
static int32_t ext_final_grid(int32_t n_cu, int32_t n) {
  return std::max(1, std::min((n + EXT_FCHUNK - 1) / EXT_FCHUNK, std::max(1, n_cu / 4)));
}
static int32_t ext_worker_grid(int32_t n_cu, int32_t n) {
  return ext_final_grid(n_cu, n) +
         std::max(1, std::min((n + EXT_PCHUNK - 1) / EXT_PCHUNK, std::max(1, n_cu / 2 - ext_final_grid(n_cu, n))));
}

// the zeroed front (table, counters) and the pre-evaluation's per-node keys / raw scores
static size_t ext_front_bytes(int32_t n_ext) {
  return ((size_t)EXT_RAW * sizeof(uint64_t) + ((size_t)EXT_CW * std::max(n_ext, 1) + 5) * sizeof(uint32_t) + 255) &
         ~(size_t)255;
}
size_t ext_worker_scratch_bytes(int32_t n_ext, int32_t n) {
  return ext_front_bytes(n_ext) + (size_t)EXT_RING * std::max(n, 1) * (sizeof(uint64_t) + sizeof(int32_t)) +
         (size_t)std::max(n, 1) * sizeof(int32_t) + 64;
}

size_t ext_worker_diag_offset(int32_t n_ext) {
  return (size_t)EXT_RAW * sizeof(uint64_t) + ((size_t)EXT_CW * std::max(n_ext, 1) + 1) * sizeof(uint32_t);
}

hipError_t launch_ext_worker(const DevCfg &c, const DevNodes &d, const DevPod *pods, const DevPodX *podx,
                             const int32_t *ext_idx, const int32_t *needc, int32_t n_ext, int32_t P, int32_t lag,
                             int32_t lead, int32_t n_cu, void *scratch, int32_t *out_node, uint32_t *out_dev,
                             PipeSync *sync, uint64_t *dbg, hipStream_t s) {
  if (n_ext <= 0) return hipSuccess;
  if (lead < lag) return hipErrorInvalidValue;
  if (seq_mode(c) != 0 || P <= 0) return hipErrorInvalidValue;  // the plain build only (the route checks it)
  char *base = static_cast<char *>(scratch);
  uint64_t *tab = reinterpret_cast<uint64_t *>(base);
  uint32_t *cnt = reinterpret_cast<uint32_t *>(tab + EXT_RAW);
  uint64_t *pk = reinterpret_cast<uint64_t *>(base + ext_front_bytes(n_ext));
  int32_t *pr = reinterpret_cast<int32_t *>(pk + (size_t)EXT_RING * std::max(d.n, 1));
  int32_t *perm = pr + (size_t)EXT_RING * std::max(d.n, 1);
  uint32_t *pc = cnt + (size_t)EXT_CW * n_ext + 2;  // (after cdone and the failure word)
  const int32_t gf = ext_final_grid(n_cu, d.n), grid = ext_worker_grid(n_cu, d.n);
  if (hipError_t e = hipMemsetAsync(scratch, 0, ext_front_bytes(n_ext), s)) return e;
  hipLaunchKernelGGL(k_ext_perm, dim3((d.n + 255) / 256), dim3(256), 0, s, d.dv, d.n, perm, pc);
  hipLaunchKernelGGL(k_ext_worker<0>, dim3(grid), dim3(EXT_THREADS), 0, s, c, d, pods, podx, ext_idx, needc, n_ext, P,
                     lag, lead, gf, tab, cnt, pk, pr, perm, out_node, out_dev, sync, dbg);
  return hipGetLastError();
}

// Every block's granules of one phase: (sum, max, max, max) of words 0..3 and
// the u64 max of words 4..5; false when a spin timed out (every block stops).
template <int NG>
__device__ __forceinline__ bool seq_gather(const uint64_t *g, uint32_t epoch, int32_t G, int32_t v4[4], uint64_t &key,
                                           int32_t (*s_red)[8], uint64_t *s_key, int32_t *s_stop, uint32_t *tmo,
                                           int t) {
  v4[0] = v4[1] = v4[2] = v4[3] = 0;
  key = 0;
  bool ok = true;
  for (int32_t q = t; q < G; q += SEQ_THREADS) {
    uint32_t gv[NG];
    ok &= sweep<NG>(g + (size_t)q * SEQ_GRAN, epoch, gv, tmo);
    v4[0] += (int32_t)gv[0];
#pragma unroll
    for (int e = 1; e < 4; e++) v4[e] = max(v4[e], (int32_t)gv[e]);
    const uint64_t kk = ((uint64_t)gv[4] << 32) | gv[5];
    key = kk > key ? kk : key;
  }
  if (t == 0) *s_stop = 0;
  __syncthreads();
  if (!ok) *s_stop = 1;
  seq_block_reduce(v4, key, s_red, s_key, t);
  return *s_stop == 0;
}

// Every block's (min, max) granule pair of one phase
__device__ __forceinline__ bool seq_gather_minmax(const uint64_t *g, uint32_t epoch, int32_t G, int32_t &mn,
                                                  int32_t &mx, PtsLds &L, int32_t *s_stop, uint32_t *tmo, int t) {
  int32_t a = INT32_MAX, b = 0;
  bool ok = true;
  for (int32_t q = t; q < G; q += SEQ_THREADS) {
    uint32_t gv[2];
    ok &= sweep<2>(g + (size_t)q * SEQ_GRAN, epoch, gv, tmo);
    a = min(a, (int32_t)gv[0]);
    b = max(b, (int32_t)gv[1]);
  }
  __syncthreads();  // the previous use of L.red is finished
  if (t == 0) {
    *s_stop = 0;
    L.red[0] = INT32_MAX;
    L.red[1] = 0;
  }
  __syncthreads();
  if (!ok) *s_stop = 1;
  wave_fold_minmax(a, b, &L.red[0], &L.red[1]);
  __syncthreads();
  mn = L.red[0];
  mx = L.red[1];
  __syncthreads();
  return *s_stop == 0;
}

// Publish one block's (min, max) over L.red (reset to neutral first by the caller)
__device__ __forceinline__ void seq_put_minmax(uint64_t *g, uint32_t epoch, const PtsLds &L, int t) {
  __syncthreads();
  if (t == 0) {
    put_granule(g, epoch, (uint32_t)L.red[0]);
    put_granule(g + 1, epoch, (uint32_t)L.red[1]);
  }
}

// One workgroup per CU: one wave per SIMD, so the kernel may take the whole
// register file (arch VGPRs + AGPRs as spill space) instead of scratch.
template <int SM>
__global__ __launch_bounds__(SEQ_THREADS) __attribute__((amdgpu_waves_per_eu(1, 1))) void k_seq(DevCfg c, DevNodes d,
                                                                                              SeqArgs a) {
  __shared__ int32_t s_red[SEQ_THREADS / 64][8];
  __shared__ int32_t s_tot[SEQ_NPT][SEQ_THREADS];
  __shared__ int32_t s_raw[SEQ_NPT][KOORDHIP_NEXT_PLUGINS][SEQ_THREADS];  // [3]: PodTopologySpread raw, -1 ignored
  __shared__ uint64_t s_key[SEQ_THREADS / 64];
  __shared__ int32_t s_stop;
  __shared__ PtsLds L;
  __shared__ IpaLds IL;
  const int t = threadIdx.x;
  const int32_t G = gridDim.x, b = blockIdx.x;
  const uint32_t ext = a.ext;
  const int32_t zero[KOORDHIP_NEXT_PLUGINS] = {0, 0, 0, 0, 0};
  const PtsArgs &pa = a.pts;
  const bool pts = pa.keys > 0;  // the snapshot has PodTopologySpread tables (and the plugin runs)
  const IpaArgs &ia = a.ipa;
  const bool ipa = ia.ents > 0;  // the snapshot has InterPodAffinity entries (and the plugin runs)
  if (pts) pts_init(pa, d.n, L, t, SEQ_THREADS);
  if (ipa) ipa_load(ia, IL, t, SEQ_THREADS);
  const bool dbg = a.dbg != nullptr && b == 0 && t == 0;
  uint64_t ts = dbg ? seq_stamp() : 0, acc[5] = {0, 0, 0, 0, 0}, sub[3] = {0, 0, 0}, tsub = 0;
  // phase A split (block 0, thread 0, its loads drained): pod prep, its node evaluation, reduce + publish
  auto sublap = [&](int q) {
    if (dbg) {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      const uint64_t u = seq_stamp();
      if (q > 0) sub[q - 1] += u - tsub;
      tsub = u;
    }
  };
  auto lap = [&](int q) {
    if (dbg) {
      const uint64_t u = seq_stamp();
      acc[q] += u - ts;
      ts = u;
    }
  };
  for (int32_t p = 0; p < a.n_pods; p++) {
    sublap(0);
    const DevPod pod = a.pods[p];
    const DevPodX &x = a.podx ? a.podx[p] : kNoPodX;
    const uint32_t eA = 2u * (uint32_t)p + 1u, eB = 2u * (uint32_t)p + 2u, eP = (uint32_t)p + 1u;
    const int par = p & 1;
    // ---- PodTopologySpread: the pod's pair counters from the replicas, and
    //      for a DoNotSchedule hostname constraint the grid's minimum over
    //      the hard-eligible nodes (its own hand-off)
    const PtsPod q = pts ? pts_pod(pa, x) : PtsPod{};
    const bool soft = q.on && q.ns > 0;
    // InterPodAffinity: Filter entries, and Score entries (weights read from
    // the staged record: a register copy of 32 weights would spill)
    const bool iaf = ipa && ia.filt && (x.ipa_aff | x.ipa_anti) != 0u;
    const uint32_t isc = (ipa && ia.score && a.podx) ? x.ipa_score : 0u;
    const int32_t *iw = isc ? a.podx[p].ipa_w : nullptr;
    const bool wide = soft || isc != 0u;  // phase A publishes words 6..16 too
    int32_t hmin = INT32_MAX;
    if (q.on) {
      pts_prep(pa, q, L, t);
      if (q.hhost) {
        int32_t m = INT32_MAX;
        for (int k = 0; k < a.npt; k++) {
          const int32_t i = (k * G + b) * SEQ_THREADS + t;
          if (i >= d.n) continue;
          for (int kk = 0; kk < PK; kk++)
            if (((q.hkeys & pa.host) >> kk) & 1u) {
              const int32_t v = pts_host_match(pa, q, kk, d.n, i);
              if (v >= 0) m = min(m, v);
            }
        }
        wave_fold_minmax(m, 0, &L.red[0], &L.red[1]);
        seq_put_minmax(a.g0 + ((size_t)par * G + b) * SEQ_GRAN, eP, L, t);
        int32_t unused;
        if (!seq_gather_minmax(a.g0 + (size_t)par * G * SEQ_GRAN, eP, G, hmin, unused, L, &s_stop, a.tmo, t)) return;
        if (t == 0) {
          L.red[0] = INT32_MAX;
          L.red[1] = 0;
        }
        __syncthreads();
      }
    }
    // ---- phase A: this block's nodes (totals and raw scores kept in LDS for
    //      phase B: registers for SEQ_NPT slices would spill).  The block also
    //      ranks its nodes as if every normalized maximum were 0, which is
    //      exact whenever it is (then every normalized score is the same
    //      constant): such pods need one hand-off, not two.
    // (PodTopologySpread Score without ScheduleAnyway constraints: 100 for every node)
    const int32_t pts_const = (pa.score && !soft) ? 100 * pa.w : 0;
    (void)pts;
    int32_t v4[4] = {0, 0, 0, 0};  // feasible count, raw maxima
    uint64_t key0 = 0;
    int32_t imn = INT32_MAX, imx = INT32_MIN;  // InterPodAffinity raw Score over this block's feasible nodes
    uint32_t smk[PK][2] = {};                  // PodTopologySpread soft pairs of this thread's feasible nodes
    int32_t snf = 0;
    if (dbg) {
      (void)pod.req[0];
      (void)x.flags;
    }
    sublap(1);
#pragma unroll 1
    for (int k = 0; k < a.npt; k++) {
      int32_t tk = -1, rk[KOORDHIP_NEXT_PLUGINS] = {0, 0, 0, -1, 0};
      const int32_t i = (k * G + b) * SEQ_THREADS + t;
      if (i < d.n) {
        tk = seq_eval<SM>(c, d, pod, x, i, a.rs != 0, rk, nullptr);
        rk[3] = -1;
        if (tk >= 0 && q.on && q.hard && !pts_filter(pa, q, L, hmin, d.n, i)) tk = -1;
        if (tk >= 0 && iaf && !ipa_filter(ia, IL, x, d.n, i)) tk = -1;
        if (tk >= 0 && isc) {
          rk[4] = ipa_raw(ia, IL, isc, iw, d.n, i);
          imn = min(imn, rk[4]);
          imx = max(imx, rk[4]);
        }
        if (tk >= 0) {
          v4[0]++;
#pragma unroll
          for (int e = 0; e < 3; e++) v4[1 + e] = max(v4[1 + e], rk[e]);
          if (soft) rk[3] = pts_soft_mark(pa, q, d.n, i, smk, snf) ? 0 : -1;
          const uint64_t kk = make_key(rank_add(c, tk, ext_total(c, ext, rk, zero) + pts_const), i);
          key0 = kk > key0 ? kk : key0;
        }
      }
      s_tot[k][t] = tk;
#pragma unroll
      for (int e = 0; e < KOORDHIP_NEXT_PLUGINS; e++) s_raw[k][e][t] = rk[e];
    }
    sublap(2);
    if (soft) pts_soft_fold(L, smk, snf);  // (L.smask / nfni zeroed by pts_prep; the reduce's barriers order it)
    if (isc) {
      if (t == 0) {
        IL.mm[0] = INT32_MAX;
        IL.mm[1] = INT32_MIN;
      }
      __syncthreads();
      wave_fold_minmax(imn, imx, &IL.mm[0], &IL.mm[1]);
    }
    seq_block_reduce(v4, key0, s_red, s_key, t);  // (its barriers order the atomics above)
    if (t == 0) {
      uint64_t *g = a.ga + ((size_t)par * G + b) * SEQ_GRAN;
#pragma unroll
      for (int e = 0; e < 4; e++) put_granule(g + e, eA, (uint32_t)v4[e]);
      put_granule(g + 4, eA, (uint32_t)(key0 >> 32));
      put_granule(g + 5, eA, (uint32_t)key0);
      if (wide) {
        put_granule(g + 6, eA, soft ? (uint32_t)L.nfni : 0u);
#pragma unroll
        for (int e = 0; e < 2 * PK; e++) put_granule(g + 7 + e, eA, soft ? (&L.smask[0][0])[e] : 0u);
        put_granule(g + 15, eA, isc ? (uint32_t)IL.mm[0] : 0u);
        put_granule(g + 16, eA, isc ? (uint32_t)IL.mm[1] : 0u);
      }
    }
    sublap(3);
    lap(0);
    // ---- every block's granules: the feasible count, the raw maxima and the
    //      best key under zero maxima (+ PodTopologySpread's PreScore pairs)
    int32_t g4[4];
    uint64_t win;
    if (wide) {
      if (!seq_gather<17>(a.ga + (size_t)par * G * SEQ_GRAN, eA, G, g4, win, s_red, s_key, &s_stop, a.tmo, t))
        return;
    } else {
      if (!seq_gather<6>(a.ga + (size_t)par * G * SEQ_GRAN, eA, G, g4, win, s_red, s_key, &s_stop, a.tmo, t)) return;
    }
    const int32_t nf_all = g4[0];
    lap(1);
    // InterPodAffinity: the grid's raw min / max over the feasible nodes
    // (words 15, 16: their epochs were checked by the sweep above)
    int32_t gimn = 0, gimx = 0;
    if (isc) {
      __syncthreads();
      if (t == 0) {
        IL.mm[0] = INT32_MAX;
        IL.mm[1] = INT32_MIN;
      }
      __syncthreads();
      int32_t a15 = INT32_MAX, a16 = INT32_MIN;
      for (int32_t g = t; g < G; g += SEQ_THREADS) {
        const uint64_t *gg = a.ga + ((size_t)par * G + g) * SEQ_GRAN;
        a15 = min(a15, (int32_t)(uint32_t)__hip_atomic_load(const_cast<uint64_t *>(gg) + 15, __ATOMIC_RELAXED,
                                                             __HIP_MEMORY_SCOPE_AGENT));
        a16 = max(a16, (int32_t)(uint32_t)__hip_atomic_load(const_cast<uint64_t *>(gg) + 16, __ATOMIC_RELAXED,
                                                             __HIP_MEMORY_SCOPE_AGENT));
      }
      wave_fold_minmax(a15, a16, &IL.mm[0], &IL.mm[1]);
      __syncthreads();
      gimn = IL.mm[0];
      gimx = IL.mm[1];
    }
    const bool inorm = isc && gimx > gimn;  // else every normalized InterPodAffinity score is 0
    int32_t pmin = 0, pmax = 0;
    if (soft) {
      // ---- PodTopologySpread PreScore + Score: weights from the grid's pairs,
      //      this block's raw scores, the grid's min / max over non-ignored nodes
      uint32_t mask[PK][2];
      int32_t nfni = 0;
      {
        // (the masks and count were reduced into s_red / s_key words by seq_gather's
        // sweep of words 6.. -- re-read them here: every thread sweeps the granules once more)
        for (int e = 0; e < PK; e++) mask[e][0] = mask[e][1] = 0u;
        __syncthreads();
        if (t == 0) {
          L.nfni = 0;
          for (int e = 0; e < 2 * PK; e++) (&L.smask[0][0])[e] = 0u;
        }
        __syncthreads();
        {
          uint32_t gm[PK][2] = {};
          int32_t gc = 0;
          for (int32_t g = t; g < G; g += SEQ_THREADS) {
            const uint64_t *gg = a.ga + ((size_t)par * G + g) * SEQ_GRAN;
            gc += (int32_t)(uint32_t)__hip_atomic_load(const_cast<uint64_t *>(gg) + 6, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
            for (int e = 0; e < 2 * PK; e++)
              gm[e >> 1][e & 1] |= (uint32_t)__hip_atomic_load(const_cast<uint64_t *>(gg) + 7 + e, __ATOMIC_RELAXED,
                                                               __HIP_MEMORY_SCOPE_AGENT);
          }
          pts_soft_fold(L, gm, gc);
        }
        __syncthreads();
        nfni = L.nfni;
        for (int e = 0; e < PK; e++) {
          mask[e][0] = L.smask[e][0];
          mask[e][1] = L.smask[e][1];
        }
        __syncthreads();
        if (t == 0) {
          L.red[0] = INT32_MAX;
          L.red[1] = 0;
        }
        __syncthreads();
      }
      double w[PP];
      pts_weights(pa, q, mask, nfni, w);
      int32_t mn = INT32_MAX, mx = 0;
#pragma unroll 1
      for (int k = 0; k < a.npt; k++) {
        const int32_t i = (k * G + b) * SEQ_THREADS + t;
        if (s_tot[k][t] < 0 || s_raw[k][3][t] < 0) continue;
        const int32_t r = pts_raw(pa, q, L, w, d.n, i);
        s_raw[k][3][t] = r;
        mn = min(mn, r);
        mx = max(mx, r);
      }
      wave_fold_minmax(mn, mx, &L.red[0], &L.red[1]);
      seq_put_minmax(a.gp + ((size_t)par * G + b) * SEQ_GRAN, eP, L, t);
      if (!seq_gather_minmax(a.gp + (size_t)par * G * SEQ_GRAN, eP, G, pmin, pmax, L, &s_stop, a.tmo, t)) return;
    }
    if ((g4[1] | g4[2] | g4[3]) || soft || inorm) {
      // ---- phase B: normalized totals, this block's best key
      const int32_t gmx[KOORDHIP_NEXT_PLUGINS] = {g4[1], g4[2], g4[3], 0};
      uint64_t best = 0;
#pragma unroll 1
      for (int k = 0; k < a.npt; k++) {
        const int32_t tk = s_tot[k][t];
        if (tk < 0) continue;
        const int32_t i = (k * G + b) * SEQ_THREADS + t;
        const int32_t rk[KOORDHIP_NEXT_PLUGINS] = {s_raw[k][0][t], s_raw[k][1][t], s_raw[k][2][t], 0};
        const int32_t pt = soft ? pa.w * pts_norm(s_raw[k][3][t], pmin, pmax) : pts_const;
        const int32_t it = inorm ? ia.w * ipa_norm(s_raw[k][4][t], gimn, gimx) : 0;
        const uint64_t key = make_key(rank_add(c, tk, ext_total(c, ext, rk, gmx) + pt + it), i);
        best = key > best ? key : best;
      }
      int32_t u4[4] = {0, 0, 0, 0};
      seq_block_reduce(u4, best, s_red, s_key, t);
      if (t == 0) {
        uint64_t *g = a.gb + ((size_t)par * G + b) * SEQ_GRAN;
#pragma unroll
        for (int e = 0; e < 4; e++) put_granule(g + e, eB, 0u);
        put_granule(g + 4, eB, (uint32_t)(best >> 32));
        put_granule(g + 5, eB, (uint32_t)best);
      }
      lap(2);
      if (!seq_gather<6>(a.gb + (size_t)par * G * SEQ_GRAN, eB, G, u4, win, s_red, s_key, &s_stop, a.tmo, t)) return;
      lap(3);
    }
    // ---- the winner's owner block commits (its nodes are read by no other block)
    const int32_t wn = win ? key_node(win) : -1;
    // PodTopologySpread: a placed pod counts for the table constraints it
    // matches; a Reserve that may fail (devices, cpusets) tells the others
    const uint32_t pmatch = (pts && wn >= 0) ? x.pts_match : 0u;
    // InterPodAffinity: the entries counting the placed pod
    const uint32_t imatch = (ipa && wn >= 0) ? x.ipa_inc : 0u;
    bool may_fail = ((c.filt | c.score) & KOORDHIP_PLUGIN_DEVICESHARE) && (x.flags & KOORDHIP_PODX_DEVICE);
    if constexpr (SM >= 1) may_fail = may_fail || (numa_on(c) && numa_active(pod, c));
    if (t == 0) {
      const bool mine = wn >= 0 ? ((wn / SEQ_THREADS) % G) == b : b == 0;
      if (mine) {
        const uint64_t c0 = a.dbg ? seq_stamp() : 0;
        seq_commit<SM>(a.gc, a.gd, a.pods + p, a.podx ? a.podx + p : nullptr, wn, nf_all, a.rs != 0, a.out_node + p,
                       a.out_cpus ? a.out_cpus + (size_t)p * NW : nullptr,
                       a.out_dev ? a.out_dev + (size_t)p * DT : nullptr);
        if (pmatch | imatch) {
          const bool done = __hip_atomic_load(a.out_node + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == wn;
          if (done) {
            for (int cc = 0; cc < pa.cons; cc++)
              if ((pmatch >> cc) & 1u) pa.cnt[(size_t)cc * d.n + wn] += 1;
            ipa_commit_cols(ia, imatch, d.n, wn);
          }
          if (may_fail) put_granule(a.gr + par, eP, done ? 1u : 0u);
        }
        if (a.dbg) atomicAdd((unsigned long long *)&a.dbg[5], (unsigned long long)(seq_stamp() - c0));
      }
      if (pmatch | imatch) {
        bool done = true;
        if (may_fail) {
          uint32_t v[1];
          if (!sweep<1>(a.gr + par, eP, v, a.tmo)) s_stop = 1;
          done = v[0] != 0;
        }
        if (done) {
          if (pmatch) pts_commit_tables(pa, L, pmatch, d.n, wn);
          if (imatch) ipa_commit_tables(ia, IL, imatch, d.n, wn);
        }
      }
    }
    __syncthreads();  // the owner's commit before its next evaluation of w
    if (s_stop) return;
    lap(4);
  }
  if (dbg) {
    for (int q2 = 0; q2 < 5; q2++) a.dbg[q2] = acc[q2];
    for (int q2 = 0; q2 < 3; q2++) a.dbg[6 + q2] = sub[q2];
  }
}

// ---- parity evaluation (koordhip_eval_ext): per (pod, node) the status bits,
// the raw score planes and the per-node total; then per pod the maxima and
// the top-k of the normalized totals
template <int SM>
__global__ __launch_bounds__(256) void k_seq_eval(DevCfg c, DevNodes d, const DevPod *__restrict__ pods, const DevPodX *__restrict__ podx,
                           int32_t n_pods, int32_t rs, uint8_t *__restrict__ status, int32_t *__restrict__ scores,
                           int32_t *__restrict__ work) {
  const int32_t i = blockIdx.x * blockDim.x + threadIdx.x, p = blockIdx.y;
  if (i >= d.n || p >= n_pods) return;
  const DevPod pod = pods[p];
  DevPodX x{};
  if (podx) {
    x = podx[p];
  } else {
    x.req[0][0] = x.req[0][1] = x.req[0][2] = -1;
  }
  int32_t raw[KOORDHIP_NEXT_PLUGINS];
  uint8_t st = 0;
  const int32_t t = seq_eval<SM>(c, d, pod, x, i, rs != 0, raw, &st);
  const size_t n = (size_t)d.n;
  int32_t *wk = work + (size_t)p * SEQ_WORK_PLANES * n;
  wk[i] = t;
  for (int e = 0; e < KOORDHIP_NEXT_PLUGINS; e++) wk[(size_t)(e + 1) * n + i] = raw[e];
  if (status) status[(size_t)p * n + i] |= st;
  if (scores) {
    int32_t *row = scores + (size_t)p * (KOORDHIP_NPLUGINS + KOORDHIP_NEXT_PLUGINS) * n;
    for (int e = 0; e < KOORDHIP_NEXT_PLUGINS; e++) row[(size_t)(KOORDHIP_NPLUGINS + e) * n + i] = raw[e];
  }
}

// PodTopologySpread for the parity evaluator: one workgroup per pod over
// every node (its own replicas of the pair counters, from the columns):
// the Filter's status bit and infeasible total, the raw Score plane (0 on
// infeasible and ignored nodes) and work plane 4 (raw, -1 = not scored).
__global__ __launch_bounds__(256) void k_pts_eval(PtsArgs pa, int32_t n, const DevPodX *__restrict__ podx,
                                                  int32_t n_pods, uint8_t *__restrict__ status,
                                                  int32_t *__restrict__ scores, int32_t *__restrict__ work) {
  __shared__ PtsLds L;
  const int32_t p = blockIdx.x, t = threadIdx.x;
  if (p >= n_pods) return;
  DevPodX x{};
  if (podx) {
    x = podx[p];
  } else {
    x.req[0][0] = x.req[0][1] = x.req[0][2] = -1;
  }
  const size_t NPX = KOORDHIP_NPLUGINS + KOORDHIP_NEXT_PLUGINS;
  int32_t *wk = work + (size_t)p * SEQ_WORK_PLANES * n;
  int32_t *w4 = wk + (size_t)4 * n;
  int32_t *plane = scores ? scores + ((size_t)p * NPX + KOORDHIP_NPLUGINS + 3) * n : nullptr;
  const PtsPod q = pts_pod(pa, x);
  if (!q.on) {
    for (int32_t i = t; i < n; i += 256) {
      w4[i] = wk[i] >= 0 ? 0 : -1;
      if (plane) plane[i] = 0;
    }
    return;
  }
  pts_init(pa, n, L, t, 256);
  pts_prep(pa, q, L, t);
  int32_t hmin = INT32_MAX;
  if (q.hhost) {
    int32_t m = INT32_MAX;
    for (int32_t i = t; i < n; i += 256)
      for (int k = 0; k < PK; k++)
        if (((q.hkeys & pa.host) >> k) & 1u) {
          const int32_t v = pts_host_match(pa, q, k, n, i);
          if (v >= 0) m = min(m, v);
        }
    wave_fold_minmax(m, 0, &L.red[0], &L.red[1]);
    __syncthreads();
    hmin = L.red[0];
  }
  for (int32_t i = t; i < n; i += 256)
    if (q.nh > 0 && !pts_filter(pa, q, L, hmin, n, i)) {
      wk[i] = -1;
      if (status) status[(size_t)p * n + i] |= KOORDHIP_ST_PTS_FAIL;
    }
  __syncthreads();
  {
    uint32_t sm[PK][2] = {};
    int32_t sc = 0;
    for (int32_t i = t; i < n; i += 256) {
      w4[i] = wk[i] >= 0 ? ((q.ns == 0 || pts_soft_mark(pa, q, n, i, sm, sc)) ? 0 : -1) : -1;
      if (plane) plane[i] = 0;
    }
    pts_soft_fold(L, sm, sc);
  }
  __syncthreads();
  if (q.ns == 0) return;
  uint32_t mask[PK][2];
  for (int e = 0; e < PK; e++) {
    mask[e][0] = L.smask[e][0];
    mask[e][1] = L.smask[e][1];
  }
  double w[PP];
  pts_weights(pa, q, mask, L.nfni, w);
  for (int32_t i = t; i < n; i += 256)
    if (w4[i] >= 0) {
      const int32_t r = pts_raw(pa, q, L, w, n, i);
      w4[i] = r;
      if (plane) plane[i] = r;
    }
}

// The launch's sums (one workgroup-local LDS table per block, then one global
// add per nonzero cell).  sums must be zeroed before.
__global__ __launch_bounds__(256) void k_ipa_sums(IpaArgs a, int32_t n) {
  __shared__ int32_t s[IPA_SUMS];
  for (int x = threadIdx.x; x < IPA_SUMS; x += blockDim.x) s[x] = 0;
  __syncthreads();
  for (int32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    for (int e = 0; e < a.ents; e++) {
      const int32_t v = a.cnt[(size_t)e * n + i];
      if (v == 0) continue;
      const int k = a.ent_key[e];
      const int32_t d = a.dom[(size_t)k * n + i];
      if (d < 0) continue;
      atomicAdd(&s[IE * PD + e], v);
      if (!((a.host >> k) & 1u)) atomicAdd(&s[e * PD + d], v);
    }
  __syncthreads();
  for (int x = threadIdx.x; x < IPA_SUMS; x += blockDim.x)
    if (s[x]) atomicAdd(&a.sums[x], s[x]);
}

// InterPodAffinity for the parity evaluator: one workgroup per pod over every
// node (the launch's sums from k_ipa_sums): the Filter's status plane and
// infeasible total, the raw Score plane and work plane 5 (every node).
__global__ __launch_bounds__(256) void k_ipa_eval(IpaArgs a, int32_t n, const DevPodX *__restrict__ podx,
                                                  int32_t n_pods, uint8_t *__restrict__ ist,
                                                  int32_t *__restrict__ scores, int32_t *__restrict__ work) {
  __shared__ IpaLds L;
  const int32_t p = blockIdx.x, t = threadIdx.x;
  if (p >= n_pods || !podx) return;
  const DevPodX &x = podx[p];
  const size_t NPX = KOORDHIP_NPLUGINS + KOORDHIP_NEXT_PLUGINS;
  int32_t *wk = work + (size_t)p * SEQ_WORK_PLANES * n;
  int32_t *w5 = wk + (size_t)5 * n;
  int32_t *plane = scores ? scores + ((size_t)p * NPX + KOORDHIP_NPLUGINS + 4) * n : nullptr;
  ipa_load(a, L, t, 256);
  const bool filt = a.filt && (x.ipa_aff | x.ipa_anti) != 0u;
  const uint32_t sc = a.score ? x.ipa_score : 0u;
  for (int32_t i = t; i < n; i += 256) {
    if (filt && !ipa_filter(a, L, x, n, i)) {
      wk[i] = -1;
      if (ist) ist[(size_t)p * n + i] = 1;
    }
    const int32_t r = sc ? ipa_raw(a, L, sc, x.ipa_w, n, i) : 0;
    w5[i] = r;
    if (plane) plane[i] = r;
  }
}

__global__ __launch_bounds__(256) void k_seq_topk(DevCfg c, int32_t n, const int32_t *__restrict__ work, int32_t k,
                                                  int32_t pts_w, int32_t ipa_w, uint64_t *__restrict__ out) {
  __shared__ uint64_t s_k[4];
  __shared__ int32_t s_m[4][KOORDHIP_NEXT_PLUGINS + 2];
  const int32_t p = blockIdx.x, t = threadIdx.x, lane = __lane_id(), wv = t >> 6;
  const int32_t *wk = work + (size_t)p * SEQ_WORK_PLANES * n;
  const uint32_t ext = ext_bits(c);
  int32_t mx[KOORDHIP_NEXT_PLUGINS] = {0, 0, 0, 0, INT32_MIN}, pmin = INT32_MAX, imin = INT32_MAX;
  for (int32_t i = t; i < n; i += 256)
    if (wk[i] >= 0) {
      for (int e = 0; e < 3; e++) mx[e] = max(mx[e], wk[(size_t)(e + 1) * n + i]);
      const int32_t r = wk[(size_t)4 * n + i];
      if (r >= 0) {
        mx[3] = max(mx[3], r);
        pmin = min(pmin, r);
      }
      const int32_t q = wk[(size_t)5 * n + i];
      mx[4] = max(mx[4], q);
      imin = min(imin, q);
    }
  for (int e = 0; e < KOORDHIP_NEXT_PLUGINS; e++) {
    for (int m = 32; m >= 1; m >>= 1) mx[e] = max(mx[e], __shfl_xor(mx[e], m));
    if (lane == 0) s_m[wv][e] = mx[e];
  }
  pmin = pts_wave_min(pmin);
  imin = pts_wave_min(imin);
  if (lane == 0) {
    s_m[wv][KOORDHIP_NEXT_PLUGINS] = pmin;
    s_m[wv][KOORDHIP_NEXT_PLUGINS + 1] = imin;
  }
  __syncthreads();
  for (int e = 0; e < KOORDHIP_NEXT_PLUGINS; e++) mx[e] = max(max(s_m[0][e], s_m[1][e]), max(s_m[2][e], s_m[3][e]));
  pmin = min(min(s_m[0][KOORDHIP_NEXT_PLUGINS], s_m[1][KOORDHIP_NEXT_PLUGINS]),
             min(s_m[2][KOORDHIP_NEXT_PLUGINS], s_m[3][KOORDHIP_NEXT_PLUGINS]));
  imin = min(min(s_m[0][KOORDHIP_NEXT_PLUGINS + 1], s_m[1][KOORDHIP_NEXT_PLUGINS + 1]),
             min(s_m[2][KOORDHIP_NEXT_PLUGINS + 1], s_m[3][KOORDHIP_NEXT_PLUGINS + 1]));
  uint64_t last = ~0ull;
  for (int32_t j = 0; j < k; j++) {
    uint64_t best = 0;
    for (int32_t i = t; i < n; i += 256) {
      if (wk[i] < 0) continue;
      int32_t raw[KOORDHIP_NEXT_PLUGINS];
      for (int e = 0; e < KOORDHIP_NEXT_PLUGINS; e++) raw[e] = wk[(size_t)(e + 1) * n + i];
      const int32_t pt = pts_w ? pts_w * pts_norm(raw[3], pmin, mx[3]) : 0;
      const int32_t it = ipa_w ? ipa_w * ipa_norm(raw[4], imin, mx[4]) : 0;
      const uint64_t key = make_key(rank_add(c, wk[i], ext_total(c, ext, raw, mx) + pt + it), i);
      if (key < last && key > best) best = key;
    }
    best = seq_wave_max(best);
    __syncthreads();
    if (lane == 0) s_k[wv] = best;
    __syncthreads();
    best = s_k[0];
    for (int w = 1; w < 4; w++) best = s_k[w] > best ? s_k[w] : best;
    if (t == 0) out[(size_t)p * k + j] = best;
    last = best ? best : 1ull;  // once exhausted, every later entry is 0
  }
}

hipError_t launch_seq(const DevCfg &c, const DevNodes &d, const DevPod *pods, const DevPodX *podx, int32_t n_pods,
                      int32_t grid, uint64_t *granules, uint32_t *tmo, int32_t *out_node, uint64_t *out_cpus,
                      uint32_t *out_dev, int32_t rs, uint64_t *dbg, void *desc, const PtsArgs &pts,
                      const IpaArgs &ipa, hipStream_t s) {
  if (n_pods <= 0) return hipSuccess;
  SeqArgs a{};
  a.dbg = dbg;
  a.pts = pts;
  a.ipa = ipa;
  if (ipa.ents > 0) {  // this launch's domain sums of the count entries
    if (hipError_t e = hipMemsetAsync(ipa.sums, 0, sizeof(int32_t) * IPA_SUMS, s)) return e;
    hipLaunchKernelGGL(k_ipa_sums, dim3(std::min<int32_t>(1024, (d.n + 255) / 256)), dim3(256), 0, s, ipa, d.n);
  }
  // the commit's copies of the config and the column descriptors (desc: 16-B aligned device buffer)
  DevCfg *gc = static_cast<DevCfg *>(desc);
  DevNodes *gd = reinterpret_cast<DevNodes *>(static_cast<char *>(desc) + seq_desc_cfg_bytes());
  if (hipError_t e = hipMemcpyAsync(gc, &c, sizeof(DevCfg), hipMemcpyHostToDevice, s)) return e;
  if (hipError_t e = hipMemcpyAsync(gd, &d, sizeof(DevNodes), hipMemcpyHostToDevice, s)) return e;
  a.gc = gc;
  a.gd = gd;
  a.pods = pods;
  a.podx = podx;
  a.n_pods = n_pods;
  a.npt = (d.n + grid * SEQ_THREADS - 1) / (grid * SEQ_THREADS);
  if (a.npt > SEQ_NPT) return hipErrorInvalidValue;
  a.ga = granules;
  a.gb = granules + (size_t)2 * grid * SEQ_GRAN;
  a.g0 = granules + (size_t)4 * grid * SEQ_GRAN;
  a.gp = granules + (size_t)6 * grid * SEQ_GRAN;
  a.gr = granules + (size_t)8 * grid * SEQ_GRAN;
  a.tmo = tmo;
  a.out_node = out_node;
  a.out_cpus = out_cpus;
  a.out_dev = out_dev;
  a.ext = 0u;
  if (c.score & KOORDHIP_PLUGIN_DEVICESHARE) a.ext |= 1u;
  if (c.score & KOORDHIP_PLUGIN_AFFINITY_SCORE) a.ext |= 2u;
  if (c.score & KOORDHIP_PLUGIN_TAINT_SCORE) a.ext |= 4u;
  a.rs = rs;
  // Every block must be resident (blocks read each other's granules).  The
  // occupancy is checked here and the kernel launched as an ordinary
  // dispatch: nothing else runs on the device meanwhile (the pipelined
  // path's persistent resolve is joined before any sequential batch), so the
  // grid of one block per CU is resident.  (hipLaunchCooperativeKernel gave
  // the same residency, but its cooperative queue is torn down by the HIP
  // runtime at process exit, after a profiler's finalisation: every
  // rocprofv3 trace of a k_seq workload died with SIGSEGV in exit().)
  const int sm = seq_mode(c);
  const void *f = sm == 3   ? (const void *)k_seq<3>
                  : sm == 2 ? (const void *)k_seq<2>
                  : sm == 1 ? (const void *)k_seq<1>
                            : (const void *)k_seq<0>;
  int dev = 0, ncu = 0, per_cu = 0;
  if (hipError_t e = hipGetDevice(&dev)) return e;
  if (hipError_t e = hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev)) return e;
  if (hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, f, SEQ_THREADS, 0)) return e;
  if ((int64_t)per_cu * ncu < grid) return hipErrorCooperativeLaunchTooLarge;
  switch (sm) {
    case 3: hipLaunchKernelGGL(k_seq<3>, dim3(grid), dim3(SEQ_THREADS), 0, s, c, d, a); break;
    case 2: hipLaunchKernelGGL(k_seq<2>, dim3(grid), dim3(SEQ_THREADS), 0, s, c, d, a); break;
    case 1: hipLaunchKernelGGL(k_seq<1>, dim3(grid), dim3(SEQ_THREADS), 0, s, c, d, a); break;
    default: hipLaunchKernelGGL(k_seq<0>, dim3(grid), dim3(SEQ_THREADS), 0, s, c, d, a);
  }
  return hipGetLastError();
}

const char *seq_kernel_name(const DevCfg &c) {
  static const char *names[4] = {"kh::k_seq<0>", "kh::k_seq<1>", "kh::k_seq<2>", "kh::k_seq<3>"};
  return names[seq_mode(c)];
}

hipError_t launch_seq_eval(const DevCfg &c, const DevNodes &d, const DevPod *pods, const DevPodX *podx, int32_t n_pods,
                           int32_t rs, uint8_t *status, uint8_t *ipa_status, int32_t *scores, int32_t *work, int32_t k,
                           uint64_t *topk, const PtsArgs &pts, const IpaArgs &ipa, hipStream_t s) {
  if (n_pods <= 0 || d.n <= 0) return hipSuccess;
  const dim3 g((d.n + 255) / 256, n_pods);
  switch (seq_mode(c)) {
    case 3: hipLaunchKernelGGL(k_seq_eval<3>, g, dim3(256), 0, s, c, d, pods, podx, n_pods, rs, status, scores, work); break;
    case 2: hipLaunchKernelGGL(k_seq_eval<2>, g, dim3(256), 0, s, c, d, pods, podx, n_pods, rs, status, scores, work); break;
    case 1: hipLaunchKernelGGL(k_seq_eval<1>, g, dim3(256), 0, s, c, d, pods, podx, n_pods, rs, status, scores, work); break;
    default: hipLaunchKernelGGL(k_seq_eval<0>, g, dim3(256), 0, s, c, d, pods, podx, n_pods, rs, status, scores, work);
  }
  // InterPodAffinity's Filter before PodTopologySpread's PreScore reads the feasible set
  if (ipa.ents > 0) {
    if (hipError_t e = hipMemsetAsync(ipa.sums, 0, sizeof(int32_t) * IPA_SUMS, s)) return e;
    hipLaunchKernelGGL(k_ipa_sums, dim3(std::min<int32_t>(1024, (d.n + 255) / 256)), dim3(256), 0, s, ipa, d.n);
    hipLaunchKernelGGL(k_ipa_eval, dim3(n_pods), dim3(256), 0, s, ipa, d.n, podx, n_pods, ipa_status, scores, work);
  }
  hipLaunchKernelGGL(k_pts_eval, dim3(n_pods), dim3(256), 0, s, pts, d.n, podx, n_pods, status, scores, work);
  if (topk && k > 0)
    hipLaunchKernelGGL(k_seq_topk, dim3(n_pods), dim3(256), 0, s, c, d.n, work, k, pts.score ? pts.w : 0,
                       ipa.score ? ipa.w : 0, topk);
  return hipGetLastError();
}

}  // namespace kh
