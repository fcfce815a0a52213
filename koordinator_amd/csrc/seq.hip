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

#include <cstdlib>
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
// k_seq's instantiation: the Reservation builds without DeviceShare and
// without a reservation holding devices or extended scalars take 4 / 5
static inline int seq_launch_mode(const DevCfg &c, const DevNodes &d) {
  const int sm = seq_mode(c);
  const bool nodev = !((c.filt | c.score) & KOORDHIP_PLUGIN_DEVICESHARE) && !d.dv.rslot && !d.dv.rxa;
  return (sm >= 2 && nodev) ? sm + 2 : sm;
}
// k_seq only: SM 4 / 5 = SM 2 / 3 without DeviceShare and without a
// reservation holding devices (the device and device-reservation code compiled
// out: the Reservation + NodeNUMAResource profiles keep their registers)
template <int SM>
constexpr int kSeqSlots = (SM == 3 || SM == 5) ? KOORDHIP_RESV_SLOTS_MAX : KOORDHIP_RESV_SLOTS;
template <int SM>
constexpr bool kSeqDev = SM < 4;
template <int SM>
using SeqResvRow = NumaRowRS<kSeqSlots<SM>>;

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
// EARLY (k_ext_pre / k_ext_final: no status, no raw planes of infeasible nodes): a node
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
    constexpr int S = kSeqSlots<SM>;
    SeqResvRow<SM> nr{};
    load_numa<false>(nr, d, i, all);  // (the zone row shares the reserved CPUs' bytes: eval_total_resv<.., Z> reads it)
    load_resv(nr, d.rv, i);
    DevRC rc{-1, 0, 0, 0u};
    ResvXS rx = no_rx();
    if constexpr (kSeqDev<SM>) {
      rc = seq_dev_resv(c, d.dv, p, x, nr, i);
      rx = seq_resv_x(d, p, x, nr, i);
      if (rx.h >= 0 && (c.filt & KOORDHIP_PLUGIN_FIT)) xfr = (rx.f & RX_XFIT) != 0u;  // on the restored scalars
    }
    t = c.zones       ? eval_total_resv<S, true, true>(p, v, nr, d.nu.cls, c, &d, i, rx)
        : c.resv_cpus ? eval_total_resv<S, true>(p, v, nr, d.nu.cls, c, nullptr, 0, rx)
                      : eval_total_resv<S, false>(p, v, nr, d.nu.cls, c, nullptr, 0, rx);
    if constexpr (kSeqDev<SM>) {
      const int32_t nq = (rs && (x.flags & KOORDHIP_PODX_DEVICE)) ? resv_nominate(p, nr, resv_matched(nr, p), rx) : -1;
      if (rc.h >= 0)
        df = rc_eval(c, d.dv, x, i, rc, nq, (c.filt & KOORDHIP_PLUGIN_DEVICESHARE) != 0,
                     (c.score & KOORDHIP_PLUGIN_DEVICESHARE) != 0, &raw[0]);
      else
        df = dev_eval(c, d.dv, x, i, nq >= 0, (c.filt & KOORDHIP_PLUGIN_DEVICESHARE) != 0,
                      (c.score & KOORDHIP_PLUGIN_DEVICESHARE) != 0, &raw[0]);
    }
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
// ROW false (k_ext_final): the Fit / LoadAware row is the pipelined
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
    if constexpr (kSeqDev<SM>) {
      rc = seq_dev_resv(c, d.dv, p, x, rv, w);
      rx = seq_resv_x(d, p, x, rv, w);
    }
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
  const bool dev = kSeqDev<SM> && ((c.filt | c.score) & KOORDHIP_PLUGIN_DEVICESHARE) != 0;
  // the loads of every row the Reserve changes go out first (one round trip
  // with the device rows' instead of one per structure): the Fit / LoadAware
  // row and the extended scalars' Requested
  NV v;
  if constexpr (ROW) load_row(v, d, w);
  int64_t xr[KOORDHIP_NXRES];
#pragma unroll
  for (int j = 0; j < KOORDHIP_NXRES; j++) xr[j] = ((x.xmask >> j) & 1u) ? d.dv.xreq[(size_t)j * d.n + w] : 0;
  if constexpr (kSeqDev<SM>)
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
  if constexpr (kSeqDev<SM>)
    if (dev) {
      dev_apply<!ROW>(d.dv, w, slots, per);
      if (rc.h >= 0 && qa == rc.h) rc_apply_allocated<!ROW>(d.dv, w, slots, per);
    }
  if constexpr (SM >= 2) {  // Reservation Reserve: assumePod into the nominated reservation
    const int qz = resv_assume(rv, p, m, rx);
    store_resv(rv, d.rv, w);
    if (kSeqDev<SM> && qz >= 0 && qz == rx.h && x.xmask)  // ... its extended scalars' Allocated (masked to its keys)
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
// Two TRANSIENT launches per device pod run that pod's reference cycle: every
// node's Filter and per-node total, DeviceShare's raw Score (0 .. 100 per
// requested type, scoring.go:33-72) and the normalization over the feasible
// nodes (DefaultNormalizeScore, scoring.go:78-80):
//   k_ext_pre    (after the resolve finished round u - lead: the state every
//                later commit is in X or the commit log of) every node's key
//                make_key(total, i) (0: infeasible) and raw score into pk / pr;
//   k_ext_final  (after the hand-off) only the X nodes and the log nodes are
//                evaluated again (every other node's value is the
//                pre-evaluation's); the normalized total of a node is its total
//                + w * norm(raw), so the winner is among the best (total,
//                lowest index) node of each raw value: every workgroup folds its
//                chunk into a [EXT_RAW] table of such keys in LDS and merges it
//                into the global one with agent-scope atomic max; the last
//                arriving workgroup takes the maximum raw value, ranks the
//                <= EXT_RAW candidates, stores out_node write-through and
//                ext_done = pod + 1, then runs DeviceShare's Reserve (device
//                choice + deviceUsed, the extended scalars; not the Fit /
//                LoadAware row, which the resolve commits in its own copy).
// Both sit on ONE stream in an order whose every wait is satisfiable by the
// launches before it (api.hip), each behind a one-workgroup wait launch: no
// workgroup of theirs waits for another kernel while it holds a CU, so the
// pipeline's only persistent workgroups are the resolve's and the class
// lists' (round 5's persistent worker grid -- 128 workgroups of one per CU --
// left some XCD no CU for a class build's 1024-thread collect workgroup, which
// is dealt to a fixed XCD: the build stream stalled behind it, the class lists
// and the resolve behind the build; profiles/r05q_ext_lead.txt,
// gpurun_out/r05j_dsmix.err).
constexpr int EXT_RAW = 320;  // raw DeviceShare scores 0 .. 300 (three device types x 100)
constexpr int EXT_THREADS = 256;
constexpr int32_t EXT_PCHUNK = EXT_THREADS;      // pre-evaluation chunk: one node per thread
constexpr int EXT_FNPT = 4;                      // final chunk: four nodes per thread (two loads each)
constexpr int32_t EXT_FCHUNK = EXT_THREADS * EXT_FNPT;
constexpr int EXT_RING = 4;   // pre-evaluation buffers: device pods evaluated ahead of their hand-off
constexpr int EXT_DMAX = 32;  // device pods a final tracks as possibly missed by its pre-evaluation

// DeviceShare's Reserve of a device pod on node w without the Fit / LoadAware
// row (seq_commit_body<0, false>: dev_reserve, allocator.go:91-122, then
// deviceUsed and the extended scalars' Requested), by ONE wave: lane l < DT x
// DS holds dev slot l % DS of type l / DS (every row in one load round trip;
// one lane's dependent loads cost ~40k cycles), the `wanted` best fitting
// devices of a type by (score desc, minor asc) -- minors are unique on a node,
// so that order is strict and each lane's rank among its type's lanes decides
// -- and lanes 32 .. 39 the extended scalars.  The same allocation as
// dev_reserve; false (nothing applied) where it fails.  All 64 lanes call it.
__device__ __noinline__ bool ext_commit_wave(const DevCfg &c, const DevNodes &d, const DevPodX &x, int32_t w,
                                             uint32_t slots[DT]) {
  const int lane = threadIdx.x & 63;
  const DevDev &dv = d.dv;
  const bool devp = ((c.filt | c.score) & KOORDHIP_PLUGIN_DEVICESHARE) && (x.flags & KOORDHIP_PODX_DEVICE) &&
                    dv.slots > 0 && dv.present;
  const int t = lane / DS, s = lane % DS;
  int64_t qt[DR] = {0, 0, 0};
  const bool req = t < DT && devp && dev_requests(x, t, qt);
  const bool mine = req && s < dv.slots;
  int32_t mi = -1;
  int64_t tot[DR] = {0, 0, 0}, usd[DR] = {0, 0, 0}, fr[DR] = {0, 0, 0};
  size_t a0 = 0;
  const bool present = devp && dv.present[w] != 0;
  if (mine) {
    a0 = dev_at(dv, w, t, s) * DR;
    mi = dv.minor[a0 / DR];
#pragma unroll
    for (int r = 0; r < DR; r++) {
      tot[r] = dv.total[a0 + r];
      usd[r] = dv.used[a0 + r];
      fr[r] = tot[r] - usd[r] > 0 ? tot[r] - usd[r] : 0;
    }
  }
  const int j = lane - 32;
  const bool xl = j >= 0 && j < KOORDHIP_NXRES && ((x.xmask >> j) & 1u);
  const int64_t xr = xl ? dv.xreq[(size_t)j * d.n + w] : 0;
  bool ok = true, any = false;
  uint64_t take = 0ull;
  int64_t myper[DR] = {0, 0, 0};
  for (int u = 0; u < DT && present; u++) {
    int64_t q[DR];
    if (!dev_requests(x, u, q)) continue;
    any = true;
    const uint64_t has = __ballot(t == u && mine && mi >= 0);
    if (!has) {
      ok = false;  // dev_has_type
      break;
    }
    if (u == KOORDHIP_DEV_GPU) {  // fillGPUTotalMem: the lowest slot with resources
      const uint64_t wr = __ballot(t == u && mine && mi >= 0 && (tot[0] != 0 || tot[1] != 0 || tot[2] != 0));
      if (!wr) {
        ok = false;
        break;
      }
      const int64_t mem = __shfl(tot[2], __builtin_ctzll(wr), 64);
      if (q[2] >= 0) {
        const double f = (double)q[2] / (double)mem;  // memoryBytesToRatio, float64
        q[1] = (int64_t)(f * 100.0);
      } else {
        q[2] = (q[1] > 0 ? q[1] : 0) * mem / 100;  // memoryRatioToBytes
      }
      if (q[0] < 0) q[0] = 0;
    }
    int64_t per[DR];
    const int64_t want = dev_wanted(u, q, per);
    const bool fit = t == u && mine && mi >= 0 && !dev_zero(fr) && dev_fits(per, fr);
    const int64_t sc = fit ? dev_scorer(c, u, tot, fr, per) : -1;
    int32_t rank = 0;
#pragma unroll
    for (int k = 0; k < DS; k++) {
      const int64_t os = __shfl(sc, u * DS + k, 64);
      const int32_t om = __shfl(mi, u * DS + k, 64);
      rank += (os >= 0 && (os > sc || (os == sc && om < mi))) ? 1 : 0;
    }
    const uint64_t fits = __ballot(fit);
    if ((int64_t)__popcll(fits) < want) {
      ok = false;
      break;
    }
    const bool mine_taken = fit && rank < want;
    take |= __ballot(mine_taken);
    if (t == u)
#pragma unroll
      for (int r = 0; r < DR; r++) myper[r] = per[r];
  }
  (void)any;
  if (!ok) return false;
  if (((take >> lane) & 1ull) && mine)
#pragma unroll
    for (int r = 0; r < DR; r++) st_wt(&dv.used[a0 + r], (int64_t)(usd[r] + myper[r]));
  if (xl) st_wt(&dv.xreq[(size_t)j * d.n + w], (int64_t)(xr + x.xreq[j]));
#pragma unroll
  for (int u = 0; u < DT; u++) slots[u] = (uint32_t)((take >> (u * DS)) & ((1ull << DS) - 1ull));
  return true;
}

// flags (ExtScr::fl), each on a 128-B line of its own (pipe.hpp: many pollers
// of one line delay its writer): pre-evaluations finished, finals finished
// (their ring buffer read), device commits published, the gates the first
// workgroup of a spinning pre-evaluation / final opens for the others; relaxed
// agent-scope words, each stored after the data it covers was written through
// and drained (Guideline 16 R1).  EXT_PERM: the permutation's two counters;
// EXT_REEV: the finals' re-evaluated nodes of the call.
enum {
  EXT_PREDONE = 0,
  EXT_FDONE = 32,
  EXT_CDONE = 64,
  EXT_PERM = 96,
  EXT_REEV = 100,
  EXT_GPRE = 128,
  EXT_GFIN = 160,
  EXT_GFA = 192,
  EXT_FLAGS = 224
};

// A gate waiter (every workgroup of a spinning grid but the first): polls its
// own line only, the pipeline's error word every 64th poll (pipe.hpp: a poller
// of the error word polls the line of sel / res_round, which the resolve and
// the class workgroups use)
static __device__ __forceinline__ uint64_t realtime() {  // 100 MHz, one clock for every CU
  uint64_t t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

static __device__ bool wait_gate(const int32_t *p, int32_t v, PipeSync *sy) {
  const uint64_t t0 = stamp();
  for (uint32_t k = 0; load_relaxed(p) < v; k++) {
    if ((k & 63u) == 63u) {
      if (load_relaxed(&sy->err)) return false;
      if (stamp() - t0 > PIPE_WATCHDOG) {
        store_release(&sy->err, 1);
        return false;
      }
    }
    __builtin_amdgcn_s_sleep(2);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  return true;
}

template <int SM>
__global__ __launch_bounds__(EXT_THREADS) void k_ext_pre(DevCfg c, DevNodes d, const DevPod *__restrict__ pods,
                                                         const DevPodX *__restrict__ podx, int32_t e, int32_t gp,
                                                         uint64_t *__restrict__ bk, int32_t *__restrict__ br,
                                                         const int32_t *__restrict__ perm, uint32_t *__restrict__ parr,
                                                         int32_t *__restrict__ fl, PipeSync *sy, int32_t rounds,
                                                         int32_t needc, int32_t fdone, int32_t spin) {
  if (spin) {  // the waits of k_wait_ext_pre inside the grid (no launch boundary after them)
    __shared__ int32_t s_ok;
    if (threadIdx.x == 0) {
      bool ok;
      if (blockIdx.x == 0) {  // one poller of the pipeline's lines, then the gate
        ok = rounds <= 0 || wait_at_least(&sy->res_round, rounds, sy);
        ok = ok && (needc <= 0 || wait_at_least(&fl[EXT_CDONE], needc, sy));
        ok = ok && (fdone <= 0 || wait_at_least(&fl[EXT_FDONE], fdone, sy));
        if (ok) __hip_atomic_store(&fl[EXT_GPRE], e + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        ok = wait_gate(&fl[EXT_GPRE], e + 1, sy);
      }
      s_ok = ok;
    }
    __syncthreads();
    if (!s_ok) return;
  }
  if (__hip_atomic_load(&sy->err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;  // the pipeline gave up
  const int32_t j = (int32_t)blockIdx.x * EXT_PCHUNK + (int32_t)threadIdx.x;
  if (j < d.n) {
    const int32_t i = perm[j];
    int32_t raw[KOORDHIP_NEXT_PLUGINS] = {0, 0, 0, 0, 0};
    const int32_t tk = seq_eval<SM, true>(c, d, pods[gp], podx[gp], i, false, raw, nullptr);
    st_wt(&bk[i], (uint64_t)(tk >= 0 ? make_key(tk, i) : 0ull));
    st_wt(&br[i], (int32_t)min(max(raw[0], 0), EXT_RAW - 1));
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0 &&
      __hip_atomic_fetch_add(parr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u == gridDim.x)
    __hip_atomic_store(&fl[EXT_PREDONE], e + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// tab: [EXT_RAW] u64 (zero between pods: the last workgroup resets it), arrive:
// this pod's arrival counter (zeroed per call).  The X nodes: pipe_xlist; the
// log nodes: out_node of rounds [xlo, xhi) (the pre-evaluation's state is after
// round u - lead - 1, the resolve's X covers rounds u - lag .. u).
template <int SM>
__global__ __launch_bounds__(EXT_THREADS) void k_ext_final(DevCfg c, DevNodes d, const DevPod *__restrict__ pods,
                                                           const DevPodX *__restrict__ podx, int32_t gp, int32_t xlo,
                                                           int32_t xhi, uint64_t *__restrict__ tab,
                                                           uint32_t *__restrict__ arrive,
                                                           uint64_t *__restrict__ bk,
                                                           int32_t *__restrict__ br, int32_t *__restrict__ out_node,
                                                           uint32_t *__restrict__ out_dev, int32_t e,
                                                           int32_t *__restrict__ fl, PipeSync *sy, uint64_t *dbg,
                                                           int32_t spin, const int32_t *__restrict__ ext_idx,
                                                           int32_t dlo) {
  __shared__ uint64_t lt[EXT_RAW];
  __shared__ uint32_t xm[EXT_FCHUNK / 32];  // the chunk's X nodes
  __shared__ int32_t s_red[SEQ_THREADS / 64][8];
  __shared__ uint64_t s_key[SEQ_THREADS / 64];
  __shared__ int32_t s_last;
  __shared__ uint32_t s_nre;
  __shared__ int32_t s_ok[2];
  __shared__ int32_t s_dn[EXT_DMAX];  // the nodes of the device pods [dlo, e): committed maybe after the pre-evaluation read
  __shared__ int32_t s_dok[EXT_DMAX], s_draw[EXT_DMAX];  // ... their DeviceShare / extended-scalar part for this pod
  __shared__ int32_t s_nd, s_cd;
  const int t = threadIdx.x;
  const int32_t c0 = (int32_t)blockIdx.x * EXT_FCHUNK;
  // spin: the grid is resident before the hand-off (launched behind the
  // previous final) -- the pre-evaluation is awaited and its values loaded
  // first, then the hand-off, so no launch boundary sits between the
  // resolve's request and the fold
  if (spin) {  // the first workgroup polls the flags and opens the gates
    if (t == 0) {
      if (blockIdx.x == 0) {
        // hand-off timeline (s_memrealtime, dbg[96..100]): [96] finals whose request was set before
        // their grid started, [97] / [99] pods whose pre-evaluation was published after the request
        // and the time waited for it, [98] request seen -> published, [100] the current request seen
        const bool req0 = dbg && load_relaxed(&sy->ext_req) >= gp + 1;
        const uint64_t ta = dbg ? realtime() : 0;
        if (req0) atomicAdd((unsigned long long *)&dbg[96], 1ull);
        s_ok[0] = wait_at_least(&fl[EXT_PREDONE], e + 1, sy);
        if (dbg && s_ok[0] && (req0 || load_relaxed(&sy->ext_req) >= gp + 1) && realtime() - ta > 20) {
          atomicAdd((unsigned long long *)&dbg[97], 1ull);
          atomicAdd((unsigned long long *)&dbg[99], (unsigned long long)(realtime() - ta));
        }
        if (s_ok[0]) __hip_atomic_store(&fl[EXT_GFA], e + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        s_ok[0] = wait_gate(&fl[EXT_GFA], e + 1, sy);
      }
    }
    __syncthreads();
    if (!s_ok[0]) return;
  }
  uint64_t kv[EXT_FNPT];
  int32_t rv[EXT_FNPT];
#pragma unroll
  for (int k = 0; k < EXT_FNPT; k++) {  // the pre-evaluated values, all loads in flight
    const int32_t i = c0 + k * EXT_THREADS + t;
    kv[k] = i < d.n ? __hip_atomic_load(&bk[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
    rv[k] = i < d.n ? __hip_atomic_load(&br[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
  }
  // The device pods [dlo, e) -- committed maybe after the pre-evaluation read
  // their nodes -- have all committed before this final runs (the finals of a
  // stream run in order; the wait covers KOORDHIP_EXT_ALT's second stream):
  // their nodes' device rows and extended scalars are final until this pod's
  // own Reserve, so the DeviceShare Filter / raw score and the extended-scalar
  // Fit of those nodes are evaluated now, while the hand-off is pending
  // (measured: ~12 us of dependent loads on the critical path otherwise)
  const int32_t gi = (t < e - dlo && t < EXT_DMAX) ? ext_idx[dlo + t] : -1;
  if (t == 0) {
    s_nre = 0u;
    s_nd = e - dlo <= EXT_DMAX ? e - dlo : -1;  // (-1: too many, every re-evaluation in full)
    s_cd = e == 0 || wait_gate(&fl[EXT_CDONE], e, sy);
  }
  __syncthreads();
  if (!s_cd) return;  // the pipeline gave up
  if (gi >= 0) s_dn[t] = __hip_atomic_load(&out_node[gi], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  if (t < s_nd) {
    const int32_t y = s_dn[t];
    if (y >= c0 && y < c0 + EXT_FCHUNK && y < d.n) {
      const DevPodX &x0 = podx[gp];
      const bool xf = !(c.filt & KOORDHIP_PLUGIN_FIT) || xfit_filter(d.dv, x0, y, d.n);
      int32_t raw0 = 0;
      const bool df = dev_eval(c, d.dv, x0, y, false, (c.filt & KOORDHIP_PLUGIN_DEVICESHARE) != 0,
                               (c.score & KOORDHIP_PLUGIN_DEVICESHARE) != 0, &raw0);
      s_dok[t] = (xf && df) ? 1 : 0;
      s_draw[t] = min(max(raw0, 0), EXT_RAW - 1);
    }
  }
  if (spin) {
    if (t == 0) {
      if (blockIdx.x == 0) {
        // the hand-off, and the previous device pod's Reserve published (the
        // finals alternate between two streams: final e - 1 may still commit)
        s_ok[1] = wait_at_least(&sy->ext_req, gp + 1, sy) && (e == 0 || wait_at_least(&fl[EXT_CDONE], e, sy));
        if (dbg) __hip_atomic_store(&dbg[100], realtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (s_ok[1]) __hip_atomic_store(&fl[EXT_GFIN], gp + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        s_ok[1] = wait_gate(&fl[EXT_GFIN], gp + 1, sy);
      }
    }
    __syncthreads();
    if (!s_ok[1]) return;
  }
  uint64_t tg = 0, tm = 0, te = 0;  // (dbg: this workgroup's phase times, s_memrealtime)
  if (dbg && t == 0) tg = realtime();
  // the hand-off happened and the pre-evaluation is published (the waits
  // above or the wait launch before this one), unless the pipeline gave up
  if (__hip_atomic_load(&sy->ext_req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != gp + 1 ||
      __hip_atomic_load(&fl[EXT_PREDONE], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < e + 1 ||
      __hip_atomic_load(&sy->err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
    return;  // (grid-uniform)
  const uint64_t t0 = (dbg && blockIdx.x == 0) ? stamp() : 0;
  const DevPod &p = pods[gp];
  const DevPodX &x = podx[gp];
  const int32_t *xl = pipe_xlist(sy);
  const int32_t wdev = (c.score & KOORDHIP_PLUGIN_DEVICESHARE) ? c.w_ext[0] : 0;
  const bool dev = ((c.filt | c.score) & KOORDHIP_PLUGIN_DEVICESHARE) != 0;
  // one round trip for X's count and nodes (read speculatively: X <= kPipeXMax
  // < EXT_THREADS nodes) and the nodes of the device pods [dlo, e) (published
  // before this pod's hand-off)
  static_assert(kPipeXMax <= EXT_THREADS, "one X node per thread");
  const int32_t nx = xl[0];
  const int32_t xv = t < kPipeXMax ? xl[1 + t] : -1;
  for (int r = t; r < EXT_RAW; r += EXT_THREADS) lt[r] = 0ull;
  for (int32_t w = t; w < EXT_FCHUNK / 32; w += EXT_THREADS) xm[w] = 0u;
  __syncthreads();
  if (t < nx) {
    const int32_t y = xv - c0;
    if (y >= 0 && y < EXT_FCHUNK) atomicOr(&xm[y >> 5], 1u << (y & 31));
  }
  for (int32_t q = xlo + t; q < xhi; q += EXT_THREADS) {
    const int32_t y = __hip_atomic_load(&out_node[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - c0;
    if (y >= 0 && y < EXT_FCHUNK) atomicOr(&xm[y >> 5], 1u << (y & 31));
  }
  __syncthreads();
  if (dbg && t == 0) tm = realtime();
  int32_t s_fullw = 0;  // (dbg: this thread evaluated a node in full)
#pragma unroll 1
  for (int k = 0; k < EXT_FNPT; k++) {
    const int32_t y = k * EXT_THREADS + t, i = c0 + y;
    // committed since the pre-evaluation: evaluate again -- unless the node was
    // infeasible then (every Filter of the plain build is monotone in the
    // commits of the batch -- Fit / LoadAware requests, DeviceShare's device
    // usage and the extended scalars only grow -- so it still is)
    //
    // A node no device pod committed to since the pre-evaluation read it keeps
    // its device rows and extended scalars (only device pods change them):
    // its DeviceShare Filter / raw score and extended-scalar Fit stand, and
    // only the row part -- seq_eval's eval_total over the Fit / LoadAware row,
    // one row load -- is evaluated again; the nodes of the device pods the
    // pre-evaluation may have missed (s_dn) take the part evaluated above.
    if (i < d.n && kv[k] != 0ull && ((xm[y >> 5] >> (y & 31)) & 1u)) {
      if (s_nd < 0) {
        s_fullw = 1;
        int32_t raw[KOORDHIP_NEXT_PLUGINS] = {0, 0, 0, 0, 0};
        const int32_t tk = seq_eval<SM, true>(c, d, p, x, i, false, raw, nullptr);
        kv[k] = tk >= 0 ? make_key(tk, i) : 0ull;
        rv[k] = min(max(raw[0], 0), EXT_RAW - 1);
      } else {
        int32_t jd = -1;
        for (int32_t j = 0; j < s_nd; j++)
          if (s_dn[j] == i) jd = j;
        NV v{};
        load_node(v, d, i, need_all(c), c);
        int32_t tk = eval_total(p, v, c);
        if (jd >= 0) {
          s_fullw = 1;
          if (!s_dok[jd]) tk = -1;
          rv[k] = s_draw[jd];
        }
        kv[k] = tk >= 0 ? make_key(tk, i) : 0ull;
      }
      atomicAdd(&s_nre, 1u);
    }
  }
  if (dbg) {
    __syncthreads();
    if (t == 0) te = realtime();
  }
  const bool anyfull = dbg && __syncthreads_or(s_fullw) != 0;
#pragma unroll
  for (int k = 0; k < EXT_FNPT; k++)
    if (kv[k]) atomicMax(&lt[rv[k]], kv[k]);
  __syncthreads();
  for (int r = t; r < EXT_RAW; r += EXT_THREADS)
    if (lt[r]) __hip_atomic_fetch_max(&tab[r], lt[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (t == 0 && s_nre)  // executed evaluations (the call's re-evaluated nodes)
    __hip_atomic_fetch_add(reinterpret_cast<uint32_t *>(&fl[EXT_REEV]), s_nre, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0) {
    const uint32_t old = __hip_atomic_fetch_add(arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = old + 1u == gridDim.x;
    if (s_last) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    if (dbg && spin) {  // [102..105] per workgroup: request seen -> gate seen -> X marked -> re-evaluated -> arrived
      const uint64_t ts = __hip_atomic_load(&dbg[100], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), ta = realtime();
      atomicAdd((unsigned long long *)&dbg[102], (unsigned long long)(tg > ts ? tg - ts : 0));
      atomicAdd((unsigned long long *)&dbg[103], (unsigned long long)(tm - tg));
      atomicAdd((unsigned long long *)&dbg[104], (unsigned long long)(te - tm));
      atomicAdd((unsigned long long *)&dbg[105], (unsigned long long)(ta - te));
      atomicAdd((unsigned long long *)&dbg[106], 1ull);
      if (anyfull) {  // [110] / [111] workgroups with a full re-evaluation, their re-evaluation time
        atomicAdd((unsigned long long *)&dbg[110], 1ull);
        atomicAdd((unsigned long long *)&dbg[111], (unsigned long long)(te - tm));
      }
      if (s_last) atomicAdd((unsigned long long *)&dbg[101], (unsigned long long)(ta - ts));
    }
  }
  __syncthreads();
  if (!s_last) return;  // block-uniform
  const uint64_t t1 = dbg ? stamp() : 0;
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
  // The node goes back to the resolve first: in the plain build the Reserve
  // cannot fail where the Filter passed on the same state (the same device
  // rows: dev_reserve takes the best `wanted` of the devices dev_eval counted,
  // the extended scalars only add), so the resolve continues while this
  // workgroup commits the devices; the next device pod's launches come after
  // this one on the stream.  A Reserve that fails anyway stops the pipeline
  // (sync->err = 4) instead of diverging.
  if (t == 0) st_wt(&out_node[gp], best ? key_node(best) : (int32_t)KOORDHIP_UNSCHEDULABLE);
  // every lane's table reset and out_node, drained, then the relaxed hand-off
  // (Guideline 16 R1: no L2 write-back fence)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0) {
    __hip_atomic_store(&sy->ext_done, gp + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (dbg && spin) {  // [98] request seen -> published; [99] / [100] pods whose pre-evaluation came later
      const uint64_t ts = __hip_atomic_load(&dbg[100], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      atomicAdd((unsigned long long *)&dbg[98], (unsigned long long)(realtime() - ts));
    }
    __hip_atomic_store(&fl[EXT_FDONE], e + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // its ring buffer is read
  }
  const uint64_t t2 = dbg ? stamp() : 0;
  if (t < 64) {  // wave 0: the device Reserve (every lane)
    uint32_t slots[DT] = {0u, 0u, 0u};
    const bool okc = !best || ext_commit_wave(c, d, x, key_node(best), slots);
    if (t == 0) {
      if (!okc) __hip_atomic_store(&sy->err, 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (out_dev)
        for (int q = 0; q < DT; q++) st_wt(&out_dev[(size_t)gp * DT + q], okc ? slots[q] : 0u);
    }
    // the device rows and extended scalars (write-through), drained, then cdone
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  if (t == 0) {
    __hip_atomic_store(&fl[EXT_CDONE], e + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (dbg) {  // [80] evaluate + fold (workgroup 0), [83] decide + publish, [84] device commit, [86] pods
      atomicAdd((unsigned long long *)&dbg[83], (unsigned long long)(t2 - t1));
      atomicAdd((unsigned long long *)&dbg[84], (unsigned long long)(stamp() - t2));
      atomicAdd((unsigned long long *)&dbg[86], 1ull);
    }
  }
  if (dbg && blockIdx.x == 0 && t == 0) atomicAdd((unsigned long long *)&dbg[80], (unsigned long long)(t1 - t0));
}

// one thread waits until a pre-evaluation may start: the resolve finished
// round `rounds` - 1 (rounds > 0), the device commits of the first `needc`
// device pods are published, the final `fdone` - 1 read its ring buffer
__global__ void k_wait_ext_pre(PipeSync *sy, int32_t *fl, int32_t rounds, int32_t needc, int32_t fdone) {
  if (threadIdx.x != 0) return;
  bool ok = rounds <= 0 || wait_at_least(&sy->res_round, rounds, sy);
  ok = ok && (needc <= 0 || wait_at_least(&fl[EXT_CDONE], needc, sy));
  ok = ok && (fdone <= 0 || wait_at_least(&fl[EXT_FDONE], fdone, sy));
  (void)ok;
}
// ... and until a final may start: the resolve's hand-off of device pod gp
// (ext_req = gp + 1) and the pod's pre-evaluation (e + 1 finished)
__global__ void k_wait_ext_final(PipeSync *sy, int32_t *fl, int32_t want, int32_t pre) {
  if (threadIdx.x != 0) return;
  if (wait_at_least(&sy->ext_req, want, sy) && wait_at_least(&fl[EXT_PREDONE], pre, sy))
    (void)(pre <= 1 || wait_at_least(&fl[EXT_CDONE], pre - 1, sy));  // (the previous device pod's Reserve)
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

// scratch: [EXT_RAW] table, per device pod the final's and the pre-evaluation's
// arrival counters, the flags (the zeroed front), then the RING
// pre-evaluation buffers (keys u64, raw i32 per node) and the node permutation
static size_t ext_fl_off(int32_t n_ext) {
  return ((size_t)EXT_RAW * sizeof(uint64_t) + (size_t)2 * std::max(n_ext, 1) * sizeof(uint32_t) + 127) &
         ~(size_t)127;
}
static size_t ext_front_bytes(int32_t n_ext) {
  return (ext_fl_off(n_ext) + (size_t)EXT_FLAGS * sizeof(int32_t) + 255) & ~(size_t)255;
}
size_t ext_scratch_bytes(int32_t n_ext, int32_t n) {
  return ext_front_bytes(n_ext) + (size_t)EXT_RING * std::max(n, 1) * (sizeof(uint64_t) + sizeof(int32_t)) +
         (size_t)std::max(n, 1) * sizeof(int32_t) + 64;
}
int32_t ext_ring() { return EXT_RING; }

struct ExtScr {
  uint64_t *tab;
  uint32_t *arrive, *parr;
  int32_t *fl;  // [EXT_FLAGS] (the enum above), 128-B aligned
  uint64_t *pk;
  int32_t *pr;
  int32_t *perm;
};
static ExtScr ext_scr(void *scratch, int32_t n_ext, int32_t n) {
  char *base = static_cast<char *>(scratch);
  ExtScr x;
  x.tab = reinterpret_cast<uint64_t *>(base);
  x.arrive = reinterpret_cast<uint32_t *>(x.tab + EXT_RAW);
  x.parr = x.arrive + std::max(n_ext, 1);
  x.fl = reinterpret_cast<int32_t *>(base + ext_fl_off(n_ext));
  x.pk = reinterpret_cast<uint64_t *>(base + ext_front_bytes(n_ext));
  x.pr = reinterpret_cast<int32_t *>(x.pk + (size_t)EXT_RING * std::max(n, 1));
  x.perm = x.pr + (size_t)EXT_RING * std::max(n, 1);
  return x;
}

// The finals spin in their own grid (launched behind the previous final, so
// resident before the hand-off: no launch boundary between the resolve's
// request and the fold); the pre-evaluations wait in a one-workgroup launch
// ahead of each (off the critical path, and a grid of a few hundred spinning
// workgroups would hold CUs the builds need).  KOORDHIP_EXT_WAITK: the finals
// behind wait launches too (A/B); KOORDHIP_EXT_PRESPIN: the pre-evaluations
// spin too (A/B).  0 / 1 / 2: none / finals / both.
static int32_t ext_spin() {
  static const int32_t v = std::getenv("KOORDHIP_EXT_WAITK") ? 0 : std::getenv("KOORDHIP_EXT_PRESPIN") ? 2 : 1;
  return v;
}

const uint32_t *ext_reevals(const void *scratch, int32_t n_ext, int32_t n) {
  const ExtScr x = ext_scr(const_cast<void *>(scratch), n_ext, n);
  return reinterpret_cast<const uint32_t *>(x.fl + EXT_REEV);
}

hipError_t launch_ext_begin(const DevNodes &d, int32_t n_ext, void *scratch, hipStream_t s) {
  const ExtScr x = ext_scr(scratch, n_ext, d.n);
  if (hipError_t e = hipMemsetAsync(scratch, 0, ext_front_bytes(n_ext), s)) return e;
  hipLaunchKernelGGL(k_ext_perm, dim3((d.n + 255) / 256), dim3(256), 0, s, d.dv, d.n, x.perm,
                     reinterpret_cast<uint32_t *>(x.fl + EXT_PERM));
  return hipGetLastError();
}

hipError_t launch_ext_pre(const DevCfg &c, const DevNodes &d, const DevPod *pods, const DevPodX *podx, int32_t e,
                          int32_t gp, int32_t rounds, int32_t needc, int32_t n_ext, void *scratch, PipeSync *sync,
                          hipStream_t s) {
  if (seq_mode(c) != 0) return hipErrorInvalidValue;  // the plain build only (the route checks it)
  const ExtScr x = ext_scr(scratch, n_ext, d.n);
  const size_t nn = (size_t)std::max(d.n, 1);
  const int32_t spin = ext_spin() > 1;  // (pre-evaluations spin only with KOORDHIP_EXT_PRESPIN)
  if (!spin && (rounds > 0 || needc > 0 || e >= EXT_RING))
    hipLaunchKernelGGL(k_wait_ext_pre, dim3(1), dim3(64), 0, s, sync, x.fl, rounds, needc, e - EXT_RING + 1);
  hipLaunchKernelGGL(k_ext_pre<0>, dim3((d.n + EXT_PCHUNK - 1) / EXT_PCHUNK), dim3(EXT_THREADS), 0, s, c, d, pods, podx,
                     e, gp, x.pk + (size_t)(e % EXT_RING) * nn, x.pr + (size_t)(e % EXT_RING) * nn, x.perm, x.parr + e,
                     x.fl, sync, rounds, needc, e - EXT_RING + 1, spin);
  return hipGetLastError();
}

hipError_t launch_ext_final(const DevCfg &c, const DevNodes &d, const DevPod *pods, const DevPodX *podx, int32_t e,
                            int32_t gp, int32_t xlo, int32_t xhi, int32_t n_ext, void *scratch, int32_t *out_node,
                            uint32_t *out_dev, PipeSync *sync, uint64_t *dbg, const int32_t *ext_idx, int32_t dlo,
                            hipStream_t s) {
  if (seq_mode(c) != 0) return hipErrorInvalidValue;
  const ExtScr x = ext_scr(scratch, n_ext, d.n);
  const size_t nn = (size_t)std::max(d.n, 1);
  const int32_t spin = ext_spin() > 0;
  if (!spin) hipLaunchKernelGGL(k_wait_ext_final, dim3(1), dim3(64), 0, s, sync, x.fl, gp + 1, e + 1);
  hipLaunchKernelGGL(k_ext_final<0>, dim3((d.n + EXT_FCHUNK - 1) / EXT_FCHUNK), dim3(EXT_THREADS), 0, s, c, d, pods,
                     podx, gp, xlo, xhi, x.tab, x.arrive + e, x.pk + (size_t)(e % EXT_RING) * nn,
                     x.pr + (size_t)(e % EXT_RING) * nn, out_node, out_dev, e, x.fl, sync, dbg, spin, ext_idx,
                     std::min(std::max(dlo, 0), e));
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
  const int sm = seq_launch_mode(c, d);
  const void *f = sm == 5   ? (const void *)k_seq<5>
                  : sm == 4 ? (const void *)k_seq<4>
                  : sm == 3 ? (const void *)k_seq<3>
                  : sm == 2 ? (const void *)k_seq<2>
                  : sm == 1 ? (const void *)k_seq<1>
                            : (const void *)k_seq<0>;
  int dev = 0, ncu = 0, per_cu = 0;
  if (hipError_t e = hipGetDevice(&dev)) return e;
  if (hipError_t e = hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev)) return e;
  if (hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, f, SEQ_THREADS, 0)) return e;
  if ((int64_t)per_cu * ncu < grid) return hipErrorCooperativeLaunchTooLarge;
  switch (sm) {
    case 5: hipLaunchKernelGGL(k_seq<5>, dim3(grid), dim3(SEQ_THREADS), 0, s, c, d, a); break;
    case 4: hipLaunchKernelGGL(k_seq<4>, dim3(grid), dim3(SEQ_THREADS), 0, s, c, d, a); break;
    case 3: hipLaunchKernelGGL(k_seq<3>, dim3(grid), dim3(SEQ_THREADS), 0, s, c, d, a); break;
    case 2: hipLaunchKernelGGL(k_seq<2>, dim3(grid), dim3(SEQ_THREADS), 0, s, c, d, a); break;
    case 1: hipLaunchKernelGGL(k_seq<1>, dim3(grid), dim3(SEQ_THREADS), 0, s, c, d, a); break;
    default: hipLaunchKernelGGL(k_seq<0>, dim3(grid), dim3(SEQ_THREADS), 0, s, c, d, a);
  }
  return hipGetLastError();
}

const char *seq_kernel_name(const DevCfg &c, const DevNodes &d) {
  static const char *names[6] = {"kh::k_seq<0>", "kh::k_seq<1>", "kh::k_seq<2>",
                                 "kh::k_seq<3>", "kh::k_seq<4>", "kh::k_seq<5>"};
  return names[seq_launch_mode(c, d)];
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
