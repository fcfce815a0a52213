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
//            scores) into registers; per block: feasible count and the raw
//            maxima over its feasible nodes, published as tagged granules
//   phase B  every block reads all blocks' granules (the data is the flag:
//            cdna_hip_programming.md Guideline 16 R2, no barrier), normalizes
//            its nodes' raw scores by the global maxima, and publishes its best
//            (total, lowest index) key the same way
//   commit   every block reads all keys: the winner w; the block owning w
//            runs the Reserve of every plugin on w (DeviceShare's device
//            choice, NodeNUMAResource's cpuset, Reservation's assume, the
//            Fit / LoadAware delta) before it evaluates its nodes for the
//            next pod.  Node w is only ever read by its owner block, so no
//            other block waits for the commit.
//
// Granule ring: 2 parities x G blocks x 4 words; a block overwrites parity
// q's granules only after it has read every block's granules of the next
// phase, which every block writes after it finished reading parity q.
#include <hip/hip_runtime.h>

#include "dev.hpp"
#include "kernels.h"

namespace kh {

constexpr int SEQ_THREADS = 256;
constexpr int SEQ_NPT = 8;  // nodes per thread held across the pod's phases (grid 256 x 256 x 8 >= 400k nodes)
constexpr uint32_t SEQ_SPIN_LIMIT = 1u << 24;

struct SeqArgs {
  const DevPod *pods;
  const DevPodX *podx;  // NULL: no pod has a device / extended request
  int32_t n_pods;
  int32_t npt;          // node slices per thread
  uint64_t *ga, *gb;    // granules [2][G][4]
  uint32_t *tmo;        // spin timeout word (0 = ok)
  int32_t *out_node;
  uint64_t *out_cpus;   // [n_pods][NW] (NULL: no NodeNUMAResource)
  uint32_t *out_dev;    // [n_pods][DT] (NULL: no DeviceShare)
  uint32_t ext;         // bit e: normalized plugin e scores (DeviceShare, NodeAffinity, TaintToleration)
  int32_t rs;           // the Reservation plugin scores (its PreScore nominates)
};

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

// One node for one pod: the total of the per-node plugins (-1: some Filter
// fails; with the Reservation plugin the ranking total of resv.hpp) and the
// raw normalized scores.  Every column is read (the parity evaluator's rows,
// like k_eval_full).
__device__ __noinline__ int32_t seq_eval(const DevCfg &c, const DevNodes &d, const DevPod &p, const DevPodX &x,
                                            int32_t i, bool rs, int32_t raw[KOORDHIP_NEXT_PLUGINS],
                                            uint8_t *status) {
  NV v{};
  const Need all = need_all(c);
  load_node(v, d, i, all, c);
  NumaRowR4 nr{};
  load_numa<true>(nr, d, i, all);
  int32_t t;
  bool nominated = false;
  if (c.resv) {
    load_resv(nr, d.rv, i);
    t = c.resv_cpus ? eval_total_resv<KOORDHIP_RESV_SLOTS, true>(p, v, nr, d.nu.cls, c)
                    : eval_total_resv<KOORDHIP_RESV_SLOTS, false>(p, v, nr, d.nu.cls, c);
    if (rs && (x.flags & KOORDHIP_PODX_DEVICE)) nominated = resv_nominate(p, nr, resv_matched(nr, p)) >= 0;
  } else if (numa_on(c)) {
    t = eval_total_numa<true>(p, v, nr, d.nu.cls, c);
  } else {
    t = eval_total(p, v, c);
  }
  const bool xf = !(c.filt & KOORDHIP_PLUGIN_FIT) || xfit_filter(d.dv, x, i, d.n);
  const bool df = !(c.filt & KOORDHIP_PLUGIN_DEVICESHARE) || dev_filter(d.dv, x, i);
  if (status) *status = (xf ? 0 : KOORDHIP_ST_XFIT_FAIL) | (df ? 0 : KOORDHIP_ST_DEVICE_FAIL);
  if (!xf || !df) t = -1;
  raw[0] = (c.score & KOORDHIP_PLUGIN_DEVICESHARE) ? dev_score(c, d.dv, x, i, nominated) : 0;
  raw[1] = (c.score & KOORDHIP_PLUGIN_AFFINITY_SCORE) ? static_raw(d.dv, 0, p.sclass, i, d.n) : 0;
  raw[2] = (c.score & KOORDHIP_PLUGIN_TAINT_SCORE) ? static_raw(d.dv, 1, p.sclass, i, d.n) : 0;
  return t;
}

// DefaultNormalizeScore(MaxNodeScore, reverse) of one raw score given the
// maximum over the feasible nodes
__device__ __forceinline__ int32_t norm_score(int32_t raw, int32_t mx, bool reverse) {
  if (mx == 0) return reverse ? 100 : raw;
  const int32_t s = (int32_t)((int64_t)100 * raw / mx);
  return reverse ? 100 - s : s;
}

__device__ __forceinline__ int32_t ext_total(const DevCfg &c, uint32_t ext, const int32_t raw[KOORDHIP_NEXT_PLUGINS],
                                             const int32_t mx[KOORDHIP_NEXT_PLUGINS]) {
  int32_t t = 0;
#pragma unroll
  for (int e = 0; e < KOORDHIP_NEXT_PLUGINS; e++)
    if ((ext >> e) & 1u) t += c.w_ext[e] * norm_score(raw[e], mx[e], e == 2);
  return t;
}

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
__device__ int32_t seq_commit(const DevCfg &c, const DevNodes &d, const DevPod &p, const DevPodX &x, int32_t w,
                              int32_t nf, bool rs, uint64_t *cpus_out, uint32_t *dev_out) {
  NumaRowR4 rv{};
  uint32_t mm = 0u;
  if (c.resv) {
    load_resv(rv, d.rv, w);
    mm = resv_matched(rv, p);
  }
  const bool prescore = rs && nf > 1;
  const bool nominated = prescore && c.resv && resv_nominate(p, rv, mm) >= 0;
  uint32_t slots[DT] = {0u, 0u, 0u};
  const bool dev = ((c.filt | c.score) & KOORDHIP_PLUGIN_DEVICESHARE) != 0;
  if (dev && !dev_reserve(c, d.dv, x, w, nominated, slots, false)) return KOORDHIP_RESERVE_FAILED;
  uint64_t m[NW] = {0, 0, 0, 0};
  if (numa_on(c) && numa_active(p, c)) {
    NumaRow r;
    load_numa_row(r, d, w);
    uint64_t pref[NW];
    resv_pref_cpus(rv, p, (c.resv && prescore) ? mm : 0u, pref);
    if (!numa_reserve<true>(d.nu.cls, r, p, m, pref)) return KOORDHIP_RESERVE_FAILED;
    store_numa_row(r, d, w);
  }
  if (dev) (void)dev_reserve(c, d.dv, x, w, nominated, slots, true);
  if (c.resv) {  // Reservation Reserve: assumePod into the nominated reservation
    resv_assume(rv, p, m);
    store_resv(rv, d.rv, w);
  }
  NV v;
  load_row(v, d, w);
  apply_delta(v, p, +1);
  store_row(v, d, w);
  if (x.xmask)
    for (int j = 0; j < KOORDHIP_NXRES; j++)
      if ((x.xmask >> j) & 1u) d.dv.xreq[(size_t)j * d.n + w] += x.xreq[j];
  if (cpus_out)
    for (int q = 0; q < NW; q++) cpus_out[q] = m[q];
  if (dev_out)
    for (int t = 0; t < DT; t++) dev_out[t] = slots[t];
  return 0;
}

__global__ __launch_bounds__(SEQ_THREADS) void k_seq(DevCfg c, DevNodes d, SeqArgs a) {
  __shared__ int32_t s_red[SEQ_THREADS / 64][8];
  __shared__ uint64_t s_key[SEQ_THREADS / 64];
  __shared__ int32_t s_nf, s_stop;
  __shared__ uint64_t s_best;
  const int t = threadIdx.x, lane = __lane_id(), wv = t >> 6;
  const int32_t G = gridDim.x, b = blockIdx.x;
  const uint32_t ext = a.ext;
  DevPodX none{};
  for (int q = 0; q < DT; q++) none.req[q][0] = none.req[q][1] = none.req[q][2] = q == 0 ? -1 : 0;
  for (int32_t p = 0; p < a.n_pods; p++) {
    const DevPod pod = a.pods[p];
    const DevPodX x = a.podx ? a.podx[p] : none;
    const uint32_t eA = 2u * (uint32_t)p + 1u, eB = 2u * (uint32_t)p + 2u;
    const int par = p & 1;
    // ---- phase A: this block's nodes
    int32_t tot[SEQ_NPT], raw[SEQ_NPT][KOORDHIP_NEXT_PLUGINS];
    int32_t nf = 0, mx[KOORDHIP_NEXT_PLUGINS] = {0, 0, 0};
#pragma unroll
    for (int k = 0; k < SEQ_NPT; k++) {
      tot[k] = -1;
      raw[k][0] = raw[k][1] = raw[k][2] = 0;
      const int32_t i = (k * G + b) * SEQ_THREADS + t;
      if (k < a.npt && i < d.n) {
        tot[k] = seq_eval(c, d, pod, x, i, a.rs != 0, raw[k], nullptr);
        if (tot[k] >= 0) {
          nf++;
#pragma unroll
          for (int e = 0; e < KOORDHIP_NEXT_PLUGINS; e++) mx[e] = max(mx[e], raw[k][e]);
        }
      }
    }
    int32_t gmx[KOORDHIP_NEXT_PLUGINS] = {0, 0, 0};
    int32_t nf_all = -1;
    if (ext) {
      // block reduce: feasible count, raw maxima
      int32_t v4[4] = {nf, mx[0], mx[1], mx[2]};
#pragma unroll
      for (int m = 32; m >= 1; m >>= 1) {
        v4[0] += __shfl_xor(v4[0], m);
#pragma unroll
        for (int e = 1; e < 4; e++) v4[e] = max(v4[e], __shfl_xor(v4[e], m));
      }
      if (lane == 0)
        for (int e = 0; e < 4; e++) s_red[wv][e] = v4[e];
      __syncthreads();
      if (t == 0) {
        int32_t r4[4] = {0, 0, 0, 0};
        for (int w = 0; w < SEQ_THREADS / 64; w++) {
          r4[0] += s_red[w][0];
          for (int e = 1; e < 4; e++) r4[e] = max(r4[e], s_red[w][e]);
        }
        uint64_t *g = a.ga + ((size_t)par * G + b) * 4;
        for (int e = 0; e < 4; e++) put_granule(g + e, eA, (uint32_t)r4[e]);
      }
      // every block's granules: the global maxima and feasible count
      int32_t r4[4] = {0, 0, 0, 0};
      bool ok = true;
      for (int32_t q = t; q < G; q += SEQ_THREADS) {
        uint32_t gv[4];
        ok &= sweep<4>(a.ga + ((size_t)par * G + q) * 4, eA, gv, a.tmo);
        r4[0] += (int32_t)gv[0];
        for (int e = 1; e < 4; e++) r4[e] = max(r4[e], (int32_t)gv[e]);
      }
      if (t == 0) s_stop = 0;
      __syncthreads();
      if (!ok) s_stop = 1;
#pragma unroll
      for (int m = 32; m >= 1; m >>= 1) {
        r4[0] += __shfl_xor(r4[0], m);
#pragma unroll
        for (int e = 1; e < 4; e++) r4[e] = max(r4[e], __shfl_xor(r4[e], m));
      }
      if (lane == 0)
        for (int e = 0; e < 4; e++) s_red[wv][4 + e] = r4[e];
      __syncthreads();
      if (s_stop) return;
      nf_all = 0;
      for (int w = 0; w < SEQ_THREADS / 64; w++) {
        nf_all += s_red[w][4];
        for (int e = 0; e < KOORDHIP_NEXT_PLUGINS; e++) gmx[e] = max(gmx[e], s_red[w][5 + e]);
      }
    }
    // ---- phase B: normalized totals, this block's best key
    uint64_t best = 0;
#pragma unroll
    for (int k = 0; k < SEQ_NPT; k++) {
      if (tot[k] < 0) continue;
      const int32_t i = (k * G + b) * SEQ_THREADS + t;
      const uint64_t key = make_key(tot[k] + ext_total(c, ext, raw[k], gmx), i);
      best = key > best ? key : best;
    }
    best = seq_wave_max(best);
    int32_t nfw = nf;
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) nfw += __shfl_xor(nfw, m);
    if (lane == 0) {
      s_key[wv] = best;
      s_red[wv][0] = nfw;
    }
    __syncthreads();
    if (t == 0) {
      uint64_t bk = 0;
      int32_t bn = 0;
      for (int w = 0; w < SEQ_THREADS / 64; w++) {
        bk = s_key[w] > bk ? s_key[w] : bk;
        bn += s_red[w][0];
      }
      uint64_t *g = a.gb + ((size_t)par * G + b) * 4;
      put_granule(g + 0, eB, (uint32_t)(bk >> 32));
      put_granule(g + 1, eB, (uint32_t)bk);
      put_granule(g + 2, eB, (uint32_t)bn);
    }
    // ---- every block's best: the winner
    uint64_t kb = 0;
    int32_t nb = 0;
    bool ok = true;
    for (int32_t q = t; q < G; q += SEQ_THREADS) {
      uint32_t gv[3];
      ok &= sweep<3>(a.gb + ((size_t)par * G + q) * 4, eB, gv, a.tmo);
      const uint64_t kk = ((uint64_t)gv[0] << 32) | gv[1];
      kb = kk > kb ? kk : kb;
      nb += (int32_t)gv[2];
    }
    if (t == 0) s_stop = 0;
    __syncthreads();
    if (!ok) s_stop = 1;
    kb = seq_wave_max(kb);
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) nb += __shfl_xor(nb, m);
    if (lane == 0) {
      s_key[wv] = kb;
      s_red[wv][1] = nb;
    }
    __syncthreads();
    if (s_stop) return;
    if (t == 0) {
      uint64_t bk = 0;
      int32_t nn = 0;
      for (int w = 0; w < SEQ_THREADS / 64; w++) {
        bk = s_key[w] > bk ? s_key[w] : bk;
        nn += s_red[w][1];
      }
      s_best = bk;
      s_nf = nn;
    }
    __syncthreads();
    const uint64_t win = s_best;
    const int32_t wn = win ? key_node(win) : -1;
    (void)nf_all;
    if (t == 0) {
      const bool mine = wn >= 0 ? ((wn / SEQ_THREADS) % G) == b : b == 0;
      if (mine) {
        int32_t res = KOORDHIP_UNSCHEDULABLE;
        uint64_t cp[NW] = {0, 0, 0, 0};
        uint32_t dv[DT] = {0u, 0u, 0u};
        if (wn >= 0) {
          const int32_t rc = seq_commit(c, d, pod, x, wn, s_nf, a.rs != 0, cp, dv);
          res = rc ? KOORDHIP_RESERVE_FAILED : wn;
          if (rc) {
            for (int q = 0; q < NW; q++) cp[q] = 0;
            for (int q = 0; q < DT; q++) dv[q] = 0u;
          }
        }
        a.out_node[p] = res;
        if (a.out_cpus)
          for (int q = 0; q < NW; q++) a.out_cpus[(size_t)p * NW + q] = cp[q];
        if (a.out_dev)
          for (int q = 0; q < DT; q++) a.out_dev[(size_t)p * DT + q] = dv[q];
      }
    }
    __syncthreads();  // the owner's commit before its next evaluation of w
  }
}

// ---- parity evaluation (koordhip_eval_ext): per (pod, node) the status bits,
// the raw score planes and the per-node total; then per pod the maxima and
// the top-k of the normalized totals
__global__ void k_seq_eval(DevCfg c, DevNodes d, const DevPod *__restrict__ pods, const DevPodX *__restrict__ podx,
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
  const int32_t t = seq_eval(c, d, pod, x, i, rs != 0, raw, &st);
  const size_t n = (size_t)d.n;
  int32_t *wk = work + (size_t)p * 4 * n;
  wk[i] = t;
  for (int e = 0; e < KOORDHIP_NEXT_PLUGINS; e++) wk[(size_t)(e + 1) * n + i] = raw[e];
  if (status) status[(size_t)p * n + i] |= st;
  if (scores) {
    int32_t *row = scores + (size_t)p * (KOORDHIP_NPLUGINS + KOORDHIP_NEXT_PLUGINS) * n;
    for (int e = 0; e < KOORDHIP_NEXT_PLUGINS; e++) row[(size_t)(KOORDHIP_NPLUGINS + e) * n + i] = raw[e];
  }
}

__global__ __launch_bounds__(256) void k_seq_topk(DevCfg c, int32_t n, const int32_t *__restrict__ work, int32_t k,
                                                  uint64_t *__restrict__ out) {
  __shared__ uint64_t s_k[4];
  __shared__ int32_t s_m[4][KOORDHIP_NEXT_PLUGINS];
  const int32_t p = blockIdx.x, t = threadIdx.x, lane = __lane_id(), wv = t >> 6;
  const int32_t *wk = work + (size_t)p * 4 * n;
  const uint32_t ext = ext_bits(c);
  int32_t mx[KOORDHIP_NEXT_PLUGINS] = {0, 0, 0};
  for (int32_t i = t; i < n; i += 256)
    if (wk[i] >= 0)
      for (int e = 0; e < KOORDHIP_NEXT_PLUGINS; e++) mx[e] = max(mx[e], wk[(size_t)(e + 1) * n + i]);
  for (int e = 0; e < KOORDHIP_NEXT_PLUGINS; e++) {
    for (int m = 32; m >= 1; m >>= 1) mx[e] = max(mx[e], __shfl_xor(mx[e], m));
    if (lane == 0) s_m[wv][e] = mx[e];
  }
  __syncthreads();
  for (int e = 0; e < KOORDHIP_NEXT_PLUGINS; e++) mx[e] = max(max(s_m[0][e], s_m[1][e]), max(s_m[2][e], s_m[3][e]));
  uint64_t last = ~0ull;
  for (int32_t j = 0; j < k; j++) {
    uint64_t best = 0;
    for (int32_t i = t; i < n; i += 256) {
      if (wk[i] < 0) continue;
      int32_t raw[KOORDHIP_NEXT_PLUGINS];
      for (int e = 0; e < KOORDHIP_NEXT_PLUGINS; e++) raw[e] = wk[(size_t)(e + 1) * n + i];
      const uint64_t key = make_key(wk[i] + ext_total(c, ext, raw, mx), i);
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
                      uint32_t *out_dev, int32_t rs, hipStream_t s) {
  if (n_pods <= 0) return hipSuccess;
  SeqArgs a{};
  a.pods = pods;
  a.podx = podx;
  a.n_pods = n_pods;
  a.npt = (d.n + grid * SEQ_THREADS - 1) / (grid * SEQ_THREADS);
  if (a.npt > SEQ_NPT) return hipErrorInvalidValue;
  a.ga = granules;
  a.gb = granules + (size_t)2 * grid * 4;
  a.tmo = tmo;
  a.out_node = out_node;
  a.out_cpus = out_cpus;
  a.out_dev = out_dev;
  a.ext = 0u;
  if (c.score & KOORDHIP_PLUGIN_DEVICESHARE) a.ext |= 1u;
  if (c.score & KOORDHIP_PLUGIN_AFFINITY_SCORE) a.ext |= 2u;
  if (c.score & KOORDHIP_PLUGIN_TAINT_SCORE) a.ext |= 4u;
  a.rs = rs;
  DevCfg cc = c;
  DevNodes dd = d;
  void *args[] = {&cc, &dd, &a};
  // every block must be resident (blocks read each other's granules): the
  // cooperative launch checks the grid against the occupancy
  return hipLaunchCooperativeKernel((const void *)k_seq, dim3(grid), dim3(SEQ_THREADS), args, 0, s);
}

hipError_t launch_seq_eval(const DevCfg &c, const DevNodes &d, const DevPod *pods, const DevPodX *podx, int32_t n_pods,
                           int32_t rs, uint8_t *status, int32_t *scores, int32_t *work, int32_t k, uint64_t *topk,
                           hipStream_t s) {
  if (n_pods <= 0 || d.n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_seq_eval, dim3((d.n + 255) / 256, n_pods), dim3(256), 0, s, c, d, pods, podx, n_pods, rs,
                     status, scores, work);
  if (topk && k > 0) hipLaunchKernelGGL(k_seq_topk, dim3(n_pods), dim3(256), 0, s, c, d.n, work, k, topk);
  return hipGetLastError();
}

}  // namespace kh
