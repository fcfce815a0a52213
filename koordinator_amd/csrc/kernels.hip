// kernels.hip -- CDNA4 (gfx950) kernels of libkoordhip.so.
//
//   k_prep_flags      LoadAware threshold masks + Fit over-commit bits, one
//                     thread per node (load_aware.go:123-254).
//   k_eval_full       parity mode: every plugin's Filter status and Score for
//                     every (pod, node), one thread per pair.
//   k_topk_partial    stream mode: each wave evaluates ONE pod over a chunk of
//                     nodes (lane = node, coalesced SoA loads) and keeps the
//                     exact top-K keys of its chunk as a sorted list spread
//                     over the 64 lanes (lane i = rank i); new keys enter by a
//                     ballot against the K-th key + rank insertion.
//   k_topk_merge      one workgroup per pod: exact top-K of the chunk lists
//                     (threshold prune by the max chunk tail, LDS rank sort).
//   k_resolve         one wave: the sequential greedy over the round's pods.
//                     Pod j's winner is max(first list entry not modified in
//                     this round, re-evaluation of the modified nodes); the
//                     winner's Reserve delta is applied to an LDS copy of the
//                     modified rows and written back at the end of the round.
#include <hip/hip_runtime.h>

#include "eval.hpp"
#include "kernels.h"

namespace kh {

// ---------------------------------------------------------------------------
// helpers

__device__ __forceinline__ uint64_t shfl_u64(uint64_t v, int src) {
  uint32_t lo = __shfl((uint32_t)v, src, 64);
  uint32_t hi = __shfl((uint32_t)(v >> 32), src, 64);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t shfl_up_u64(uint64_t v, int d) {
  uint32_t lo = __shfl_up((uint32_t)v, d, 64);
  uint32_t hi = __shfl_up((uint32_t)(v >> 32), d, 64);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int m) {
  uint32_t lo = __shfl_xor((uint32_t)v, m, 64);
  uint32_t hi = __shfl_xor((uint32_t)(v >> 32), m, 64);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    uint64_t o = shfl_xor_u64(v, m);
    v = o > v ? o : v;
  }
  return v;
}
__device__ __forceinline__ int lane_id() { return __lane_id(); }

// uniform-source lane read (v_readlane: SALU-visible, no LDS crossbar)
__device__ __forceinline__ uint64_t readlane_u64(uint64_t v, int src) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, src);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), src);
  return ((uint64_t)hi << 32) | lo;
}

template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ uint64_t dpp_u64(uint64_t v) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)v, CTRL, ROW_MASK, 0xf, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v >> 32), CTRL, ROW_MASK, 0xf, false);
  return ((uint64_t)hi << 32) | lo;
}

// Wave max of a u64 with DPP row shifts + row broadcasts (GFX9 DPP), result
// uniform.  Max is idempotent, so shifted prefix-max steps are a reduction.
__device__ __forceinline__ uint64_t wave_max_u64_dpp(uint64_t v) {
  uint64_t o;
  o = dpp_u64<0x111>(v); v = o > v ? o : v;        // row_shr:1
  o = dpp_u64<0x112>(v); v = o > v ? o : v;        // row_shr:2
  o = dpp_u64<0x114>(v); v = o > v ? o : v;        // row_shr:4
  o = dpp_u64<0x118>(v); v = o > v ? o : v;        // row_shr:8
  o = dpp_u64<0x142, 0xa>(v); v = o > v ? o : v;   // row_bcast:15
  o = dpp_u64<0x143, 0xc>(v); v = o > v ? o : v;   // row_bcast:31
  return readlane_u64(v, 63);
}

// ---------------------------------------------------------------------------
// k_prep_flags: load_aware.go:123-254 resolved per node, plus the Fit
// over-commit bits.  usage = int64(math.Round(float64(used)/float64(total)*100)).

__device__ __forceinline__ int64_t usage_percent(int64_t used, int64_t total) {
  double u = (double)used / (double)total;
  u = u * 100.0;
  return (int64_t)round(u);
}

__global__ void k_prep_flags(PrepIn in, DevNodes d, const int32_t *__restrict__ rows, int32_t m) {
  int32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= m) return;
  int32_t i = rows ? rows[t] : t;
  uint32_t f = in.la_flags[i];
  uint32_t o = 0;
  if (!(f & KOORDHIP_LA_HAS_METRIC) || (f & KOORDHIP_LA_FILTER_SKIP)) {
    o = NF_LA_OK_NONPROD | NF_LA_OK_PROD;
  } else {
    bool np = true;
    if (f & KOORDHIP_LA_FILTER_USAGE) {
      for (int r = 0; r < 2; r++) {
        int64_t thr = in.thr[r][i], total = in.total_m[r][i];
        if (thr == 0 || total == 0) continue;
        if (usage_percent(in.used_m[r][i], total) >= thr) np = false;
      }
    }
    bool p = np;
    if (f & KOORDHIP_LA_PROD_MODE) {
      p = true;
      if (f & KOORDHIP_LA_HAS_PODS_METRIC) {
        for (int r = 0; r < 2; r++) {
          int64_t thr = in.prod_thr[r][i], total = in.total_m[r][i];
          if (thr == 0 || total == 0) continue;
          if (usage_percent(in.prod_used_m[r][i], total) >= thr) p = false;
        }
      }
    }
    o = (np ? NF_LA_OK_NONPROD : 0u) | (p ? NF_LA_OK_PROD : 0u);
  }
  if (!(f & KOORDHIP_LA_HAS_METRIC) || (f & KOORDHIP_LA_SCORE_EXPIRED)) o |= NF_LA_SCORE_ZERO;
  if (d.requested[KOORDHIP_RES_CPU][i] > d.alloc[KOORDHIP_RES_CPU][i]) o |= NF_OVER_CPU;
  if (d.requested[KOORDHIP_RES_MEM][i] > d.alloc[KOORDHIP_RES_MEM][i]) o |= NF_OVER_MEM;
  if (d.requested[KOORDHIP_RES_EPH][i] > d.alloc[KOORDHIP_RES_EPH][i]) o |= NF_OVER_EPH;
  d.flags[i] = (uint8_t)o;
}

// ---------------------------------------------------------------------------
// k_eval_full: parity mode, no short-circuit.

__global__ void k_eval_full(DevCfg c, DevNodes d, const DevPod *__restrict__ pods, int32_t n_pods,
                            uint8_t *__restrict__ status, int32_t *__restrict__ scores) {
  int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  int32_t p = blockIdx.y;
  if (i >= d.n || p >= n_pods) return;
  const DevPod pod = pods[p];
  NV v{};
  const Need all = need_all(c);
  load_node(v, d, i, all, c);
  NumaRow nr{};
  load_numa(nr, d, i, all);
  if (status) {
    uint8_t b = 0;
    if ((c.filt & KOORDHIP_PLUGIN_FIT) && !fit_filter(pod, v)) b |= KOORDHIP_ST_FIT_FAIL;
    if ((c.filt & KOORDHIP_PLUGIN_LOADAWARE) && !la_filter(pod, v)) b |= KOORDHIP_ST_LA_FAIL;
    if ((c.filt & KOORDHIP_PLUGIN_NUMA) && !numa_filter(pod, nr, d.nu.cls)) b |= KOORDHIP_ST_NUMA_FAIL;
    status[(size_t)p * d.n + i] = b;
  }
  if (scores) {
    int32_t *row = scores + (size_t)p * KOORDHIP_NPLUGINS * d.n;
    row[i] = (c.score & KOORDHIP_PLUGIN_FIT) ? fit_score(pod, v, c) : 0;
    row[(size_t)d.n + i] = (c.score & KOORDHIP_PLUGIN_LOADAWARE) ? la_score(pod, v, c) : 0;
    row[2 * (size_t)d.n + i] = (c.score & KOORDHIP_PLUGIN_NUMA) ? numa_score(pod, v, nr, d.nu.cls, c) : 0;
  }
}

// ---------------------------------------------------------------------------
// k_topk_partial: one wave = one pod x one chunk of 64*R nodes.
//
// Lane l evaluates nodes c0 + r*64 + l (r < R): every column load is a
// coalesced 512-B (i64) or 256-B (i32) wave access, the R evaluations are
// independent so their loads overlap.  The chunk's exact top-k is then found
// without sorting: a radix select over the (small) total-score values with
// wave ballots finds the k-th largest score T; every key with score > T is
// taken and, for score == T, the lowest node indexes (r-major, lane-minor =
// index order) up to k.  Output: k keys per (pod, chunk), unsorted, 0-padded.

template <int R, bool NUMA>
__global__ __launch_bounds__(256) void k_topk_partial(DevCfg c, DevNodes d, const DevPod *__restrict__ pods,
                                                      int32_t n_pods, int32_t lo, int32_t hi, int32_t k,
                                                      int32_t score_bits, uint64_t *__restrict__ out) {
  const int lane = lane_id();
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: pod fields in SGPRs
  const int32_t p = blockIdx.y * (blockDim.x >> 6) + wave;
  if (p >= n_pods) return;  // wave-uniform
  const int32_t c0 = lo + blockIdx.x * (64 * R);
  const DevPod pod = pods[p];
  const Need need = pod_needs(pod, c);
  int32_t s[R];  // total score + 1, 0 = infeasible / past the end
#pragma unroll
  for (int r = 0; r < R; r++) {
    const int32_t i = c0 + r * 64 + lane;
    s[r] = 0;
    if (i < hi) {
      NV v;
      load_node(v, d, i, need, c);
      if constexpr (NUMA) {
        NumaRow nr;
        load_numa(nr, d, i, need);
        s[r] = eval_total_numa(pod, v, nr, d.nu.cls, c) + 1;
      } else {
        s[r] = eval_total(pod, v, c) + 1;
      }
    }
  }
  // k-th largest score value T (radix select, MSB first)
  int32_t feasible = 0;
#pragma unroll
  for (int r = 0; r < R; r++) feasible += __popcll(__ballot(s[r] > 0));
  int32_t T = 1;
  if (feasible > k) {
    T = 0;
    for (int b = score_bits - 1; b >= 0; b--) {
      const int32_t cand = T | (1 << b);
      int32_t cnt = 0;
#pragma unroll
      for (int r = 0; r < R; r++) cnt += __popcll(__ballot(s[r] >= cand));
      if (cnt >= k) T = cand;
    }
  }
  // selection in node-index order
  int32_t gt = 0;
#pragma unroll
  for (int r = 0; r < R; r++) gt += __popcll(__ballot(s[r] > T));
  int32_t eq_left = k - gt;  // ties at T still to take (lowest index first)
  int32_t base = 0;
  const size_t list = (size_t)p * gridDim.x + blockIdx.x;
  uint64_t *o = out + list * k;
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
#pragma unroll
  for (int r = 0; r < R; r++) {
    const bool eq = s[r] == T && s[r] > 0;
    const uint64_t me = __ballot(eq);
    const int32_t eq_rank = __popcll(me & lt);
    const bool sel = s[r] > T || (eq && eq_rank < eq_left);
    eq_left -= min(__popcll(me), max(eq_left, 0));
    const uint64_t ms = __ballot(sel);
    if (sel) {
      const int32_t i = c0 + r * 64 + lane;
      const uint64_t key = (((uint64_t)(uint32_t)s[r]) << 32) | (uint64_t)(0xFFFFFFFFu - (uint32_t)i);
      o[base + __popcll(ms & lt)] = key;
    }
    base += __popcll(ms);
  }
  for (int32_t j = base + lane; j < k; j += 64) o[j] = 0;
}

// ---------------------------------------------------------------------------
// k_topk_merge: per pod, the exact top-k of L lists of k keys.
//
// Input contract: list l holds the exact top-k of a contiguous node range,
// the ranges ascend with l, and inside a list keys of equal score appear in
// ascending node order (0 = empty slot).  Then the pod's k-th largest score
// S over the union of the lists is the global one; every key scoring > S is
// in some list (fewer than k of them), and the lowest-index ties at S are the
// first ties of the first lists.  So: radix-select S on the score (two 8-bit
// digits, LDS histograms), gather the > S keys, and take the ties list by
// list in order with a block prefix sum -- no comparison sort of candidates.

typedef __attribute__((address_space(1))) void gvoid_t;
typedef __attribute__((address_space(3))) void lvoid_t;

// Copy `bytes` (a multiple of 1 KiB) global -> LDS with LDS-DMA, 16 B per lane
// per instruction, all in flight at once; the caller waits (vmcnt) + barriers.
__device__ __forceinline__ void dma_to_lds(void *lds, const void *src, int32_t bytes, int lane) {
  const char *g = static_cast<const char *>(src);
  char *l = static_cast<char *>(lds);
  for (int32_t off = 0; off < bytes; off += 1024)
    __builtin_amdgcn_global_load_lds((gvoid_t *)(g + off + lane * 16), (lvoid_t *)(l + off), 16, 0, 0);
}

// The same across a whole workgroup (each wave takes every 4th KiB).
__device__ __forceinline__ void dma_to_lds_block(void *lds, const void *src, int32_t bytes) {
  const int lane = lane_id(), w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const char *g = static_cast<const char *>(src);
  char *l = static_cast<char *>(lds);
  for (int32_t off = w * 1024; off < bytes; off += nw * 1024)
    __builtin_amdgcn_global_load_lds((gvoid_t *)(g + off + lane * 16), (lvoid_t *)(l + off), 16, 0, 0);
}

constexpr int MERGE_THREADS = 256;
constexpr int RES_MAXP = 64;         // max pods per round = max k
constexpr int MERGE_STAGE = 8192;    // keys staged in LDS (64 KiB)
constexpr int MERGE_MAXL = 4096;     // lists per pod

__device__ __forceinline__ int32_t key_sc(uint64_t k) { return (int32_t)(k >> 32); }  // score + 1

// Block-wide exclusive prefix sum of one value per thread (wave shuffles + one
// LDS exchange of the 4 wave totals).
__device__ __forceinline__ int32_t block_exclusive_scan(int32_t v, int32_t *wsum, int32_t *total) {
  const int lane = lane_id(), w = threadIdx.x >> 6;
  int32_t x = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int32_t y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  int32_t base = 0, tot = 0;
  for (int q = 0; q < MERGE_THREADS / 64; q++) {
    if (q < w) base += wsum[q];
    tot += wsum[q];
  }
  __syncthreads();
  *total = tot;
  return base + x - v;
}

__global__ __launch_bounds__(MERGE_THREADS) void k_topk_merge(const uint64_t *__restrict__ in, int64_t pod_stride,
                                                              int64_t list_stride, int32_t L, int32_t k,
                                                              int32_t score_bits, uint64_t *__restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint64_t stage[MERGE_STAGE + 128];
  __shared__ int32_t tie_pre[MERGE_MAXL];
  __shared__ uint64_t gtbuf[RES_MAXP];
  __shared__ int32_t wsum[MERGE_THREADS / 64];
  __shared__ int32_t cnt_gt;
  const int t = threadIdx.x, lane = lane_id(), w = threadIdx.x >> 6;
  const int32_t p = blockIdx.x;
  const uint64_t *lists = in + (size_t)p * pod_stride;
  const int32_t total = L * k;
  const bool staged = total <= MERGE_STAGE && L <= MERGE_MAXL;
  auto gkey = [&](int32_t l, int32_t j) -> uint64_t { return lists[(size_t)l * list_stride + j]; };
  auto key = [&](int32_t l, int32_t j) -> uint64_t { return staged ? stage[l * k + j] : gkey(l, j); };
  // ---- 1. stage the lists in LDS
  if (t == 0) {

    cnt_gt = 0;
  }
  if (staged && list_stride == k) {
    // contiguous lists: one LDS-DMA burst (the buffer is padded to 1 KiB)
    dma_to_lds_block(stage, lists, (total * 8 + 1023) & ~1023);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else if (staged) {
    for (int32_t l = w; l < L; l += MERGE_THREADS / 64)
      for (int32_t j = lane; j < k; j += 64) stage[l * k + j] = gkey(l, j);
  }
  __syncthreads();
  // ---- 2. k-th largest score S: bitwise search on counts, keys' scores held
  //         in registers (up to MERGE_STAGE / MERGE_THREADS per thread)
  constexpr int PER = MERGE_STAGE / MERGE_THREADS;
  int32_t sc[PER];
  int32_t mine = 0;
#pragma unroll
  for (int i = 0; i < PER; i++) {
    const int32_t q = t + i * MERGE_THREADS;
    if (staged) {
      sc[i] = q < total ? key_sc(stage[q]) : 0;
    } else {
      sc[i] = 0;
    }
    mine += sc[i] > 0;
  }
  if (!staged)  // large inputs: count from global memory
    for (int32_t q = t; q < total; q += MERGE_THREADS) {
      const int32_t l = q / k;
      mine += key_sc(gkey(l, q - l * k)) > 0;
    }
  int32_t n_keys;
  (void)block_exclusive_scan(mine, wsum, &n_keys);
  int32_t S = 1;
  if (n_keys > k) {
    S = 0;
    for (int b = score_bits; b >= 0; b--) {
      const int32_t cand = S | (1 << b);
      int32_t c = 0;
      if (staged) {
#pragma unroll
        for (int i = 0; i < PER; i++) c += sc[i] >= cand;
      } else {
        for (int32_t q = t; q < total; q += MERGE_THREADS) {
          const int32_t l = q / k;
          c += key_sc(gkey(l, q - l * k)) >= cand;
        }
      }
      int32_t cnt;
      (void)block_exclusive_scan(c, wsum, &cnt);
      if (cnt >= k) S = cand;
    }
  }
  // ---- 3. keys above S (fewer than k) and tie counts per list
  const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  for (int32_t l = w; l < L; l += MERGE_THREADS / 64) {
    int32_t ties = 0;
    for (int32_t j0 = 0; j0 < k; j0 += 64) {
      const int32_t j = j0 + lane;
      const uint64_t x = j < k ? key(l, j) : 0;
      const int32_t sc = key_sc(x);
      if (sc > S) gtbuf[atomicAdd(&cnt_gt, 1)] = x;
      ties += __popcll(__ballot(sc == S));
    }
    if (lane == 0 && l < MERGE_MAXL) tie_pre[l] = ties;
  }
  __syncthreads();
  // per-list exclusive prefix of the tie counts (lists in node order)
  const int32_t per = (L + MERGE_THREADS - 1) / MERGE_THREADS;
  const int32_t l0 = min(L, t * per), l1 = min(L, l0 + per);
  int32_t seg = 0;
  for (int32_t l = l0; l < l1; l++) seg += tie_pre[l];
  int32_t all_ties;
  int32_t run = block_exclusive_scan(seg, wsum, &all_ties);
  for (int32_t l = l0; l < l1; l++) {
    const int32_t c = tie_pre[l];
    tie_pre[l] = run;
    run += c;
  }
  __syncthreads();
  // ---- 4. output: sorted keys above S, then the lowest-index ties
  const int32_t gt = cnt_gt;
  const int32_t need = k - gt;
  uint64_t *o = out + (size_t)p * k;
  for (int32_t j = t; j < gt; j += MERGE_THREADS) {
    const uint64_t x = gtbuf[j];
    int32_t rank = 0;
    for (int32_t q = 0; q < gt; q++) rank += gtbuf[q] > x;
    o[rank] = x;
  }
  for (int32_t l = w; l < L; l += MERGE_THREADS / 64) {
    int32_t base = tie_pre[l];
    if (base >= need) continue;  // wave-uniform
    for (int32_t j0 = 0; j0 < k; j0 += 64) {
      const int32_t j = j0 + lane;
      const uint64_t x = j < k ? key(l, j) : 0;
      const bool tie = key_sc(x) == S;
      const uint64_t tb = __ballot(tie);
      const int32_t pos = base + __popcll(tb & lt);
      if (tie && pos < need) o[gt + pos] = x;
      base += __popcll(tb);
    }
  }
  const int32_t filled = gt + min(need, all_ties);
  for (int32_t j = filled + t; j < k; j += MERGE_THREADS) o[j] = 0;
}

// ---------------------------------------------------------------------------
// k_resolve: sequential greedy over one round (one wave, 64 lanes).
//
// Exactness: within a round only the nodes committed by earlier pods of the
// round (set M, |M| <= j) differ from the snapshot the lists were built on.
// For pod j the best unmodified node is the first list entry not in M (its
// key is exact); the modified nodes are re-evaluated on their current rows.
// Because |M| < k the list always holds an unmodified entry unless it ran out
// of feasible nodes.  With monotone scoring (every enabled strategy is
// LeastAllocated-style: a commit can only lower a node's key) a modified node
// can only win if it ranks above that first entry, so the re-evaluation is
// skipped when no list prefix entry is modified.

__device__ __forceinline__ void copy_row(NV *dst, const NV *src, int lane) {
  constexpr int W = (int)(sizeof(NV) / 8);
  static_assert(sizeof(NV) % 8 == 0 && W <= 64, "NV must be a whole number of 8-byte words");
  if (lane < W) reinterpret_cast<uint64_t *>(dst)[lane] = reinterpret_cast<const uint64_t *>(src)[lane];
}

__device__ __forceinline__ uint64_t stamp() {
  uint64_t t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

constexpr int RES_PRE = 128;  // prefetched snapshot rows per round

template <bool NUMA>
__global__ __launch_bounds__(64) void k_resolve(DevCfg c, DevNodes d, const DevPod *__restrict__ pods,
                                                int32_t n_pods, int32_t k, const uint64_t *__restrict__ lists,
                                                int32_t monotone, int32_t *__restrict__ out_node,
                                                uint64_t *__restrict__ out_cpus, uint64_t *__restrict__ dbg) {
  // dbg (diagnostic builds only, KOORDHIP_STAMPS): s_memtime segment sums
  uint64_t t_entry = dbg ? stamp() : 0, t_a = 0, t_b = 0, t_c = 0, t_mark = 0, n_eval = 0, n_miss = 0;
  __shared__ __attribute__((aligned(16))) uint64_t lk[RES_MAXP * RES_MAXP];
  __shared__ __attribute__((aligned(16))) DevPod lp[RES_MAXP + 16];
  // Prefetched snapshot rows: slot t holds pod (t % n_pods)'s list entry at
  // position t / n_pods.  A round's winner is either a node already modified
  // in the round (kept in registers) or its pod's first unmodified list
  // entry, which is nearly always among the first few positions.
  __shared__ NV pre[RES_PRE];
  __shared__ int32_t pre_node[RES_PRE];
  extern __shared__ uint32_t modmap[];  // one bit per node: committed this round
  const int lane = lane_id();
  // LDS-DMA the round's lists and pod records (buffers are padded to 1 KiB)
  dma_to_lds(lk, lists, ((n_pods * k * 8) + 1023) & ~1023, lane);
  dma_to_lds(lp, pods, ((n_pods * (int32_t)sizeof(DevPod)) + 1023) & ~1023, lane);
  const int32_t words = (d.n + 31) >> 5;
  for (int32_t j = lane; j < words; j += 64) modmap[j] = 0;
  for (int32_t t = lane; t < RES_PRE; t += 64) {
    const int32_t j = t % n_pods, q = t / n_pods;
    int32_t nd = -1;
    if (q < k) {
      const uint64_t e = lists[(size_t)j * k + q];
      if (e != 0) nd = key_node(e);
    }
    if (nd >= 0) {
      NV v;
      load_row(v, d, nd);
      pre[t] = v;
    }
    pre_node[t] = nd;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const uint64_t t_pro = dbg ? stamp() : 0;
  // Lane r owns modified row r in registers (evaluated and committed in place).
  NV my{};
  NumaRow mynr{};  // ... and its NodeNUMAResource state (NUMA builds)
  int32_t my_node = -1;
  int32_t nm = 0;  // modified rows this round (wave-uniform)
  uint64_t e = lane < k ? lk[lane] : 0;
  bool mod = false;
  for (int32_t j = 0; j < n_pods; j++) {
    if (dbg) t_mark = stamp();
    const DevPod pod = lp[j];
    const uint64_t free_mask = __ballot(e != 0 && !mod);
    const int first = free_mask ? __builtin_ctzll(free_mask) : 64;
    const uint64_t cand = free_mask ? readlane_u64(e, first) : 0;
    uint64_t best = cand;
    const bool prefix_modified = __ballot(e != 0 && mod && lane < first) != 0;
    // Speculatively stage the row of `cand` (the winner whenever the winner is
    // not an already-modified node) into lane nm, the owner such a new row
    // gets; the LDS/global latency overlaps the re-evaluation below.
    int32_t staged = -1;
    if (cand != 0) {
      const int32_t cn = key_node(cand);
      const uint64_t pm0 = __ballot(pre_node[lane] == cn);
      const uint64_t pm1 = __ballot(pre_node[lane + 64] == cn);
      const int src = pm0 ? __builtin_ctzll(pm0) : (pm1 ? 64 + __builtin_ctzll(pm1) : -1);
      if (src >= 0) {
        if (lane == nm) my = pre[src];
      } else {
        n_miss++;
        if (lane == nm) load_row(my, d, cn);
      }
      if constexpr (NUMA) {
        if (lane == nm) load_numa_row(mynr, d, cn);
      }
      staged = cn;
    }
    if (dbg) {
      const uint64_t t = stamp();
      t_a += t - t_mark;
      t_mark = t;
    }
    // a required-policy cpuset pod's NUMA feasibility is not monotone in the
    // node's free CPUs (numa_spread_ok): re-evaluate the modified rows for it
    const bool nonmono = NUMA && is_cpuset(pod) && KOORDHIP_NUMA_REQUIRED(pod.numa_policy) != KOORDHIP_CPUBIND_NONE;
    if (nm > 0 && (!monotone || prefix_modified || nonmono)) {
      uint64_t key = 0;
      if constexpr (NUMA) {
        if (lane < nm) key = make_key(eval_total_numa(pod, my, mynr, d.nu.cls, c), my_node);
      } else {
        if (lane < nm) key = make_key(eval_total(pod, my, c), my_node);
      }
      key = wave_max_u64_dpp(key);
      best = key > best ? key : best;
      n_eval++;
    }
    if (dbg) {
      const uint64_t t = stamp();
      t_b += t - t_mark;
      t_mark = t;
    }
    uint64_t cpus[NW] = {0, 0, 0, 0};
    if (best == 0) {
      if (lane == 0) out_node[j] = KOORDHIP_UNSCHEDULABLE;
    } else {
      const int32_t w = key_node(best);
      const uint64_t hit = __ballot(lane < nm && my_node == w);
      // w is either a modified row (lane `hit`) or new this round, hence pod j's
      // first unmodified list entry, whose row lane nm already staged
      const int32_t r = hit ? __builtin_ctzll(hit) : nm;
      if (!hit && staged != w && lane == r) {  // unreachable by construction; kept for safety
        load_row(my, d, w);
        if constexpr (NUMA) load_numa_row(mynr, d, w);
      }
      bool ok = true;
      if constexpr (NUMA) {
        if (numa_on(c) && is_cpuset(pod)) {
          // NodeNUMAResource Reserve: every lane replays the accumulator on row r
          NumaRow br;
          br.cls = __builtin_amdgcn_readlane(mynr.cls, r);
          br.nflags = (uint32_t)__builtin_amdgcn_readlane((int)mynr.nflags, r);
          br.cnt = __builtin_amdgcn_readlane(mynr.cnt, r);
          for (int q = 0; q < NW; q++) {
            br.fr[q] = readlane_u64(mynr.fr[q], r);
            br.ep[q] = readlane_u64(mynr.ep[q], r);
            br.en[q] = readlane_u64(mynr.en[q], r);
          }
          ok = br.cls >= 0 && numa_allocate(d.nu.cls[br.cls], br, pod, cpus);
        }
      }
      if (!ok) {
        if (lane == 0) out_node[j] = KOORDHIP_RESERVE_FAILED;  // every Reserve is rolled back
      } else {
        if (lane == 0) out_node[j] = w;
        if (!hit) {
          nm++;
          if (lane == r) {
            my_node = w;
            modmap[w >> 5] |= 1u << (w & 31);
          }
        }
        if (lane == r) {
          apply_delta(my, pod, +1);
          if constexpr (NUMA) {
            if (numa_on(c) && is_cpuset(pod)) numa_apply(mynr, pod, cpus, +1);
          }
        }
      }
    }
    if (out_cpus && lane < NW)
      out_cpus[(size_t)j * NW + lane] = lane == 0 ? cpus[0] : (lane == 1 ? cpus[1] : (lane == 2 ? cpus[2] : cpus[3]));
    // next pod's list against the state after pod j's commit
    if (j + 1 < n_pods) {
      e = lane < k ? lk[(j + 1) * k + lane] : 0;
      mod = false;
      if (e != 0) {
        const int32_t nd = key_node(e);
        mod = (modmap[nd >> 5] >> (nd & 31)) & 1u;
      }
    }
    if (dbg) t_c += stamp() - t_mark;
  }
  if (lane < nm) {
    store_row(my, d, my_node);
    if constexpr (NUMA) store_numa_row(mynr, d, my_node);
  }
  if (dbg && lane == 0) {
    const uint64_t t_end = stamp();
    atomicAdd((unsigned long long *)&dbg[0], (unsigned long long)(t_pro - t_entry));
    atomicAdd((unsigned long long *)&dbg[1], (unsigned long long)t_a);
    atomicAdd((unsigned long long *)&dbg[2], (unsigned long long)t_b);
    atomicAdd((unsigned long long *)&dbg[3], (unsigned long long)t_c);
    atomicAdd((unsigned long long *)&dbg[4], (unsigned long long)(t_end - t_entry));
    atomicAdd((unsigned long long *)&dbg[5], (unsigned long long)n_eval);
    atomicAdd((unsigned long long *)&dbg[6], (unsigned long long)n_miss);
    atomicAdd((unsigned long long *)&dbg[7], (unsigned long long)n_pods);
  }
}

// ---------------------------------------------------------------------------
// single-pod commit / uncommit (Reserve / Unreserve from the host)

__global__ void k_commit(DevCfg c, DevNodes d, const DevPod *__restrict__ pod, int32_t node, int32_t sign,
                         uint64_t *__restrict__ cpus, int32_t *__restrict__ rc) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const DevPod p = *pod;
  *rc = 0;
  if (numa_on(c) && is_cpuset(p)) {
    NumaRow r;
    load_numa_row(r, d, node);
    uint64_t m[NW];
    if (sign > 0) {
      if (r.cls < 0 || !numa_allocate(d.nu.cls[r.cls], r, p, m)) {
        *rc = KOORDHIP_ERESERVE;  // Reserve fails: nothing is committed
        return;
      }
    } else {
      for (int w = 0; w < NW; w++) m[w] = cpus[w];
    }
    numa_apply(r, p, m, sign);
    store_numa_row(r, d, node);
    if (sign > 0)
      for (int w = 0; w < NW; w++) cpus[w] = m[w];
  } else if (sign > 0) {
    for (int w = 0; w < NW; w++) cpus[w] = 0;
  }
  NV v;
  load_row(v, d, node);
  apply_delta(v, p, sign);
  store_row(v, d, node);
}

// ---------------------------------------------------------------------------
// row scatter (koordhip_update_nodes)

template <typename T>
__global__ void k_scatter(T *__restrict__ dst, const T *__restrict__ src, const int32_t *__restrict__ idx, int32_t m) {
  int32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < m) dst[idx[t]] = src[t];
}

// ---------------------------------------------------------------------------
// host-side launch wrappers

template <typename T>
hipError_t launch_scatter(T *dst, const T *src, const int32_t *idx, int32_t m, hipStream_t s) {
  if (m <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_scatter<T>, dim3((m + 255) / 256), dim3(256), 0, s, dst, src, idx, m);
  return hipGetLastError();
}
template hipError_t launch_scatter<int64_t>(int64_t *, const int64_t *, const int32_t *, int32_t, hipStream_t);
template hipError_t launch_scatter<int32_t>(int32_t *, const int32_t *, const int32_t *, int32_t, hipStream_t);
template hipError_t launch_scatter<uint8_t>(uint8_t *, const uint8_t *, const int32_t *, int32_t, hipStream_t);

hipError_t launch_prep_flags(const PrepIn &in, const DevNodes &d, const int32_t *rows, int32_t m, hipStream_t s) {
  if (m <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_prep_flags, dim3((m + 255) / 256), dim3(256), 0, s, in, d, rows, m);
  return hipGetLastError();
}

hipError_t launch_eval_full(const DevCfg &c, const DevNodes &d, const DevPod *pods, int32_t n_pods,
                            uint8_t *status, int32_t *scores, hipStream_t s) {
  if (n_pods <= 0 || d.n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_eval_full, dim3((d.n + 255) / 256, n_pods), dim3(256), 0, s, c, d, pods, n_pods, status,
                     scores);
  return hipGetLastError();
}

hipError_t launch_topk_partial(int R, const DevCfg &c, const DevNodes &d, const DevPod *pods, int32_t n_pods,
                               int32_t lo, int32_t hi, int32_t nchunks, int32_t k, int32_t score_bits,
                               uint64_t *out, hipStream_t s) {
  dim3 grid(nchunks, (n_pods + 3) / 4);
  const bool numa = ((c.filt | c.score) & KOORDHIP_PLUGIN_NUMA) != 0;
#define KH_PARTIAL(RR, NN) \
  hipLaunchKernelGGL((k_topk_partial<RR, NN>), grid, dim3(256), 0, s, c, d, pods, n_pods, lo, hi, k, score_bits, out)
  if (numa) {
    switch (R) {
      case 1: KH_PARTIAL(1, true); break;
      case 2: KH_PARTIAL(2, true); break;
      default: KH_PARTIAL(4, true); break;
    }
  } else {
    switch (R) {
      case 1: KH_PARTIAL(1, false); break;
      case 2: KH_PARTIAL(2, false); break;
      case 4: KH_PARTIAL(4, false); break;
      default: KH_PARTIAL(8, false); break;
    }
  }
#undef KH_PARTIAL
  return hipGetLastError();
}

hipError_t launch_topk_merge(const uint64_t *in, int64_t pod_stride, int64_t list_stride, int32_t n_pods, int32_t L,
                             int32_t k, int32_t score_bits, uint64_t *out, hipStream_t s) {
  if (score_bits > 16 || L > MERGE_MAXL) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_topk_merge, dim3(n_pods), dim3(MERGE_THREADS), 0, s, in, pod_stride, list_stride, L, k,
                     score_bits, out);
  return hipGetLastError();
}

hipError_t launch_resolve(const DevCfg &c, const DevNodes &d, const DevPod *pods, int32_t n_pods, int32_t k,
                          const uint64_t *lists, int32_t monotone, int32_t *out_node, uint64_t *out_cpus,
                          uint64_t *dbg, hipStream_t s) {
  const size_t bitmap = (size_t)((d.n + 31) >> 5) * sizeof(uint32_t);
  if ((c.filt | c.score) & KOORDHIP_PLUGIN_NUMA)
    hipLaunchKernelGGL(k_resolve<true>, dim3(1), dim3(64), bitmap, s, c, d, pods, n_pods, k, lists, monotone, out_node,
                       out_cpus, dbg);
  else
    hipLaunchKernelGGL(k_resolve<false>, dim3(1), dim3(64), bitmap, s, c, d, pods, n_pods, k, lists, monotone,
                       out_node, out_cpus, dbg);
  return hipGetLastError();
}

hipError_t launch_commit(const DevCfg &c, const DevNodes &d, const DevPod *pod, int32_t node, int32_t sign,
                         uint64_t *cpus, int32_t *rc, hipStream_t s) {
  hipLaunchKernelGGL(k_commit, dim3(1), dim3(64), 0, s, c, d, pod, node, sign, cpus, rc);
  return hipGetLastError();
}

}  // namespace kh
