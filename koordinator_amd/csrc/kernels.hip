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

#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "eval.hpp"
#include "karg.hpp"
#include "kernels.h"
#include "pipe.hpp"
#include "rows.hpp"

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
__device__ __forceinline__ uint32_t wave_max_u32_dpp(uint32_t v) {
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false));  // row_shr:1
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false));  // row_shr:2
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false));  // row_shr:4
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false));  // row_shr:8
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false));  // row_bcast:15
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false));  // row_bcast:31
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

// Wave max of a u64 as two 32-bit DPP max reductions (v_max_u32 takes the DPP
// operand directly, a 64-bit compare-select does not): the high word first,
// then the low word among the lanes holding that high word.  Result uniform.
__device__ __forceinline__ uint64_t wave_max_u64_dpp(uint64_t v) {
  const uint32_t hi = (uint32_t)(v >> 32), lo = (uint32_t)v;
  const uint32_t mh = wave_max_u32_dpp(hi);
  const uint32_t ml = wave_max_u32_dpp(hi == mh ? lo : 0u);
  return ((uint64_t)mh << 32) | ml;
}


// Wave max of an i32 (same DPP pattern), result uniform.
__device__ __forceinline__ int32_t wave_max_i32_dpp(int32_t v) {
  v = max(v, __builtin_amdgcn_update_dpp(INT32_MIN, v, 0x111, 0xf, 0xf, false));  // row_shr:1
  v = max(v, __builtin_amdgcn_update_dpp(INT32_MIN, v, 0x112, 0xf, 0xf, false));  // row_shr:2
  v = max(v, __builtin_amdgcn_update_dpp(INT32_MIN, v, 0x114, 0xf, 0xf, false));  // row_shr:4
  v = max(v, __builtin_amdgcn_update_dpp(INT32_MIN, v, 0x118, 0xf, 0xf, false));  // row_shr:8
  v = max(v, __builtin_amdgcn_update_dpp(INT32_MIN, v, 0x142, 0xa, 0xf, false));  // row_bcast:15
  v = max(v, __builtin_amdgcn_update_dpp(INT32_MIN, v, 0x143, 0xc, 0xf, false));  // row_bcast:31
  return __builtin_amdgcn_readlane(v, 63);
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
  NumaRowR8 nr{};  // (every slot count: the sequential cycle's snapshots hold up to KOORDHIP_RESV_SLOTS_MAX)
  load_numa<true>(nr, d, i, all);
  int nmatch = 0;
  uint32_t mm = 0;
  uint64_t P[NW] = {0, 0, 0, 0};  // the nominated reservation's reserved CPUs (scoring.go:82 -> plugin.go:503-524)
  if (c.resv) {  // the cycle's Reservation restore: every plugin sees the restored node
    load_resv(nr, d.rv, i);
    nmatch = resv_restore(v, nr, pod, mm);
    resv_pref_cpus(nr, pod, (c.score & KOORDHIP_PLUGIN_RESERVATION) ? mm : 0u, P);
    // a topology-policy node's zone row shares the reserved CPUs' bytes: read it again
    if (c.zones && topo_policy(nr.nflags) != 0) load_zones(nr, d, i);
  }
  if (status) {
    uint8_t b = 0;
    if ((c.filt & KOORDHIP_PLUGIN_NODE_STATIC) && !((v.sa >> pod.sclass) & 1u)) b |= KOORDHIP_ST_STATIC_FAIL;
    if ((c.filt & KOORDHIP_PLUGIN_FIT) && !fit_filter(pod, v)) b |= KOORDHIP_ST_FIT_FAIL;
    if ((c.filt & KOORDHIP_PLUGIN_LOADAWARE) && !la_filter(pod, v)) b |= KOORDHIP_ST_LA_FAIL;
    if ((c.filt & KOORDHIP_PLUGIN_NUMA) &&
        (!numa_filter<true>(pod, nr, d.nu.cls) || (c.amp && !amp_filter_ok(pod, v, nr))))
      b |= KOORDHIP_ST_NUMA_FAIL;
    if ((c.filt & KOORDHIP_PLUGIN_RESERVATION) &&
        (nmatch > 0 ? !resv_filter(pod, v, nr, mm, nmatch) : (pod.flags & KOORDHIP_POD_RESV_AFFINITY) != 0))
      b |= KOORDHIP_ST_RESV_FAIL;
    status[(size_t)p * d.n + i] = b;
  }
  if (scores) {
    int32_t *row = scores + (size_t)p * KOORDHIP_NPLUGINS * d.n;
    row[i] = (c.score & KOORDHIP_PLUGIN_FIT) ? fit_score(pod, v, c) : 0;
    row[(size_t)d.n + i] = (c.score & KOORDHIP_PLUGIN_LOADAWARE) ? la_score(pod, v, c) : 0;
    row[2 * (size_t)d.n + i] =
        (c.score & KOORDHIP_PLUGIN_NUMA) ? numa_score<true>(pod, v, nr, d.nu.cls, c, false, P) : 0;
    row[3 * (size_t)d.n + i] = (c.score & KOORDHIP_PLUGIN_BALANCED) ? bal_score(pod, v) : 0;
  }
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
constexpr int RES_MAXP = 128;        // max k (list length per pod)
constexpr int RES_MAXP_ROUND = 64;   // max pods per round
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
                                                              int32_t score_bits, uint64_t *__restrict__ out,
                                                              PipeSync *sy, int32_t sel_par) {
  // dynamic LDS (merge_lds_bytes): the staged lists, padded to the 1 KiB
  // LDS-DMA granule, then one tie count per list -- a one-shard copy asks for
  // none, so it fits beside a co-running evaluation's workgroups
  extern __shared__ __attribute__((aligned(16))) char mlds[];
  __shared__ uint64_t gtbuf[RES_MAXP];
  __shared__ int32_t wsum[MERGE_THREADS / 64];
  __shared__ int32_t cnt_gt;
  const int t = threadIdx.x, lane = lane_id(), w = threadIdx.x >> 6;
  const int32_t p = blockIdx.x;
  const uint64_t *lists = in + (size_t)p * pod_stride;
  const int32_t total = L * k;
  const bool staged = total <= MERGE_STAGE && L <= MERGE_MAXL;
  uint64_t *stage = reinterpret_cast<uint64_t *>(mlds);
  int32_t *tie_pre = reinterpret_cast<int32_t *>(mlds + (staged ? ((total * 8 + 1023) & ~1023) : 0));
  auto gkey = [&](int32_t l, int32_t j) -> uint64_t { return lists[(size_t)l * list_stride + j]; };
  auto key = [&](int32_t l, int32_t j) -> uint64_t { return staged ? stage[l * k + j] : gkey(l, j); };
  uint64_t *o = out + (size_t)p * k;
  if (L == 1) {  // one shard: its list is already in the output form
    for (int32_t j = t; j < k; j += MERGE_THREADS) st_wt(&o[j], lists[j]);
    if (sy) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (t == 0) pipe_count_pod(sy, sel_par);
    }
    return;
  }
  // ---- 1. stage the lists in LDS
  if (t == 0) cnt_gt = 0;
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
  for (int32_t j = t; j < gt; j += MERGE_THREADS) {
    const uint64_t x = gtbuf[j];
    int32_t rank = 0;
    for (int32_t q = 0; q < gt; q++) rank += gtbuf[q] > x;
    st_wt(&o[rank], x);
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
      if (tie && pos < need) st_wt(&o[gt + pos], x);
      base += __popcll(tb);
    }
  }
  const int32_t filled = gt + min(need, all_ties);
  for (int32_t j = filled + t; j < k; j += MERGE_THREADS) st_wt(&o[j], (uint64_t)0);
  if (sy) {  // the pod's merged list is published: count it into the pipeline (no signal kernel)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) pipe_count_pod(sy, sel_par);
  }
}

// ---------------------------------------------------------------------------
// k_scan: one wave = one pod x one chunk of 64*R nodes of the shard [lo, hi).
//
// Lane l evaluates nodes c0 + 64r + l (r < R): every column read is a
// coalesced 512-B (f64) / 256-B (i32) wave access and the R evaluations are
// independent, so their loads overlap.  The result, score + 1 (0 =
// infeasible), goes to the pod's row of the score matrix S (u16, a coalesced
// 128-B store per r).  No selection here: k_select finds the pod's top-k from
// S afterwards with one LDS histogram, which costs far less than a per-chunk
// top-k list plus a merge of ~N/512 such lists.
//
// XCD-aware grid: workgroup b is dispatched to XCD b % 8, so the chunks are
// split into 8 contiguous ranges and XCD x only ever touches range x: each
// XCD's 4 MB L2 then holds its eighth of the node table (50k nodes: ~0.5 MB)
// and the 4 x (pods/4) re-reads of a row hit L2 instead of the MALL.

// SCAN_WPE1 / SCAN_WPE3: minimum waves per SIMD the compiler must fit the
// NodeNUMAResource / Reservation scans into (1 = no constraint).  The
// Reservation scan at 4 waves (<= 128 VGPRs, a few spilled dwords instead of
// 162 VGPRs at 3 waves): config 5 scan 175 -> 138 us, 150k -> 169k pods/s;
// the NUMA scan measured no different (config 3 is resolve-bound)
#ifndef SCAN_WPE1
#define SCAN_WPE1 1
#endif
#ifndef SCAN_WPE3
#define SCAN_WPE3 4
#endif
constexpr int32_t kScanPodFastNodes = 65536;

// NM: 0 = no NodeNUMAResource, 1 = NodeNUMAResource, 2 = ... with
// topology-policy nodes (the zone code is compiled only here), 3 = with the
// Reservation plugin (NUMA side rows carry the node's reservation), 4 = ...
// with several reservations per node (KOORDHIP_RESV_SLOTS slots per row), 5 =
// ... with reservations holding CPUs (the Score's preferred-CPU Allocate runs
// the accumulator: its registers cap these kernels at 2 waves per SIMD)
template <int R, int NM>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(NM == 5 ? 2 : (NM >= 3 ? SCAN_WPE3 : (NM == 1 ? SCAN_WPE1 : 1))))) void k_scan(DevCfg c, DevNodes d, const DevPod *__restrict__ pods, int32_t n_pods,
                                              int32_t lo, int32_t hi, int32_t nchunks, int32_t cpx, int32_t pfast,
                                              uint16_t *__restrict__ S, int64_t s_stride,
                                              uint16_t *__restrict__ Mx, int32_t m_stride) {
  const int32_t b = blockIdx.x;
  const int32_t xcd = b & 7, local = b >> 3;
  // pfast: a chunk's pod groups are consecutive blocks of its XCD, so they run
  // together and share the chunk's columns in L2.  The chunk-fastest order
  // sweeps the XCD's whole node range once per pod group: at 200k nodes that
  // range (~4 MB per XCD) overflows L2 and every pod group re-fetches it
  // (config 5 PMC: 126 -> 48 MB per launch, scan 136 -> 129 us)
  const int32_t npg = (n_pods + 3) >> 2;
  const int32_t chunk = pfast ? xcd * cpx + local / npg : xcd * cpx + local % cpx;
  const int32_t pg = pfast ? local - (local / npg) * npg : local / cpx;
  if (chunk >= nchunks) return;  // block-uniform
  const DevNumaClass *cls = d.nu.cls;
  if constexpr (NM != 0) {  // topology classes -> LDS (launch_scan sizes it when ncls <= NUMA_LDS_CLASSES)
    extern __shared__ uint4 scan_cls[];
    if (d.nu.ncls <= NUMA_LDS_CLASSES) {
      const uint4 *src = reinterpret_cast<const uint4 *>(d.nu.cls);
      for (int32_t x = threadIdx.x; x < d.nu.ncls * (int32_t)(sizeof(DevNumaClass) / 16); x += 256) scan_cls[x] = src[x];
      __syncthreads();
      cls = reinterpret_cast<const DevNumaClass *>(scan_cls);
    }
  }
  const int lane = lane_id();
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: pod fields in SGPRs
  const int32_t p = pg * 4 + wave;
  if (p >= n_pods) return;
  const int32_t c0 = lo + chunk * (64 * R);
  const DevPod pod = pods[p];
  const Need need = pod_needs(pod, c);
  uint16_t *row = S + (size_t)p * s_stride;
  // evaluate all R nodes first, store afterwards: the u16 stores may alias the
  // node columns as far as the compiler knows, and a store between two
  // evaluations would serialise their loads
  int32_t s[R];
  const bool full = c0 + 64 * R <= hi;  // wave-uniform
#pragma unroll
  for (int r = 0; r < R; r++) {
    const int32_t i = c0 + r * 64 + lane;
    s[r] = 0;
    if (full || i < hi) {
      NV v;
      load_node(v, d, i, need, c);
      if constexpr (NM >= 3) {
        side_row_t<NM> nr;
        load_numa<false>(nr, d, i, need);
        load_resv(nr, d.rv, i);
        s[r] = eval_total_resv<side_row_t<NM>::kSlots, NM == 5>(pod, v, nr, cls, c) + 1;
      } else if constexpr (NM != 0) {
        NumaRow nr;
        load_numa<NM == 2>(nr, d, i, need);
        s[r] = eval_total_numa<NM == 2>(pod, v, nr, cls, c) + 1;
      } else {
        s[r] = eval_total(pod, v, c) + 1;
      }
    }
  }
#pragma unroll
  for (int r = 0; r < R; r++) {
    const int32_t i = c0 + r * 64 + lane;
    if (full || i < hi) col(row, i - lo) = (uint16_t)s[r];
  }
  // the chunk's best value: k_select's lower bound for the pod's k-th score
  int32_t mx = s[0];
#pragma unroll
  for (int r = 1; r < R; r++) mx = max(mx, s[r]);
  mx = wave_max_i32_dpp(mx);
  if (lane == 0) Mx[(size_t)p * m_stride + chunk] = (uint16_t)mx;
}

// ---------------------------------------------------------------------------
// k_scan_nm: the node-major evaluation (the default).
//
// k_scan above gives every (pod, chunk) pair its own wave, so each of a
// round's P pods re-issues the loads of the same node columns: P x the
// column VMEM instructions, served by L1/L2, and the kernel is bound by that
// issue rate.  Here a wave owns one chunk of 64*R nodes, loads the columns
// the union of its pod group's needs ONCE into VGPRs (lane l: nodes
// c0 + 64r + l), and then loops over the group's pods with the pod record in
// SGPRs (a uniform scalar load per pod).  The output is the same score matrix
// S and chunk maxima Mx, so k_select / k_select_split are unchanged.
//
// A workgroup = 4 waves = 4 consecutive chunks x one pod group of `ppw` pods;
// the host sizes ppw so the grid still holds ~2 waves per SIMD (fewer pods per
// wave when the node table is small).  XCD-aware like k_scan: block b runs on
// XCD b % 8 and XCD x only touches the x-th eighth of the chunk quads.
//
// Semantics: a pod's evaluation must see exactly the side row its own needs
// would load (pod_needs: e.g. cls = -1 / amp = 1 / nflags = 0 when the pod's
// NodeNUMAResource work is skipped), so the union row is narrowed per pod by
// numa_view before the evaluation; NV fields outside a pod's needs are never
// read by its evaluation.
__device__ __forceinline__ uint32_t need_pack(const Need &n) {
  return (uint32_t)n.pods | (uint32_t)n.r_cpu << 1 | (uint32_t)n.r_mem << 2 | (uint32_t)n.eph << 3 |
         (uint32_t)n.bcpu << 4 | (uint32_t)n.bmem << 5 | (uint32_t)n.a_cpu << 6 | (uint32_t)n.a_mem << 7 |
         (uint32_t)n.nz_cpu << 8 | (uint32_t)n.nz_mem << 9 | (uint32_t)n.la << 10 | (uint32_t)n.la_nonprod << 11 |
         (uint32_t)n.la_prod << 12 | (uint32_t)n.numa << 13 | (uint32_t)n.numa_masks << 14 | (uint32_t)n.zones << 15 |
         (uint32_t)n.amp << 16 | (uint32_t)n.resv << 17 | (uint32_t)n.sa << 18;
}
__device__ __forceinline__ Need need_unpack(uint32_t b) {
  b = __builtin_amdgcn_readfirstlane(b);
  Need n{};
  n.pods = b & 1;
  n.r_cpu = (b >> 1) & 1;
  n.r_mem = (b >> 2) & 1;
  n.eph = (b >> 3) & 1;
  n.bcpu = (b >> 4) & 1;
  n.bmem = (b >> 5) & 1;
  n.a_cpu = (b >> 6) & 1;
  n.a_mem = (b >> 7) & 1;
  n.nz_cpu = (b >> 8) & 1;
  n.nz_mem = (b >> 9) & 1;
  n.la = (b >> 10) & 1;
  n.la_nonprod = (b >> 11) & 1;
  n.la_prod = (b >> 12) & 1;
  n.numa = (b >> 13) & 1;
  n.numa_masks = (b >> 14) & 1;
  n.zones = (b >> 15) & 1;
  n.amp = (b >> 16) & 1;
  n.resv = (b >> 17) & 1;
  n.sa = (b >> 18) & 1;
  return n;
}
// OR over the wave (DPP within rows, then the row broadcasts), result in every lane
__device__ __forceinline__ uint32_t wave_or_u32(uint32_t v) {
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);  // row_shr:2
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);  // row_shr:8
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

template <bool Z>
__device__ __forceinline__ void numa_view(NumaRow &r, const Need &n) {
  if (!n.numa) {
    r.cls = -1;
    r.nflags = 0;
    r.amp = 1.0;
    return;
  }
  if (!n.amp) r.amp = 1.0;
  if (!(n.numa_masks || (Z && n.zones))) r.nflags = 0;
}

template <int R, int NM>
__global__ __launch_bounds__(256) void k_scan_nm(DevCfg c, DevNodes d, const DevPod *__restrict__ pods, int32_t n_pods,
                                                 int32_t lo, int32_t hi, int32_t nchunks, int32_t cqx, int32_t ppw,
                                                 uint16_t *__restrict__ S, int64_t s_stride,
                                                 uint16_t *__restrict__ Mx, int32_t m_stride) {
  const int32_t b = blockIdx.x;
  const int32_t xcd = b & 7, local = b >> 3;
  const int32_t cq = xcd * cqx + local % cqx;
  const int32_t pg = local / cqx;
  if (cq * 4 >= nchunks) return;  // block-uniform
  const DevNumaClass *cls = d.nu.cls;
  if constexpr (NM != 0) {  // topology classes -> LDS (as k_scan)
    extern __shared__ uint4 scan_cls[];
    if (d.nu.ncls <= NUMA_LDS_CLASSES) {
      const uint4 *src = reinterpret_cast<const uint4 *>(d.nu.cls);
      for (int32_t x = threadIdx.x; x < d.nu.ncls * (int32_t)(sizeof(DevNumaClass) / 16); x += 256) scan_cls[x] = src[x];
      __syncthreads();
      cls = reinterpret_cast<const DevNumaClass *>(scan_cls);
    }
  }
  const int lane = lane_id();
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int32_t chunk = cq * 4 + wave;
  const int32_t p0 = pg * ppw, p1 = min(p0 + ppw, n_pods);
  if (chunk >= nchunks || p0 >= p1) return;  // wave-uniform, no barrier follows
  // the union of the group's needs: lane j evaluates pod p0 + j's needs (one
  // round of vector loads instead of a chain of dependent scalar loads), the
  // packed bits are OR-reduced across the wave
  uint32_t nb = 0;
  if (lane < p1 - p0) {
    // the whole record in six 16-B loads issued together (pod_needs reads its
    // fields under short-circuit conditions: field-wise loads would chain)
    const uint4 *q = reinterpret_cast<const uint4 *>(pods + p0 + lane);
    uint4 t[sizeof(DevPod) / 16];
#pragma unroll
    for (int k = 0; k < (int)(sizeof(DevPod) / 16); k++) t[k] = q[k];
    DevPod pl;
    __builtin_memcpy(&pl, t, sizeof(DevPod));
    nb = need_pack(pod_needs(pl, c));
  }
  const Need need = need_unpack(wave_or_u32(nb));
  const int32_t c0 = lo + chunk * (64 * R);
  NV v[R];
  side_row_t<NM> nr[R];
  bool in[R];
#pragma unroll
  for (int r = 0; r < R; r++) {
    const int32_t i = c0 + r * 64 + lane;
    in[r] = i < hi;
    const int32_t ii = in[r] ? i : hi - 1;  // out-of-range lanes evaluate a valid row, stored nowhere
    load_node(v[r], d, ii, need, c);
    if constexpr (NM >= 3) {
      load_numa<false>(nr[r], d, ii, need);
      load_resv(nr[r], d.rv, ii);
    } else if constexpr (NM != 0) {
      load_numa<NM == 2>(nr[r], d, ii, need);
    }
  }
  // pod records in SGPRs, the next one's scalar loads issued before this
  // pod's evaluation so their latency hides behind it
  DevPod nxt = pods[p0];
  for (int32_t p = p0; p < p1; p++) {
    const DevPod pod = nxt;
    nxt = pods[min(p + 1, p1 - 1)];
    uint16_t *row = S + (size_t)p * s_stride;
    int32_t s[R];
    if constexpr (NM != 0) {
      const Need pn = pod_needs(pod, c);
#pragma unroll
      for (int r = 0; r < R; r++) {
        side_row_t<NM> w = nr[r];
        numa_view<NM == 2>(w, pn);
        if constexpr (NM >= 3)
          s[r] = eval_total_resv(pod, v[r], w, cls, c) + 1;
        else
          s[r] = eval_total_numa<NM == 2>(pod, v[r], w, cls, c) + 1;
      }
    } else {
#pragma unroll
      for (int r = 0; r < R; r++) s[r] = eval_total(pod, v[r], c) + 1;
    }
    int32_t mx = 0;
#pragma unroll
    for (int r = 0; r < R; r++) {
      s[r] = in[r] ? s[r] : 0;
      if (in[r]) col(row, c0 + r * 64 + lane - lo) = (uint16_t)s[r];
      mx = max(mx, s[r]);
    }
    mx = wave_max_i32_dpp(mx);
    if (lane == 0) Mx[(size_t)p * m_stride + chunk] = (uint16_t)mx;
  }
}

// ---------------------------------------------------------------------------
// k_select: one workgroup per pod, the exact top-k of its score row.
//
// Keys order by (score desc, node asc), i.e. the reference's selectHost with
// the lowest-index tie rule.  A lower bound L <= S* comes first: the k-th
// largest of the pod's chunk maxima (k_scan), since k distinct chunks each
// hold a node scoring >= it -- with 128-node chunks L is close to S*.  Pass 1
// builds the histogram of the row's scores >= L in LDS (one bin per total-
// score value, <= 30002 bins; few atomics thanks to L); the k-th largest S*
// follows by a top-down cumulative count, and gt = #(score > S*) < k.  Pass 2
// walks the row in node order: scores > S* go to a small LDS buffer (rank
// sorted at the end), ties at S* are numbered by a block prefix sum so the
// lowest k - gt indexes are taken.  Fewer than k feasible nodes -> all of
// them (S* = the lowest feasible value).  Output: k keys, best first, 0-padded.

constexpr int SEL_THREADS = 1024;
constexpr int SEL_WAVES = SEL_THREADS / 64;

// inclusive block prefix sum of one value per thread (WAVES x 64 threads)
template <int WAVES>
__device__ __forceinline__ int32_t block_scan_incl(int32_t v, int32_t *wsum, int32_t *total) {
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
#pragma unroll
  for (int q = 0; q < WAVES; q++) {
    const int32_t s = wsum[q];
    base += q < w ? s : 0;
    tot += s;
  }
  __syncthreads();
  *total = tot;
  return base + x;
}
__device__ __forceinline__ int32_t sel_scan(int32_t v, int32_t *wsum, int32_t *total) {
  return block_scan_incl<SEL_WAVES>(v, wsum, total);
}

// Row layout: tiles of SEL_THREADS x SEL_PER nodes; thread t owns the
// contiguous nodes [tile + t * SEL_PER, +SEL_PER), read as SEL_ITER 16-B
// loads issued back to back (the row comes from HBM: latency, not bandwidth,
// bounds this kernel), so numbering per thread in thread order is node order.  The per-value tests only build bit masks (unrolled, register
// resident); the few values that pass them are handled in a rolled loop that
// re-reads them (L2 hits).  A one-tile row (<= 65536 nodes per shard) is
// loaded once and kept in registers for pass 2.
constexpr int SEL_ITER = 8;
constexpr int SEL_PER = SEL_ITER * 8;
constexpr int32_t SEL_TILE = SEL_THREADS * SEL_PER;

__device__ __forceinline__ int32_t sel_node(int32_t tile, int t, int h) {
  return tile * SEL_TILE + t * SEL_PER + h;
}

// IT 16-B loads of one thread's contiguous run of 8 * IT row values from i0
// (values past the row end read as 0 = infeasible)
template <int IT>
__device__ __forceinline__ void row_load(const uint16_t *row, int32_t m, int32_t i0, uint4 *q) {
#pragma unroll
  for (int j = 0; j < IT; j++) {
    const int32_t i = i0 + 8 * j;
    if (i + 8 <= m) {
      q[j] = *reinterpret_cast<const uint4 *>(row + i);
    } else {
      uint32_t w[4];
#pragma unroll
      for (int h = 0; h < 4; h++) {
        const uint32_t a = i + 2 * h < m ? row[i + 2 * h] : 0u, b = i + 2 * h + 1 < m ? row[i + 2 * h + 1] : 0u;
        w[h] = a | (b << 16);
      }
      q[j] = make_uint4(w[0], w[1], w[2], w[3]);
    }
  }
}
__device__ __forceinline__ void sel_load(const uint16_t *row, int32_t m, int32_t tile, int t, uint4 *q) {
  row_load<SEL_ITER>(row, m, sel_node(tile, t, 0), q);
}

// bit h of the result: value h of q satisfies (v >= x) [ge] or (v == x) [eq]
template <int IT = SEL_ITER>
__device__ __forceinline__ uint64_t sel_mask_ge(const uint4 *q, uint32_t x) {
  uint64_t m = 0;
#pragma unroll
  for (int j = 0; j < IT; j++) {
    const uint32_t w4[4] = {q[j].x, q[j].y, q[j].z, q[j].w};
#pragma unroll
    for (int h = 0; h < 4; h++) {
      m |= (uint64_t)((w4[h] & 0xFFFFu) >= x) << (8 * j + 2 * h);
      m |= (uint64_t)((w4[h] >> 16) >= x) << (8 * j + 2 * h + 1);
    }
  }
  return m;
}
template <int IT = SEL_ITER>
__device__ __forceinline__ uint64_t sel_mask_eq(const uint4 *q, uint32_t x) {
  uint64_t m = 0;
#pragma unroll
  for (int j = 0; j < IT; j++) {
    const uint32_t w4[4] = {q[j].x, q[j].y, q[j].z, q[j].w};
#pragma unroll
    for (int h = 0; h < 4; h++) {
      m |= (uint64_t)((w4[h] & 0xFFFFu) == x) << (8 * j + 2 * h);
      m |= (uint64_t)((w4[h] >> 16) == x) << (8 * j + 2 * h + 1);
    }
  }
  return m;
}

// Wave-level walk of a histogram from the top bin down to bin `floor`: the
// k-th largest value (0 if fewer than k values >= floor) and how many values
// lie strictly above it.  `count(v)` reads bin v; wave-uniform results.
// `words` (BPW bins per 32-bit word, the histogram's storage): windows of
// 256 words whose bins are all zero are skipped in one probe (4 words per
// lane + a ballot) -- the Reservation ranking totals put a few reservation
// nodes ~30k values above the rest, which one-bin-per-lane steps crossed in
// ~500 iterations.
template <int BPW = 1, typename F>
__device__ __forceinline__ void sel_walk(F count, int32_t nbins, int32_t floor, int32_t k, int32_t &thr, int32_t &gt,
                                         int32_t top0 = -1, const uint32_t *words = nullptr) {
  const int lane = lane_id();
  int32_t cum = 0;
  thr = 0;
  gt = 0;
  // top0: no value lies above it (the walk starts there instead of at the top bin)
  int32_t top = top0 >= 0 ? min(top0, nbins - 1) : nbins - 1;
  while (top >= floor && thr == 0) {
    int32_t stop = floor - 1;  // the fine walk below runs down to bin stop + 1
    if (words) {
      const int32_t w1 = top / BPW, w0 = w1 - 255;
      uint32_t any = 0;
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const int32_t wi = w0 + lane * 4 + u;
        if (wi >= 0 && wi <= w1) any |= words[wi];
      }
      if (__ballot(any != 0) == 0) {  // bins [w0 * BPW, top] are all empty
        top = w0 * BPW - 1;
        continue;
      }
      stop = max(stop, w0 * BPW - 1);
    }
    for (; top > stop && thr == 0; top -= 64) {
      const int32_t v = top - lane;
      const int32_t c = v >= floor ? count(v) : 0;
      if (__ballot(c != 0) == 0) continue;  // wave-uniform
      int32_t x = c;  // inclusive prefix over lanes = bins top, top-1, ...
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const int32_t y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
      }
      const uint64_t hit = __ballot(c != 0 && cum + x >= k);
      if (hit) {
        const int l = __builtin_ctzll(hit);
        thr = top - l;
        gt = cum + __shfl(x, l, 64) - __shfl(c, l, 64);
      } else {
        cum += __shfl(x, 63, 64);
      }
    }
  }
}

__global__ __launch_bounds__(SEL_THREADS) void k_select(const uint16_t *__restrict__ S, int64_t s_stride, int32_t lo,
                                                        int32_t m, int32_t k, int32_t nbins,
                                                        const uint16_t *__restrict__ Mx, int32_t m_stride,
                                                        int32_t nchunks, uint64_t *__restrict__ out,
                                                        uint64_t *__restrict__ dbg) {
  // dbg (diagnostic builds only, KOORDHIP_STAMPS): per-phase s_memtime sums of thread 0
  uint64_t ts[6] = {0, 0, 0, 0, 0, 0};
  if (dbg && threadIdx.x == 0) ts[0] = stamp();
  extern __shared__ uint32_t hist[];  // nbins score bins, then (nbins + 1) / 2 packed u16 chunk-max bins
  uint32_t *mhist = hist + nbins;
  __shared__ uint64_t gtbuf[RES_MAXP];
  __shared__ int32_t wsum[SEL_WAVES];
  __shared__ int32_t sh_thr, sh_gt, sh_cnt_gt;
  const int t = threadIdx.x, lane = lane_id();
  const int32_t p = blockIdx.x;
  const uint16_t *row = S + (size_t)p * s_stride;
  const int32_t ntiles = (m + SEL_TILE - 1) / SEL_TILE;
  // first tile in flight while the lower bound is computed
  uint4 q[SEL_ITER];
  sel_load(row, m, 0, t, q);
  const int32_t mwords = nchunks >= k ? (nbins + 1) >> 1 : 0;
  for (int32_t j = t; j < nbins + mwords; j += SEL_THREADS) hist[j] = 0;
  if (t == 0) sh_cnt_gt = 0;
  // ---- lower bound L: k-th largest chunk maximum (histogram of the chunk
  //      maxima, then one wave walks it top-down)
  uint32_t L = 1;
  if (mwords) {
    const uint16_t *mrow = Mx + (size_t)p * m_stride;
    __syncthreads();
    for (int32_t j = t; j < nchunks; j += SEL_THREADS) {
      const uint32_t v = mrow[j];
      if (v) atomicAdd(&mhist[v >> 1], 1u << (16 * (v & 1)));  // counts <= nchunks < 2^16
    }
    __syncthreads();
    if (t < 64) {
      int32_t thr, gt;
      sel_walk<2>([&](int32_t v) { return (int32_t)((mhist[v >> 1] >> (16 * (v & 1))) & 0xFFFFu); }, nbins, 1, k, thr,
                  gt, -1, mhist);
      if (lane == 0) sh_thr = thr;
    }
    __syncthreads();
    L = sh_thr > 1 ? (uint32_t)sh_thr : 1u;
  }
  __syncthreads();
  if (dbg && t == 0) ts[1] = stamp();
  // ---- pass 1: histogram of the scores >= L
  for (int32_t tile = 0; tile < ntiles; tile++) {
    if (tile > 0) sel_load(row, m, tile, t, q);
    uint64_t hit = sel_mask_ge(q, L);
    while (hit) {
      const int h = __builtin_ctzll(hit);
      hit &= hit - 1;
      atomicAdd(&hist[row[sel_node(tile, t, h)]], 1u);
    }
  }
  __syncthreads();
  if (dbg && t == 0) ts[2] = stamp();
  // ---- k-th largest value S*: wave 0 walks the bins top-down, 64 at a time
  if (t < 64) {
    int32_t thr, gt;
    sel_walk<1>([&](int32_t v) { return (int32_t)hist[v]; }, nbins, (int32_t)L, k, thr, gt, -1, hist);
    if (thr == 0) {  // fewer than k feasible (then L == 1): take every feasible node
      thr = 1;
      gt = 0;
      for (int32_t v = 2 + lane; v < nbins; v += 64) gt += (int32_t)hist[v];
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) gt += __shfl_xor(gt, off, 64);
    }
    if (lane == 0) {
      sh_thr = thr;
      sh_gt = gt;
    }
  }
  __syncthreads();
  if (dbg && t == 0) ts[3] = stamp();
  const uint32_t thr = (uint32_t)sh_thr;
  const int32_t gt = sh_gt, need = k - gt;
  uint64_t *o = out + (size_t)p * k;
  // ---- pass 2: scores > S* (fewer than k) and the lowest-index ties at S*
  int32_t ties = 0;  // ties numbered so far (block-uniform)
  for (int32_t tile = 0; tile < ntiles; tile++) {
    if (ntiles > 1) sel_load(row, m, tile, t, q);
    const uint64_t above = sel_mask_ge(q, thr + 1);
    uint64_t eq = sel_mask_eq(q, thr);
    for (uint64_t x = above; x;) {
      const int h = __builtin_ctzll(x);
      x &= x - 1;
      const int32_t i = sel_node(tile, t, h);
      const int32_t pos = atomicAdd(&sh_cnt_gt, 1);
      gtbuf[pos] = ((uint64_t)row[i] << 32) | (uint64_t)(0xFFFFFFFFu - (uint32_t)(lo + i));
    }
    const int32_t mine = __popcll(eq);
    int32_t total;
    int32_t pos = ties + sel_scan(mine, wsum, &total) - mine;
    while (eq && pos < need) {  // ties in node order: thread-major, then h
      const int h = __builtin_ctzll(eq);
      eq &= eq - 1;
      o[gt + pos] = ((uint64_t)thr << 32) | (uint64_t)(0xFFFFFFFFu - (uint32_t)(lo + sel_node(tile, t, h)));
      pos++;
    }
    ties += total;
    if (ties >= need && sh_cnt_gt >= gt) break;  // uniform: read after sel_scan's barriers, before any later add
    __syncthreads();
  }
  __syncthreads();
  if (dbg && t == 0) ts[4] = stamp();
  // ---- gt keys in descending order, then pad
  for (int32_t j = t; j < gt; j += SEL_THREADS) {
    const uint64_t x = gtbuf[j];
    int32_t rank = 0;
    for (int32_t q2 = 0; q2 < gt; q2++) rank += gtbuf[q2] > x;
    st_wt(&o[rank], x);
  }
  const int32_t filled = gt + min(need, ties);
  for (int32_t j = filled + t; j < k; j += SEL_THREADS) o[j] = 0;
  if (dbg && t == 0) {
    ts[5] = stamp();
    for (int q2 = 1; q2 < 6; q2++) atomicAdd((unsigned long long *)&dbg[8 + q2], (unsigned long long)(ts[q2] - ts[q2 - 1]));
    atomicAdd((unsigned long long *)&dbg[8], 1ull);
  }
  (void)lane;
}

// ---------------------------------------------------------------------------
// ---------------------------------------------------------------------------
// k_select_split: the same exact top-k with G workgroups per pod.
//
// One workgroup per pod (k_select) keeps 32 of 256 CUs busy at the default
// round size and its walk over a 100 KB row is latency-bound.  Here
// workgroup (g, p) owns slice g of pod p's row (whole tiles of SPL_TILE
// nodes, 16 per thread, two 16-B loads).  It derives the pod's lower bound L
// from the chunk maxima exactly like k_select, then the exact top-k by key of
// its slice restricted to scores >= L: every node of the pod's top-k scores
// >= S* >= L and has fewer than k better keys in its own slice, so the union
// of the slice lists holds the whole answer.  Each slice list is written
// sorted (best first; equal scores are then contiguous and in node order).
//
// Hand-off (cdna_hip_programming.md Guideline 16, counter form): plain list
// stores -> every wave's vmcnt(0) -> barrier -> lane 0 agent release + asm
// vmcnt(0) -> agent fetch_add on the pod's arrival counter.  The workgroup
// that draws G-1 resets the counter (zeroed once at allocation; the next
// launch is ordered by the kernel boundary), takes an agent acquire and
// merges: the k-th largest score S over the G lists (LDS histogram walk), the
// keys above S (fewer than k) rank-sorted, then the ties at S list by list
// (lists ascend in node range, a list's ties are contiguous and ascending).
// With `done`, it then publishes the pod's final list the same way and adds
// 1 to the pipeline's list counter -- what k_resolve waits on, so no signal
// kernel runs between the evaluation and the resolve.

constexpr int SPL_THREADS = 256;
constexpr int SPL_WAVES = SPL_THREADS / 64;
#ifndef SPL_ITER_N
#define SPL_ITER_N 4  // 32 values per thread per tile (16: config 4 select 22.7 -> 21.8 us, config 5 78.8 -> 76.9 us)
#endif
constexpr int SPL_ITER = SPL_ITER_N;
constexpr int SPL_PER = SPL_ITER * 8;
constexpr int32_t SPL_TILE = SPL_THREADS * SPL_PER;
constexpr int SPL_GMAX = 16;

struct SplHdr {  // start of k_select_split's dynamic LDS (all of its LDS: the base stays 16-B aligned)
  uint64_t lst[RES_MAXP];
  int32_t wsum[SPL_WAVES];
  int32_t thr, gt, cnt_gt, last, nties;
  int32_t hmax, smax, mmax;  // largest chunk maximum / slice value >= L / merged key value (walk starts)
  int32_t gtc[SPL_GMAX], tie[SPL_GMAX];
};
static_assert(SPL_GMAX == kSelGMax, "k_select_split group bound");
constexpr int32_t SPL_HDR = (int32_t)((sizeof(SplHdr) + 15) & ~(size_t)15);

// PK: the score histogram holds two u16 counts per word (ranking totals of the
// Reservation plugin span ~31k values: a u32 per bin plus the chunk-max
// histogram would not fit LDS, and without the chunk-max lower bound every
// feasible node of the slice is counted).  Slices stay below 65536 nodes.
template <bool PK>
__global__ __launch_bounds__(SPL_THREADS) void k_select_split(
    const uint16_t *__restrict__ S, int64_t s_stride, int32_t lo, int32_t m, int32_t k, int32_t nbins,
    const uint16_t *__restrict__ Mx, int32_t m_stride, int32_t nchunks, int32_t G, int32_t tiles_per,
    uint64_t *__restrict__ part, uint32_t *__restrict__ cnt, uint64_t *__restrict__ out, PipeSync *__restrict__ sy,
    int32_t sel_par, int32_t res_wait) {
  extern __shared__ __attribute__((aligned(16))) char spl_lds[];
  SplHdr &h = *reinterpret_cast<SplHdr *>(spl_lds);
  uint64_t *mk = reinterpret_cast<uint64_t *>(spl_lds + SPL_HDR);                    // merge: G x k keys
  uint32_t *hist = reinterpret_cast<uint32_t *>(spl_lds + SPL_HDR + (((size_t)G * k * 8 + 15) & ~(size_t)15));  // score bins
  const int32_t hwords = PK ? (nbins + 1) >> 1 : nbins;
  uint32_t *mhist = hist + hwords;                                                     // packed chunk-max bins
  auto hadd = [&](uint32_t v) {
    if constexpr (PK) {
      atomicAdd(&hist[v >> 1], 1u << (16 * (v & 1)));
    } else {
      atomicAdd(&hist[v], 1u);
    }
  };
  auto hget = [&](int32_t v) -> int32_t {
    if constexpr (PK) {
      return (int32_t)((hist[v >> 1] >> (16 * (v & 1))) & 0xFFFFu);
    } else {
      return (int32_t)hist[v];
    }
  };
  const int t = threadIdx.x, lane = lane_id();
  const int32_t g = blockIdx.x, p = blockIdx.y;
  const uint16_t *row = S + (size_t)p * s_stride;
  const int32_t ntiles = (m + SPL_TILE - 1) / SPL_TILE;
  const int32_t tb = min(ntiles, g * tiles_per), te = min(ntiles, tb + tiles_per);
  auto first = [&](int32_t tile) -> int32_t { return tile * SPL_TILE + t * SPL_PER; };
  uint4 q[SPL_ITER];
  if (tb < te) row_load<SPL_ITER>(row, m, first(tb), q);
  const int32_t mwords = nchunks >= k ? (nbins + 1) >> 1 : 0;
  {  // zero both histograms, 16 B per store (the launch rounds the LDS size up)
    uint4 *h4 = reinterpret_cast<uint4 *>(hist);
    const int32_t n4 = (hwords + mwords + 3) >> 2;
    for (int32_t j = t; j < n4; j += SPL_THREADS) h4[j] = make_uint4(0u, 0u, 0u, 0u);
  }
  if (t == 0) {
    h.cnt_gt = 0;
    h.hmax = 0;
    h.smax = 0;
  }
  // ---- lower bound L: the k-th largest chunk maximum of the whole row
  uint32_t L = 1;
  if (mwords) {
    const uint16_t *mrow = Mx + (size_t)p * m_stride;
    __syncthreads();
    uint32_t mx = 0;
    for (int32_t j = t; j < nchunks; j += SPL_THREADS) {
      const uint32_t v = mrow[j];
      if (v) atomicAdd(&mhist[v >> 1], 1u << (16 * (v & 1)));  // counts <= nchunks < 2^16
      mx = v > mx ? v : mx;
    }
    const int32_t wm = wave_max_i32_dpp((int32_t)mx);
    if (lane == 0 && wm > 0) atomicMax(&h.hmax, wm);
    __syncthreads();
    if (t < 64) {
      int32_t thr, gt;
      sel_walk<2>([&](int32_t v) { return (int32_t)((mhist[v >> 1] >> (16 * (v & 1))) & 0xFFFFu); }, nbins, 1, k, thr,
                  gt, h.hmax, mhist);
      if (lane == 0) h.thr = thr;
    }
    __syncthreads();
    L = h.thr > 1 ? (uint32_t)h.thr : 1u;
  }
  __syncthreads();
  // ---- pass 1: histogram of the slice's scores >= L
  uint32_t sx = 0;
  for (int32_t tile = tb; tile < te; tile++) {
    if (tile > tb) row_load<SPL_ITER>(row, m, first(tile), q);
    uint64_t hit = sel_mask_ge<SPL_ITER>(q, L);
    while (hit) {
      const int b = __builtin_ctzll(hit);
      hit &= hit - 1;
      const uint32_t v = row[first(tile) + b];
      hadd(v);
      sx = v > sx ? v : sx;
    }
  }
  {
    const int32_t wm = wave_max_i32_dpp((int32_t)sx);
    if (lane == 0 && wm > 0) atomicMax(&h.smax, wm);
  }
  __syncthreads();
  // ---- the slice's k-th largest value T (or L with all of its >= L values)
  if (t < 64) {
    int32_t thr, gt;
    const int32_t top = h.smax;
    sel_walk<PK ? 2 : 1>(hget, nbins, (int32_t)L, k, thr, gt, top, hist);
    if (thr == 0) {
      thr = (int32_t)L;
      gt = 0;
      for (int32_t v = thr + 1 + lane; v <= top && v < nbins; v += 64) gt += hget(v);
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) gt += __shfl_xor(gt, off, 64);
    }
    if (lane == 0) {
      h.thr = thr;
      h.gt = gt;
    }
  }
  __syncthreads();
  const uint32_t thr = (uint32_t)h.thr;
  const int32_t gt = h.gt, need = k - gt;
  // ---- pass 2: values > T (fewer than k) and the lowest-index ties at T
  int32_t ties = 0;
  for (int32_t tile = tb; tile < te; tile++) {
    if (te - tb > 1) row_load<SPL_ITER>(row, m, first(tile), q);
    const uint64_t above = sel_mask_ge<SPL_ITER>(q, thr + 1);
    uint64_t eq = sel_mask_eq<SPL_ITER>(q, thr);
    for (uint64_t x = above; x;) {
      const int b = __builtin_ctzll(x);
      x &= x - 1;
      const int32_t i = first(tile) + b;
      h.lst[atomicAdd(&h.cnt_gt, 1)] = ((uint64_t)row[i] << 32) | (uint64_t)(0xFFFFFFFFu - (uint32_t)(lo + i));
    }
    const int32_t mine = __popcll(eq);
    int32_t total;
    int32_t pos = ties + block_scan_incl<SPL_WAVES>(mine, h.wsum, &total) - mine;
    while (eq && pos < need) {  // ties in node order: thread-major, then b
      const int b = __builtin_ctzll(eq);
      eq &= eq - 1;
      h.lst[gt + pos] = ((uint64_t)thr << 32) | (uint64_t)(0xFFFFFFFFu - (uint32_t)(lo + first(tile) + b));
      pos++;
    }
    ties += total;
    if (ties >= need && h.cnt_gt >= gt) break;  // uniform: read after the scan's barriers, before any later add
    __syncthreads();
  }
  __syncthreads();
  // ---- the slice list, best first: values > T rank-sorted, then the ties
  const int32_t filled = gt + min(need, ties);
  uint64_t *dst = part + ((size_t)p * G + g) * k;
  for (int32_t j = t; j < k; j += SPL_THREADS) {
    if (j < gt) {
      const uint64_t x = h.lst[j];
      int32_t rank = 0;
      for (int32_t q2 = 0; q2 < gt; q2++) rank += h.lst[q2] > x;
      dst[rank] = x;
    } else {
      dst[j] = j < filled ? h.lst[j] : 0ull;
    }
  }
  // ---- publish; the pod's last workgroup merges
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t old = __hip_atomic_fetch_add(&cnt[p], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int32_t last = old + 1 == (uint32_t)G;
    if (last) {
      __hip_atomic_store(&cnt[p], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    h.last = last;
  }
  __syncthreads();
  if (!h.last) return;  // block-uniform
  const int32_t total = G * k;
  const uint64_t *src = part + (size_t)p * G * k;
  for (int32_t j = t; j < total; j += SPL_THREADS) mk[j] = src[j];
  for (int32_t j = t; j < hwords; j += SPL_THREADS) hist[j] = 0;
  if (t < SPL_GMAX) {
    h.gtc[t] = 0;
    h.tie[t] = 0;
  }
  if (t == 0) {
    h.cnt_gt = 0;
    h.mmax = 0;
  }
  __syncthreads();
  {
    int32_t mx = 0;
    for (int32_t j = t; j < total; j += SPL_THREADS) {
      const uint64_t x = mk[j];
      if (x) {
        hadd((uint32_t)key_sc(x));
        mx = max(mx, key_sc(x));
      }
    }
    const int32_t wm = wave_max_i32_dpp(mx);
    if (lane == 0 && wm > 0) atomicMax(&h.mmax, wm);
  }
  __syncthreads();
  if (t < 64) {
    int32_t sth, sgt;
    const int32_t top = h.mmax;
    sel_walk<PK ? 2 : 1>(hget, nbins, 1, k, sth, sgt, top, hist);
    if (sth == 0) {  // fewer than k keys in all: every one of them
      sth = 1;
      sgt = 0;
      for (int32_t v = 2 + lane; v <= top && v < nbins; v += 64) sgt += hget(v);
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) sgt += __shfl_xor(sgt, off, 64);
    }
    if (lane == 0) {
      h.thr = sth;
      h.gt = sgt;
    }
  }
  __syncthreads();
  const int32_t St = h.thr, mgt = h.gt, mneed = k - mgt;
  for (int32_t j = t; j < total; j += SPL_THREADS) {
    const uint64_t x = mk[j];
    const int32_t sc = key_sc(x), s = j / k;
    if (sc > St) {
      h.lst[atomicAdd(&h.cnt_gt, 1)] = x;
      atomicAdd(&h.gtc[s], 1);
    } else if (sc == St) {
      atomicAdd(&h.tie[s], 1);
    }
  }
  __syncthreads();
  if (t == 0) {  // ties before each list (exclusive prefix over the G lists)
    int32_t run = 0;
    for (int32_t s = 0; s < G; s++) {
      const int32_t c = h.tie[s];
      h.tie[s] = run;
      run += c;
    }
    h.nties = run;
  }
  __syncthreads();
  uint64_t *o = out + (size_t)p * k;
  for (int32_t j = t; j < mgt; j += SPL_THREADS) {
    const uint64_t x = h.lst[j];
    int32_t rank = 0;
    for (int32_t q2 = 0; q2 < mgt; q2++) rank += h.lst[q2] > x;
    st_wt(&o[rank], x);
  }
  for (int32_t j = t; j < total; j += SPL_THREADS) {
    const uint64_t x = mk[j];
    if (key_sc(x) != St) continue;
    const int32_t s = j / k;
    const int32_t pos = mgt + h.tie[s] + (j - s * k - h.gtc[s]);
    if (pos < k) st_wt(&o[pos], x);
  }
  for (int32_t j = mgt + min(mneed, h.nties) + t; j < k; j += SPL_THREADS) st_wt(&o[j], (uint64_t)0);
  if (sy) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) {
      pipe_count_pod(sy, sel_par);
      // the next scan on this stream may read the node columns only once the
      // resolve has written back round res_wait - 1: the launch ends no earlier
      // (replaces a k_wait_resolved launch between this kernel and the scan)
      if (res_wait > 0) (void)wait_at_least(&sy->res_round, res_wait, sy);
    }
  }
}

// ---------------------------------------------------------------------------
// k_eval_topk: evaluation AND the exact per-pod top-k in one launch, without
// a score matrix.
//
// Workgroup (p, s) evaluates pod p on slice s of the shard (256 x VT nodes:
// evaluation q of thread t takes node c0 + q * 256 + t, so every column read
// is a coalesced wave access, and all R evaluations of an iteration have their
// loads in flight together) and parks the values (total + 1, 0 = infeasible;
// 32 bits, so any ranking total fits) in LDS.  Thread t then takes the
// contiguous run [t * VT, t * VT + VT) back into registers -- node order is
// thread-major from here on -- and the workgroup finds the slice's k-th
// largest value T by an LDS radix select (11-bit digit histograms from the top
// digit down: one or two levels for ranking totals below 2^22).  Every node of
// the pod's top-k scores >= S* >= T and has fewer than k better keys in its
// slice, so the slice's own top-k -- its keys above T, then its lowest-index
// ties at T -- holds all of the pod's answer that lies in the slice.  The
// slice list is written in node order per part ([keys > T][ties at T]), with
// its length in pcnt[p][s].
//
// Hand-off (cdna_hip_programming.md Guideline 16): the list is stored
// write-through (sc1), every wave drains its stores, a barrier, then one lane
// adds to arrive[p] (agent scope) -- no release fence, i.e. no L2 write-back
// per workgroup.  The last slice of pod p to arrive takes one agent acquire,
// gathers the slice lists (slice order = node order, and inside a list the
// keys of one value are in node order, so equal values are in node order
// everywhere), radix-selects their k-th largest value S and writes the final
// list: the keys above S rank-sorted, then the lowest-index ties at S.  With
// `sy` it then counts the pod into the pipeline's list counter (release +
// counter add, like k_select_split), so the resolve needs no signal kernel.
constexpr int ETK_THREADS = 256;
constexpr int ETK_WAVES = ETK_THREADS / 64;
constexpr int ETK_MAX_SLICES = 256;   // one slice list per thread in the merge's offset scan
constexpr int ETK_MERGE_KEYS = 4096;  // candidates the merge stages in LDS (more: read from L2)
constexpr int ETK_DIGIT = 11;         // radix-select digit: 2048 bins, 8 per thread
constexpr int ETK_BINS = 1 << ETK_DIGIT;

struct EtkHdr {
  uint64_t gtk[RES_MAXP];             // merge: the keys above S (fewer than k)
  int32_t off[ETK_MAX_SLICES + 1];    // merge: first candidate of each slice list
  uint32_t hist[ETK_BINS];            // radix-select digit histogram
  int32_t wsum[ETK_WAVES];            // block scans
  int32_t rmax[ETK_WAVES], rcnt[ETK_WAVES];
  int32_t cnt_gt, last, sel_b, sel_above;
};
constexpr int32_t ETK_HDR = (int32_t)((sizeof(EtkHdr) + 15) & ~(size_t)15);

// block max of v and sum of c, one barrier
__device__ __forceinline__ void etk_maxsum(uint32_t v, int32_t c, EtkHdr &h, uint32_t *mx, int32_t *sum) {
  v = (uint32_t)wave_max_u32_dpp(v);
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) c += __shfl_xor(c, m, 64);
  if (lane_id() == 0) {
    h.rmax[threadIdx.x >> 6] = (int32_t)v;
    h.rcnt[threadIdx.x >> 6] = c;
  }
  __syncthreads();
  uint32_t m = 0;
  int32_t s = 0;
#pragma unroll
  for (int w = 0; w < ETK_WAVES; w++) {
    m = max(m, (uint32_t)h.rmax[w]);
    s += h.rcnt[w];
  }
  *mx = m;
  *sum = s;
}

// The k-th largest T of the block's values (every thread passes its values
// through `each`, which calls its argument once per value) and gt = how many
// values exceed T; T = 1 and gt = #values > 1 when at most k are nonzero.
// top: the largest value; nnz: the nonzero count.  Radix select, one 11-bit
// digit per level from the top: histogram of the digit among the values that
// match the digits fixed so far, then the bucket where the count from the top
// reaches k (thread t owns bins [2040 - 8t, 2048 - 8t): a block prefix over
// threads is a count from the top).
template <typename F>
__device__ __forceinline__ uint32_t etk_kth(F each, uint32_t top, int32_t nnz, int32_t k, EtkHdr &h, int32_t *gt_out) {
  const int t = threadIdx.x;
  if (nnz <= k || top <= 1) {
    int32_t g = 0;
    each([&](uint32_t v) { g += v > 1u; });
    uint32_t dummy;
    int32_t tot;
    etk_maxsum(0u, g, h, &dummy, &tot);
    *gt_out = tot;
    return 1u;
  }
  const int hb = 31 - __builtin_clz(top);
  int shift = max(0, hb + 1 - ETK_DIGIT);
  int fixed = 32;       // bits >= fixed are fixed to prefix's
  uint32_t prefix = 0;
  int32_t above = 0;    // values above every bucket range examined (they exceed T)
  for (;;) {
    uint4 *h4 = reinterpret_cast<uint4 *>(h.hist);
    for (int x = t; x < ETK_BINS / 4; x += ETK_THREADS) h4[x] = make_uint4(0u, 0u, 0u, 0u);
    __syncthreads();
    each([&](uint32_t v) {
      if (v != 0u && (fixed >= 32 || (v >> fixed) == (prefix >> fixed)))
        atomicAdd(&h.hist[(v >> shift) & (ETK_BINS - 1)], 1u);
    });
    __syncthreads();
    const int b0 = ETK_BINS - 8 * (t + 1);  // this thread's 8 bins, from the top
    uint32_t c[8];
    int32_t mine = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      c[j] = h.hist[b0 + 7 - j];
      mine += (int32_t)c[j];
    }
    int32_t total;
    const int32_t incl = block_scan_incl<ETK_WAVES>(mine, h.wsum, &total);
    const int32_t before = above + incl - mine;  // values in the digit buckets above this thread's
    if (before < k && before + mine >= k) {      // exactly one thread
      int32_t run = before;
#pragma unroll
      for (int j = 0; j < 8; j++) {
        if (run + (int32_t)c[j] >= k) {
          h.sel_b = b0 + 7 - j;
          h.sel_above = run;
          break;
        }
        run += (int32_t)c[j];
      }
    }
    __syncthreads();
    const uint32_t b = (uint32_t)h.sel_b;
    above = h.sel_above;
    prefix |= b << shift;
    if (shift == 0) break;
    fixed = shift;
    shift = max(0, shift - ETK_DIGIT);
    __syncthreads();  // h.sel_* / hist reused by the next level
  }
  *gt_out = above;
  return prefix;
}

// G: pods per workgroup -- one load of a node's columns serves G evaluations
// (the evaluation phase is bound by the column loads' latency); the slice
// selections then run pod after pod, and the workgroup merges every pod whose
// last slice it was.
// (karg.hpp) k_eval_topk re-reads DevCfg / DevNodes per evaluation; 0: keep the by-value copies
#ifndef ETK_KARG
#define ETK_KARG 1
#endif

// compile-time A/B knobs (make variant): the NUMA / Reservation builds' waves
// per SIMD and evaluations in flight per thread
#ifndef ETK_WPE3
#define ETK_WPE3 4
#endif
#ifndef ETK_R3
#define ETK_R3 4
#endif
template <int NM, int VT, int R, int G>
__global__ __launch_bounds__(ETK_THREADS) __attribute__((amdgpu_waves_per_eu(NM == 5 ? 2 : (NM >= 3 ? ETK_WPE3 : 1)))) void k_eval_topk(
    DevCfg c_arg, DevNodes d_arg, const DevPod *__restrict__ pods, int32_t n_pods, int32_t lo, int32_t hi,
    int32_t nslices, int32_t spx, int32_t k, uint64_t *part, int32_t *pcnt, uint32_t *arrive,
    uint64_t *__restrict__ out, PipeSync *__restrict__ sy, int32_t sel_par, int32_t res_wait, int32_t stage_cap,
    uint64_t *dbg) {
  static_assert(VT % 4 == 0 && VT % R == 0, "slice shape");
  const DevCfg &c = c_arg;
  const DevNodes &d = d_arg;
  constexpr int32_t SL = ETK_THREADS * VT;
  // slice values (G rows), or (merge) up to stage_cap candidate keys: what the launch sized
  const int32_t VBYTES = (G * SL * 4 > stage_cap * 8) ? G * SL * 4 : stage_cap * 8;
  extern __shared__ __attribute__((aligned(16))) char etk_lds[];
  EtkHdr &h = *reinterpret_cast<EtkHdr *>(etk_lds);
  uint32_t *vals = reinterpret_cast<uint32_t *>(etk_lds + ETK_HDR);  // slice values, then merge candidates
  uint64_t *mk = reinterpret_cast<uint64_t *>(etk_lds + ETK_HDR);
  // dbg (KOORDHIP_STAMPS): per-phase s_memtime sums of thread 0 at dbg[40..47]
  uint64_t ts[4] = {0, 0, 0, 0};
  // XCD-aware: block b runs on XCD b % 8, which owns slices [xcd * spx, ...):
  // a slice's pods are consecutive blocks of one XCD and share its columns in L2
  const int32_t b = blockIdx.x, xcd = b & 7, local = b >> 3;
  const int32_t npg = (n_pods + G - 1) / G;
  const int32_t p0 = (local % npg) * G;
  const int32_t s = xcd * spx + local / npg;
  if (s >= nslices) return;  // block-uniform
  const int ng = min(G, n_pods - p0);
  const int t = threadIdx.x;
  if (dbg && t == 0) ts[0] = stamp();
  const DevNumaClass *cls = d.nu.cls;
  if constexpr (NM != 0) {  // topology classes -> LDS (launch_eval_topk sizes it when ncls <= NUMA_LDS_CLASSES)
    if (d.nu.ncls <= NUMA_LDS_CLASSES) {
      uint4 *dst = reinterpret_cast<uint4 *>(etk_lds + ETK_HDR + VBYTES);
      const uint4 *src = reinterpret_cast<const uint4 *>(d.nu.cls);
      for (int32_t x = t; x < d.nu.ncls * (int32_t)(sizeof(DevNumaClass) / 16); x += ETK_THREADS) dst[x] = src[x];
      __syncthreads();
      cls = reinterpret_cast<const DevNumaClass *>(dst);
    }
  }
  DevPod gpod[G];
  Need need{};
#pragma unroll
  for (int g = 0; g < G; g++) {
    gpod[g] = pods[p0 + (g < ng ? g : 0)];
    if (g == 0) need = pod_needs(gpod[g], c);
    else need_or(need, pod_needs(gpod[g], c));
  }
  const int32_t c0 = lo + s * SL;
  // ---- evaluate: R nodes in flight per thread, each row evaluated for the G
  //      pods, values parked in LDS (pod g's at vals[g * SL ...])
  uint32_t vmax[G];
  int32_t vnz[G];
#pragma unroll
  for (int g = 0; g < G; g++) vmax[g] = 0u, vnz[g] = 0;
#pragma unroll 1
  for (int q0 = 0; q0 < VT; q0 += R) {
    // (karg.hpp) re-read per R evaluations, outside the divergent node guard
    const DevCfg &cq = ETK_KARG ? kernarg_fresh<DevCfg>(0) : c_arg;
    const DevNodes &dq = ETK_KARG ? kernarg_fresh<DevNodes>(KARG_NODES) : d_arg;
    uint32_t sv[R][G];
#pragma unroll
    for (int r = 0; r < R; r++) {
      const int32_t i = c0 + (q0 + r) * ETK_THREADS + t;
#pragma unroll
      for (int g = 0; g < G; g++) sv[r][g] = 0u;
      if (i < hi) {
        const DevCfg &c = cq;
        const DevNodes &d = dq;
        NV v;
        load_node(v, d, i, need, c);
        if constexpr (NM >= 3) {
          side_row_t<NM> nr;
          load_numa<false>(nr, d, i, need);
          load_resv(nr, d.rv, i);
#pragma unroll
          for (int g = 0; g < G; g++)
            sv[r][g] = (uint32_t)(eval_total_resv<side_row_t<NM>::kSlots, NM == 5>(gpod[g], v, nr, cls, c) + 1);
        } else if constexpr (NM != 0) {
          NumaRow nr;
          load_numa<NM == 2>(nr, d, i, need);
#pragma unroll
          for (int g = 0; g < G; g++) sv[r][g] = (uint32_t)(eval_total_numa<NM == 2>(gpod[g], v, nr, cls, c) + 1);
        } else {
#pragma unroll
          for (int g = 0; g < G; g++) sv[r][g] = (uint32_t)(eval_total(gpod[g], v, c) + 1);
        }
      }
    }
#pragma unroll
    for (int r = 0; r < R; r++)
#pragma unroll
      for (int g = 0; g < G; g++) {
        vals[g * SL + (q0 + r) * ETK_THREADS + t] = sv[r][g];
        vmax[g] = max(vmax[g], sv[r][g]);
        vnz[g] += sv[r][g] != 0u;
      }
  }
  uint32_t lastmask = 0;  // (thread 0) pods whose last slice this workgroup is
#pragma unroll 1
  for (int g = 0; g < ng; g++) {
  const int32_t p = p0 + g;
  uint32_t top;
  int32_t nnz;
  etk_maxsum(vmax[g], vnz[g], h, &top, &nnz);  // (its barrier also publishes vals)
  if (dbg && t == 0 && g == 0) ts[1] = stamp();
  uint32_t v[VT];
  {
    const uint4 *src = reinterpret_cast<const uint4 *>(vals + g * SL + t * VT);
#pragma unroll
    for (int q = 0; q < VT / 4; q++) {
      const uint4 x = src[q];
      v[4 * q] = x.x;
      v[4 * q + 1] = x.y;
      v[4 * q + 2] = x.z;
      v[4 * q + 3] = x.w;
    }
  }
  int32_t gt;
  const uint32_t T = etk_kth(
      [&](auto f) {
#pragma unroll
        for (int q = 0; q < VT; q++) f(v[q]);
      },
      top, nnz, k, h, &gt);
  // the slice list: its keys above T, then its first k - gt ties at T, each
  // part in node order (one block scan of packed per-thread counts)
  int32_t ngt = 0, nt = 0;
#pragma unroll
  for (int q = 0; q < VT; q++) {
    ngt += v[q] > T;
    nt += v[q] == T;
  }
  int32_t packed_total;
  const int32_t pre = block_scan_incl<ETK_WAVES>((ngt << 16) | nt, h.wsum, &packed_total) - ((ngt << 16) | nt);
  const int32_t all_ties = packed_total & 0xFFFF;
  const int32_t tie_budget = k - gt;
  uint64_t *dst = part + ((size_t)p * nslices + s) * k;
  {
    int32_t pg = pre >> 16, pt = pre & 0xFFFF;
#pragma unroll
    for (int q = 0; q < VT; q++) {
      const uint64_t key = ((uint64_t)v[q] << 32) | (uint64_t)(0xFFFFFFFFu - (uint32_t)(c0 + t * VT + q));
      if (v[q] > T) {
        __hip_atomic_store(dst + pg, key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // sc1
        pg++;
      } else if (v[q] == T) {
        if (pt < tie_budget) __hip_atomic_store(dst + gt + pt, key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        pt++;
      }
    }
  }
  const int32_t emitted = gt + min(tie_budget, all_ties);
  if (t == 0) __hip_atomic_store(pcnt + (size_t)p * nslices + s, emitted, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }  // pods g
  if (dbg && t == 0) ts[2] = stamp();
  // ---- publish (Guideline 16 R1: every wave drains its sc1 stores, barrier,
  //      one relaxed agent-scope counter add per pod); a pod's last slice merges
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0) {
    for (int g = 0; g < ng; g++) {
      const uint32_t old = __hip_atomic_fetch_add(&arrive[p0 + g], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (old + 1 == (uint32_t)nslices) {
        __hip_atomic_store(&arrive[p0 + g], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        lastmask |= 1u << g;
      }
    }
    if (lastmask) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    h.last = (int32_t)lastmask;
  }
  __syncthreads();
  if (dbg && t == 0) {
    ts[3] = stamp();
    for (int q = 1; q < 4; q++) atomicAdd((unsigned long long *)&dbg[40 + q], (unsigned long long)(ts[q] - ts[q - 1]));
    atomicAdd((unsigned long long *)&dbg[40], 1ull);
  }
  lastmask = (uint32_t)h.last;
  if (!lastmask) return;  // block-uniform
#pragma unroll 1
  for (int g = 0; g < ng; g++) {
  if (!((lastmask >> g) & 1u)) continue;  // block-uniform
  const int32_t p = p0 + g;
  __syncthreads();  // the previous merge's LDS reads are done
  if (t == 0) h.cnt_gt = 0;
  // ---- merge: offsets of the slice lists (one per thread), then the candidates
  const int32_t ns = t < nslices ? pcnt[(size_t)p * nslices + t] : 0;
  int32_t total;
  const int32_t o0 = block_scan_incl<ETK_WAVES>(ns, h.wsum, &total) - ns;
  if (t < nslices) h.off[t] = o0;
  if (t == 0) h.off[nslices] = total;
  __syncthreads();
  const bool staged = total <= stage_cap;
  const uint64_t *src = part + (size_t)p * nslices * k;
  auto gkey = [&](int32_t x) -> uint64_t {  // candidate x (flattened slice order) from L2
    int32_t a = 0, z = nslices;               // largest slice a with off[a] <= x
    while (z - a > 1) {
      const int32_t m = (a + z) >> 1;
      if (h.off[m] <= x) a = m; else z = m;
    }
    return src[(size_t)a * k + (x - h.off[a])];
  };
  // thread t owns the flattened run [x0, x1): node order is thread-major
  const int32_t per = (total + ETK_THREADS - 1) / ETK_THREADS;
  const int32_t x0 = min(total, t * per), x1 = min(total, x0 + per);
  if (staged)
    for (int32_t x = x0; x < x1; x++) mk[x] = gkey(x);
  auto key = [&](int32_t x) -> uint64_t { return staged ? mk[x] : gkey(x); };
  uint32_t mtop = 0;
  for (int32_t x = x0; x < x1; x++) mtop = max(mtop, (uint32_t)(key(x) >> 32));
  uint32_t mmax;
  int32_t dummy;
  etk_maxsum(mtop, 0, h, &mmax, &dummy);
  int32_t mgt;
  const uint32_t S = etk_kth(
      [&](auto f) {
        for (int32_t x = x0; x < x1; x++) f((uint32_t)(key(x) >> 32));
      },
      mmax, total, k, h, &mgt);
  // keys above S (fewer than k) rank-sorted; ties at S in flattened order
  int32_t myt = 0;
  for (int32_t x = x0; x < x1; x++) {
    const uint64_t kk = key(x);
    const uint32_t sc = (uint32_t)(kk >> 32);
    if (sc > S) h.gtk[atomicAdd(&h.cnt_gt, 1)] = kk;
    myt += sc == S;
  }
  int32_t mties;
  const int32_t tpos0 = block_scan_incl<ETK_WAVES>(myt, h.wsum, &mties) - myt;  // (its barriers order the gtk adds)
  const int32_t mneed = k - mgt;
  uint64_t *o = out + (size_t)p * k;
  for (int32_t j = t; j < mgt; j += ETK_THREADS) {
    const uint64_t x = h.gtk[j];
    int32_t rank = 0;
    for (int32_t q = 0; q < mgt; q++) rank += h.gtk[q] > x;
    st_wt(&o[rank], x);
  }
  {
    int32_t pos = tpos0;
    for (int32_t x = x0; x < x1 && pos < mneed; x++) {
      const uint64_t kk = key(x);
      if ((uint32_t)(kk >> 32) == S) st_wt(&o[mgt + pos++], kk);
    }
  }
  for (int32_t j = mgt + min(mneed, mties) + t; j < k; j += ETK_THREADS) st_wt(&o[j], (uint64_t)0);
  if (dbg && t == 0) {
    atomicAdd((unsigned long long *)&dbg[44], (unsigned long long)(stamp() - ts[3]));
    atomicAdd((unsigned long long *)&dbg[45], 1ull);
    atomicAdd((unsigned long long *)&dbg[46], (unsigned long long)total);
  }
  if (sy) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) pipe_count_pod(sy, sel_par);
  }
  }  // merged pods g
  if (sy && res_wait > 0 && t == 0) (void)wait_at_least(&sy->res_round, res_wait, sy);
}

// ---------------------------------------------------------------------------
// k_resolve: the sequential greedy over the staged stream -- one persistent
// workgroup, rounds of n_pods <= 64 pods, lag-1 pipelined with the evaluation
// of the next round.
//
// Round r's lists (k >= 2 x round size keys per pod, best first: the exact
// top-k of the scanned nodes) were computed by k_scan / k_select WHILE round
// r-1 was resolved: they are exact for every node except M' = the nodes round
// r-1 committed to, whose columns k_scan may have read half-updated.  A
// Reserve only raises the columns a key depends on and every enabled score is
// non-increasing in them (a "monotone" configuration), so such a stale key is
// an upper bound of the node's current key.
//
// X = M' u M (M = the nodes committed in THIS round) is the set of nodes whose
// list keys may be stale.  Pod l's winner is the best of
//   c  = its first list entry outside X: exact, and it bounds every node
//        outside X, listed or not (the list is sorted; |X| < k keeps a full
//        list from running out of entries outside X);
//   the current keys of the X nodes (M' rows and M rows are in LDS).
// With monotone scores only the X entries ranked above c can beat c.
//
// Prologue (all waves, every pod at once): walk each list from the top while
// its entries are M' nodes (evaluated on their current M' rows), up to the
// first entry outside M' -- that walk is the pod's decision if no earlier pod
// of the round commits to a node it walked (its "examined" set E).  The
// winner's row is staged (list-head prefetch, M' row, or one HBM load).
// Loop (wave 0, s_setprio 3): pod l takes its staged decision unless E meets
// M (one LDS gather of E against the M bitmap + a ballot) or the pod is
// non-monotone / a cpuset pod; those take the general path (c, then every M
// and M' row evaluated, one row per lane).  The Reserve delta is applied lane
// per row word.  M is written back at the end of the round and becomes the
// next round's M'.

// Wave 0 runs the sequential loop with a lot of state in registers: 8 waves
// (4 for NUMA builds) keep 256 (512) VGPRs available to it.
template <int NM>
constexpr int res_threads() { return NM ? 256 : 512; }
// waves 1 .. RES_LOADERS load the next round while wave 0 resolves this one
// (the rest build key tables): three of eight, one of four (seven of eight
// measured no faster with the chained decisions, r05o)
template <int NM>
constexpr int res_loaders() { return res_threads<NM>() >= 512 ? 3 : 1; }

constexpr int RES_PRE = 128;    // prefetched rows of list heads (RES_PRE / round size per pod)
constexpr int RES_HASH = 256;   // node -> M' slot (open addressing)
constexpr int RES_WE = 8;       // list entries the prologue walks per pod
constexpr int RES_CHAIN_PASSES = 3;  // passes of chained decisions per round
constexpr int RES_LDS_MAX = 160 * 1024 - 3 * 1024;  // dynamic LDS cap (static LDS: M' nodes, hashes, flags)

// An NV row as 8-byte words (the lane-parallel Reserve): words 0-4 a[], 5-9
// r[], 10-11 nz, 12-13 la_a, 14-15 la_u, 16-17 la_up (f64), 18 = a_pods |
// npods << 32, 19 = flags.
constexpr int RES_WORDS = 20;
static_assert(sizeof(NV) == RES_WORDS * 8, "NV row = 20 words");
static_assert(offsetof(NV, r) == 40 && offsetof(NV, nz_cpu) == 80 && offsetof(NV, la_u_cpu) == 112 &&
                  offsetof(NV, la_up_cpu) == 128 && offsetof(NV, a_pods) == 144 && offsetof(NV, npods) == 148 &&
                  offsetof(NV, flags) == 152,
              "NV word layout");

// M rows carry a stale over-commit part of `flags` (the lane-wise Reserve
// only adds the deltas): every read of such a row for an evaluation or a
// write-back goes through here.
__device__ __forceinline__ NV slot_row(const NV &src) {
  NV v = src;
  uint32_t f = v.flags & ~(uint32_t)(NF_OVER_CPU | NF_OVER_MEM | NF_OVER_EPH);
  if (v.r[KOORDHIP_RES_CPU] > v.a[KOORDHIP_RES_CPU]) f |= NF_OVER_CPU;
  if (v.r[KOORDHIP_RES_MEM] > v.a[KOORDHIP_RES_MEM]) f |= NF_OVER_MEM;
  if (v.r[KOORDHIP_RES_EPH] > v.a[KOORDHIP_RES_EPH]) f |= NF_OVER_EPH;
  v.flags = f;
  return v;
}

struct ResLds {  // byte offsets into the dynamic LDS of k_resolve
  int32_t dep;  // per pod: the earlier pods whose staged commits its chained decision assumed (u64 masks)
  int32_t lists, pods, prev_rows, prev_numa, cur_rows, cur_numa, hash_node, hash_slot, pre_rows, pre_numa, pre_node,
      dec_key, dec_n, dec_src, dec_e, dec_c, moved, mhash, gbits, kpre, ktab, ready, classes, modmap, total;
  int32_t kwide;  // key-table entries are u32 (ranking totals above 16 bits), else u16
  // second copies of the per-round inputs, filled by waves 1.. while wave 0
  // resolves the previous round (overlap = 0: every round loads serially)
  int32_t overlap, lists2, pods2, pre_rows2, pre_numa2, pre_node2;
};

__host__ __device__ inline int32_t res_align(int32_t x) { return (x + 15) & ~15; }

// chain: room for the chained decisions' dependency masks (the plain and NUMA
// builds; the Reservation builds are never monotone, and their rows need the LDS)
__host__ __device__ inline ResLds res_lds(int32_t n_pods_max, int32_t kp, int32_t n_nodes, int32_t nrow,
                                          bool overlap = false, bool tables = true, int32_t lag = 1,
                                          bool wide = false, bool chain = true) {
  const bool numa = nrow > 0;  // nrow: bytes of a NUMA side row (0: none)
  ResLds o;
  int32_t at = 0;
  const int32_t bitmap = res_align(((n_nodes + 31) >> 5) * 4);
  o.lists = at;
  at += res_align(n_pods_max * kp * 8);
  o.pods = at;
  at += res_align(n_pods_max * (int32_t)sizeof(DevPod));
  // two row regions, M' (prev) and M (cur), swapped at the end of every round;
  // a round commits to at most n_pods_max nodes, M' spans `lag` rounds
  const int32_t rows_b = res_align(lag * n_pods_max * (int32_t)sizeof(NV));
  const int32_t numa_b = numa ? res_align(lag * n_pods_max * nrow) : 0;
  o.prev_rows = at;
  o.prev_numa = at + rows_b;
  at += rows_b + numa_b;
  o.cur_rows = at;
  o.cur_numa = at + rows_b;
  at += rows_b + numa_b;
  o.hash_node = at;
  at += RES_HASH * 4;
  o.hash_slot = at;
  at += RES_HASH * 4;
  o.pre_rows = at;
  at += res_align(RES_PRE * (int32_t)sizeof(NV));
  o.pre_numa = at;
  at += numa ? res_align(RES_PRE * nrow) : 0;
  o.pre_node = at;
  at += RES_PRE * 4;
  // the prologue's per-pod decisions: winner key, walked entries (-1: general
  // path), winner row source, the walked nodes
  o.dec_key = at;
  at += RES_MAXP_ROUND * 8;
  o.dec_n = at;
  at += RES_MAXP_ROUND * 4;
  o.dec_src = at;
  at += RES_MAXP_ROUND * 4;
  o.dec_e = at;
  at += RES_MAXP_ROUND * RES_WE * 4;
  o.dec_c = at;  // per pod: bit 0 = its walk met an earlier pod's staged winner, bit 1 = general path only
  at += RES_MAXP_ROUND * 4;
  o.dep = chain ? at : -1;
  at += chain ? RES_MAXP_ROUND * 8 : 0;
  o.moved = at;  // per M' slot: committed to again this round (its row moved into M)
  at += RES_MAXP_ROUND * 4;
  o.mhash = at;  // lazy staged rows: the pod of each M slot, the M slot of each pod
  at += 2 * RES_MAXP_ROUND * 4;
  o.gbits = at;  // the nodes general-path pods committed to this round
  at += bitmap;
  // helper waves' key tables, per pod l (total + 1 as u16 / u32, 0 = infeasible):
  // kpre[l][i] on the row staged pod i commits to (its staged source row +
  // its Reserve delta), ktab[l][s] on M' row s; ready[l] once both are written
  // (tables = false when they do not fit: kpre = -1, the general path then
  // always evaluates and the helper waves idle)
  o.kpre = o.ktab = -1;
  o.kwide = wide ? 1 : 0;
  o.ready = at;
  at += RES_MAXP_ROUND * 4;
  if (tables) {
    o.kpre = at;
    at += RES_MAXP_ROUND * RES_MAXP_ROUND * (wide ? 4 : 2);
    o.ktab = at;
    at += RES_MAXP_ROUND * RES_MAXP_ROUND * (wide ? 4 : 2);
  }
  o.classes = at;  // NodeNUMAResource topology classes (when <= NUMA_LDS_CLASSES)
  at += numa ? NUMA_LDS_CLASSES * (int32_t)sizeof(DevNumaClass) : 0;
  o.modmap = at;  // X bitmap
  at += bitmap;
  o.overlap = overlap ? 1 : 0;
  o.lists2 = o.pods2 = o.pre_rows2 = o.pre_numa2 = o.pre_node2 = 0;
  if (overlap) {
    o.lists2 = at;
    at += res_align(n_pods_max * kp * 8);
    o.pods2 = at;
    at += res_align(n_pods_max * (int32_t)sizeof(DevPod));
    o.pre_rows2 = at;
    at += res_align(RES_PRE * (int32_t)sizeof(NV));
    o.pre_numa2 = at;
    at += numa ? res_align(RES_PRE * nrow) : 0;
    o.pre_node2 = at;
    at += RES_PRE * 4;
  }
  o.total = at;
  return o;
}

__device__ __forceinline__ uint32_t res_hash(int32_t node) { return ((uint32_t)node * 2654435761u) >> 24; }
// A pod record read from LDS made wave-uniform (SGPRs): every lane read the
// same record, readfirstlane tells the compiler so.
__device__ __forceinline__ DevPod uniform_pod(const DevPod &src) {
  DevPod p;
  const uint32_t *s = reinterpret_cast<const uint32_t *>(&src);
  uint32_t *o = reinterpret_cast<uint32_t *>(&p);
#pragma unroll
  for (int i = 0; i < (int)(sizeof(DevPod) / 4); i++) o[i] = __builtin_amdgcn_readfirstlane(s[i]);
  return p;
}
__device__ __forceinline__ bool xbit(const uint32_t *m, int32_t nd) { return (m[nd >> 5] >> (nd & 31)) & 1u; }
// a key-table entry (total + 1, 0 = infeasible) -> the ranking key of node nd
__device__ __forceinline__ uint64_t ktab_key(uint32_t v, int32_t nd) {
  return v ? ((uint64_t)v << 32) | (uint64_t)(0xFFFFFFFFu - (uint32_t)nd) : 0ull;
}

// Evaluation stream, before k_scan of round r: rounds < r - 1 must be written back.
__global__ void k_wait_resolved(PipeSync *sy, int32_t rounds) {
  if (threadIdx.x == 0) (void)wait_at_least(&sy->res_round, rounds, sy);
}
// Evaluation stream, after round r's lists are complete (kernel boundary = visible).
__global__ void k_signal_lists(PipeSync *sy, int32_t par, int32_t pods) {
  if (threadIdx.x == 0) store_release(&sy->sel[par], pods);
}

template <int NM, bool DBG>
__global__ __launch_bounds__(res_threads<NM>()) void k_resolve(DevCfg c, const DevNodes *__restrict__ dn, int32_t n_nodes,
                                                                 const DevNumaClass *__restrict__ ncls, const DevPod *__restrict__ pods,
                                                                 int32_t total, int32_t P, int32_t k, int32_t kp,
                                                                 int32_t r_begin, int32_t r_end,
                                                                 int32_t *__restrict__ mbuf,
                                                                 const uint64_t *__restrict__ lists0,
                                                                 int64_t list_buf, int32_t monotone, int32_t lag,
                                                                 PipeSync *sy, ResLds ofs, int32_t *__restrict__ out_node,
                                                                 uint64_t *__restrict__ out_cpus,
                                                                 uint64_t *__restrict__ dbg, int32_t trace) {
  constexpr int RES_THREADS = res_threads<NM>();
  constexpr bool NUMA = NM != 0, ZONES = NM == 2;
  // the cycle stamps (KOORDHIP_STAMPS) are a separate instantiation: their ~20
  // running counters otherwise stay live across the loop and push the product
  // build of the kernel into scratch spills
  if constexpr (!DBG) dbg = nullptr;
  using NR = side_row_t<NM>;  // the NUMA side row (+ the node's reservation with NM >= 3)
  (void)trace;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  uint64_t *lk = reinterpret_cast<uint64_t *>(lds + ofs.lists);
  DevPod *lpod = reinterpret_cast<DevPod *>(lds + ofs.pods);
  NV *prow = reinterpret_cast<NV *>(lds + ofs.prev_rows);  // M' rows, slot = M' index
  NR *pnr = reinterpret_cast<NR *>(lds + ofs.prev_numa);
  NV *mrow = reinterpret_cast<NV *>(lds + ofs.cur_rows);   // M rows, slot = M index
  NR *mnr = reinterpret_cast<NR *>(lds + ofs.cur_numa);
  int32_t *hnode = reinterpret_cast<int32_t *>(lds + ofs.hash_node);
  int32_t *hslot = reinterpret_cast<int32_t *>(lds + ofs.hash_slot);
  NV *pre = reinterpret_cast<NV *>(lds + ofs.pre_rows);
  NR *prenr = reinterpret_cast<NR *>(lds + ofs.pre_numa);
  int32_t *pre_node = reinterpret_cast<int32_t *>(lds + ofs.pre_node);
  uint64_t *dec_key = reinterpret_cast<uint64_t *>(lds + ofs.dec_key);
  int32_t *dec_n = reinterpret_cast<int32_t *>(lds + ofs.dec_n);
  int32_t *dec_src = reinterpret_cast<int32_t *>(lds + ofs.dec_src);
  int32_t *dec_e = reinterpret_cast<int32_t *>(lds + ofs.dec_e);
  int32_t *dec_c = reinterpret_cast<int32_t *>(lds + ofs.dec_c);
  int32_t *moved = reinterpret_cast<int32_t *>(lds + ofs.moved);
  // lazy staged rows: the pod a bulk commit put in M slot s (its row =
  // that pod's staged source row + its Reserve delta until materialised),
  // and the M slot each staged pod committed to
  int32_t *seg_p = reinterpret_cast<int32_t *>(lds + ofs.mhash);
  uint32_t *gbits = reinterpret_cast<uint32_t *>(lds + ofs.gbits);
  char *kpre = lds + (ofs.kpre >= 0 ? ofs.kpre : 0);
  char *ktab = lds + (ofs.ktab >= 0 ? ofs.ktab : 0);
  const bool kwide = ofs.kwide != 0;  // wave-uniform
  auto kget = [kwide](const char *tb, int32_t x) -> uint32_t {
    return kwide ? reinterpret_cast<const uint32_t *>(tb)[x] : (uint32_t)reinterpret_cast<const uint16_t *>(tb)[x];
  };
  auto kput = [kwide](char *tb, int32_t x, uint32_t v) {
    if (kwide)
      reinterpret_cast<uint32_t *>(tb)[x] = v;
    else
      reinterpret_cast<uint16_t *>(tb)[x] = (uint16_t)v;
  };
  const bool have_tables = ofs.kpre >= 0;
  int32_t *ready = reinterpret_cast<int32_t *>(lds + ofs.ready);
  uint32_t *modmap = reinterpret_cast<uint32_t *>(lds + ofs.modmap);
  // the next round's copies (ofs.overlap): swapped with the above every round
  uint64_t *lk2 = reinterpret_cast<uint64_t *>(lds + ofs.lists2);
  DevPod *lpod2 = reinterpret_cast<DevPod *>(lds + ofs.pods2);
  NV *pre2 = reinterpret_cast<NV *>(lds + ofs.pre_rows2);
  NR *prenr2 = reinterpret_cast<NR *>(lds + ofs.pre_numa2);
  int32_t *pre_node2 = reinterpret_cast<int32_t *>(lds + ofs.pre_node2);
  __shared__ int32_t pnode[RES_MAXP_ROUND];  // M' = the nodes the previous `lag` rounds committed to
  __shared__ int32_t pgen[RES_MAXP_ROUND];   // ... and the round that last did (lag 2)
  __shared__ int32_t seg_w[RES_MAXP_ROUND];  // staged winners by M slot (bulk commits)
  __shared__ int32_t ckey[RES_HASH], cval[RES_HASH];  // staged winner -> first pod (conflict detection)
  __shared__ int32_t sh_mp, sh_stop, sh_done, sh_chain;
  __shared__ uint64_t sh_rsv;  // the chained decisions: pods resolved in the current pass
  const int t = threadIdx.x, lane = lane_id();
  const int32_t words = (n_nodes + 31) >> 5;
  const int32_t HP = max(1, RES_PRE / P);  // prefetched list heads per pod
  // The column pointers are read from a device-side copy of DevNodes at each
  // (rare) row load/store instead of living in SGPRs for the whole kernel:
  // ~40 pointers would otherwise spill through VGPR lanes in the hot loop.
  auto nodes = [dn]() -> DevNodes {
    const DevNodes *p = dn;
    asm volatile("" : "+s"(p));
    return *p;
  };
  const bool two = kp > 64;
  const bool chain_on = (monotone & 2) && ofs.dep >= 0;  // the chained decisions (phase 2c)
  const uint64_t t_kernel = (dbg && t == 0) ? stamp() : 0;
  if (t == 0) {
    sh_mp = r_begin > 0 ? min(mbuf[0], P) : 0;
    sh_stop = 0;
  }
  for (int32_t x = t; x < words; x += RES_THREADS) {
    modmap[x] = 0;
    gbits[x] = 0;
  }
  for (int32_t x = t; x < RES_MAXP_ROUND; x += RES_THREADS) {
    moved[x] = 0;
    ready[x] = 0;
  }
  for (int32_t x = t; x < RES_HASH; x += RES_THREADS) {
    ckey[x] = -1;
    cval[x] = 64;
  }
  const DevNumaClass *cls = ncls;
  if constexpr (NUMA) {  // topology classes -> LDS
    const int32_t nc = nodes().nu.ncls;
    if (nc <= NUMA_LDS_CLASSES) {
      uint4 *dst = reinterpret_cast<uint4 *>(lds + ofs.classes);
      const uint4 *src = reinterpret_cast<const uint4 *>(ncls);
      for (int32_t x = t; x < nc * (int32_t)(sizeof(DevNumaClass) / 16); x += RES_THREADS) dst[x] = src[x];
      cls = reinterpret_cast<const DevNumaClass *>(lds + ofs.classes);
    }
  }
  __syncthreads();
  if (t < sh_mp) {  // resumed pipeline (one launch per round): M' from the previous launch
    const int32_t nd = mbuf[1 + t];
    pnode[t] = nd;
    NV v;
    load_row(v, nodes(), nd);
    prow[t] = v;
    if constexpr (NUMA) {
      NR rr;
      load_side_row<NM>(rr, nodes(), nd);
      pnr[t] = rr;
    }
    atomicOr(&modmap[nd >> 5], 1u << (nd & 31));
  }
  __syncthreads();
  // wave 0: lane s < |M| holds the node of M slot s (its row is mrow[s] in LDS);
  // lane q < RES_WORDS owns word q of a row in the lane-parallel Reserve
  int32_t my_node = -1;
  // byte offset in DevPod of word q's Reserve delta (apply_delta), -1: none
  auto word_doff = [](int q) -> int32_t {
    if (q >= 5 && q < 10) return (q - 5) * 8;  // r[] += req[]
    if (q == 10 || q == 11) return (int32_t)offsetof(DevPod, nz_cpu_m) + (q - 10) * 8;
    if (q == 14 || q == 16) return (int32_t)offsetof(DevPod, est_cpu);  // la_u / la_up (prod)
    if (q == 15 || q == 17) return (int32_t)offsetof(DevPod, est_mem);
    return -1;
  };
  const int32_t doff = word_doff(lane);
  // diagnostics (KOORDHIP_STAMPS): cycles and counts per phase
  uint64_t c_pro = 0, c_wait = 0, c_loop = 0, c_rel = 0, c_hash = 0, c_wb = 0;
  uint64_t c_w1wait = 0, c_w1load = 0, c_bar = 0;  // wave 1: waiting for the next lists, loading them; wave 0: end-of-round barrier
  uint64_t c_l[4] = {0, 0, 0, 0};  // conflict detection, bulk commits, general-path candidate + keys, general commit
  uint64_t n_slow = 0, n_miss = 0, n_staged = 0, n_bulk = 0, n_tab = 0;
  uint64_t c_g[2] = {0, 0};  // general path: candidate from the list, row evaluations (to the last value)
  uint64_t c_nx[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // NUMA: accumulator replays {full, spread} and row passes {req. spread, other}: cycles, count
  // prologue phases 1 / 2 / 2b (cycles), phase-2 HBM row loads, general-path causes: conflicts, slow, voided by a general commit
  uint64_t c_p[3] = {0, 0, 0}, n_p2 = 0, n_conf = 0, n_slowc = 0, n_void = 0;
  uint64_t c_cand = 0, n_evpass = 0, n_tready = 0;  // general path: list + X + c cycles, evaluation passes, pods with ready tables
  uint64_t c_gc[3] = {0, 0, 0}, n_ghit = 0;          // general commit: row source, Reserve delta, voiding + outputs; winners in M
  uint64_t c_chain = 0;                              // chained decisions: cycles (pods resolved: dbg[63])
  uint64_t c_ch[4] = {0, 0, 0, 0};                   // ... split: claim tables, re-walks, re-check + closure, final table
  uint64_t c_rw[4] = {0, 0, 0, 0}, n_chbm = 0;             // ... re-walks: walk + keys, winners' rows; chain HBM row loads
  uint64_t c_ext = 0, n_ext = 0;                     // device pods: cycles from the hand-off to the worker's answer, pods
  // ---- a round's global reads: lists -> LDS (stride kp, zero padded), pod
  //      records, and the rows of each pod's first HP list entries (slot HP j + q)
  // Every loop keeps several global loads in flight per thread before its LDS
  // stores: wave 1 alone runs this for the next round (64 threads), where one
  // load-store pair per iteration serialised ~40 HBM round trips.
  auto load_round = [&](int32_t rr, int32_t rp0, int32_t rn, uint64_t *Lk, DevPod *Lp, NV *Pr, NR *Pn,
                        int32_t *Pnode, int32_t tid, int32_t nth) {
    // Issue order keeps the HBM round trips few for wave 1 alone (one
    // load-store pair per iteration serialised ~40 of them): the list-head
    // entries with the first batch of list loads (16-B vectors of the dense
    // [rn][k] global lists), then the head rows' column loads while the
    // remaining list batches stream in.
    const uint64_t *L = lists0 + (size_t)(rr & (2 * lag - 1)) * list_buf;
    const int32_t tot = rn * k;
    int32_t nd[2];
#pragma unroll
    for (int u = 0; u < 2; u++) {
      const int32_t sl = tid + u * nth, j = sl / HP, q = sl - j * HP;
      nd[u] = -1;
      if (sl < RES_PRE && j < rn && q < k) {
        const uint64_t e = L[(size_t)j * k + q];
        if (e != 0) nd[u] = key_node(e);
      }
    }
    constexpr int LB = 4;  // 16-B list loads in flight per thread (more: the kernel spills)
    const uint4 *L4 = reinterpret_cast<const uint4 *>(L);  // list buffers are 16-B aligned
    const int32_t n16 = (tot + 1) >> 1;
    auto put = [&](int32_t e, uint64_t v) {
      if (e < tot) {
        const int32_t j = e / k, q = e - j * k;
        Lk[j * kp + q] = v;
      }
    };
    uint4 lv[LB];
#pragma unroll
    for (int u = 0; u < LB; u++)
      if (tid + u * nth < n16) lv[u] = L4[tid + u * nth];
#pragma unroll
    for (int u = 0; u < LB; u++) {
      const int32_t x = tid + u * nth;
      if (x < n16) {
        put(2 * x, ((uint64_t)lv[u].y << 32) | lv[u].x);
        put(2 * x + 1, ((uint64_t)lv[u].w << 32) | lv[u].z);
      }
    }
    NV v[2];  // (issued after the first list batch's stores: both at once spill)
#pragma unroll
    for (int u = 0; u < 2; u++)
      if (nd[u] >= 0) load_row(v[u], nodes(), nd[u]);
    for (int32_t x0 = tid + LB * nth; x0 < n16; x0 += LB * nth) {  // rounds whose lists exceed one batch
#pragma unroll
      for (int u = 0; u < LB; u++)
        if (x0 + u * nth < n16) lv[u] = L4[x0 + u * nth];
#pragma unroll
      for (int u = 0; u < LB; u++) {
        const int32_t x = x0 + u * nth;
        if (x < n16) {
          put(2 * x, ((uint64_t)lv[u].y << 32) | lv[u].x);
          put(2 * x + 1, ((uint64_t)lv[u].w << 32) | lv[u].z);
        }
      }
    }
    for (int32_t x = tid; x < rn * (kp - k); x += nth) {  // zero padding of each row up to kp
      const int32_t j = x / (kp - k), q = k + x - j * (kp - k);
      Lk[j * kp + q] = 0ull;
    }
    {
      const uint4 *src = reinterpret_cast<const uint4 *>(pods + rp0);
      uint4 *dst = reinterpret_cast<uint4 *>(Lp);
      const int32_t p16 = rn * (int32_t)(sizeof(DevPod) / 16);
      // four loads in flight per thread, named (an array here went to scratch)
      for (int32_t x0 = tid; x0 < p16; x0 += 4 * nth) {
        const int32_t x1 = x0 + nth, x2 = x0 + 2 * nth, x3 = x0 + 3 * nth;
        const uint4 a0 = src[x0];
        const uint4 a1 = x1 < p16 ? src[x1] : a0;
        const uint4 a2 = x2 < p16 ? src[x2] : a0;
        const uint4 a3 = x3 < p16 ? src[x3] : a0;
        dst[x0] = a0;
        if (x1 < p16) dst[x1] = a1;
        if (x2 < p16) dst[x2] = a2;
        if (x3 < p16) dst[x3] = a3;
      }
    }
#pragma unroll
    for (int u = 0; u < 2; u++) {
      const int32_t sl = tid + u * nth;
      if (sl >= RES_PRE) continue;
      if (nd[u] >= 0) {
        Pr[sl] = v[u];
        if constexpr (NUMA) {
          NR rr2;
          load_side_row<NM>(rr2, nodes(), nd[u]);
          Pn[sl] = rr2;
        }
      }
      Pnode[sl] = nd[u];
    }
    for (int32_t sl = tid + 2 * nth; sl < RES_PRE; sl += nth) {  // more head slots than 2 per thread (never with 64+ threads)
      const int32_t j = sl / HP, q = sl - j * HP;
      int32_t n1 = -1;
      if (j < rn && q < k) {
        const uint64_t e = L[(size_t)j * k + q];
        if (e != 0) n1 = key_node(e);
      }
      if (n1 >= 0) {
        NV v1;
        load_row(v1, nodes(), n1);
        Pr[sl] = v1;
        if constexpr (NUMA) {
          NR rr2;
          load_side_row<NM>(rr2, nodes(), n1);
          Pn[sl] = rr2;
        }
      }
      Pnode[sl] = n1;
    }
  };
  auto prev_slot = [&](int32_t nd) -> int32_t {
    uint32_t h = res_hash(nd);
    for (;;) {
      const int32_t x = hnode[h];
      if (x == nd) return hslot[h];
      if (x < 0) return -1;
      h = (h + 1) & (RES_HASH - 1);
    }
  };
  for (int32_t r = r_begin, p0 = r_begin * P; r < r_end && p0 < total; r++, p0 += P) {
    const int32_t n_pods = min(P, total - p0);
    // ---- 0. this round's inputs: loaded by waves 1.. during the previous
    //         round's loop (overlap), else wait for the lists and load them now
    const bool preloaded = ofs.overlap && r > r_begin;
    const uint64_t t_w0 = (dbg && t == 0) ? stamp() : 0;
    if (!preloaded) {
      if (t == 0 && !wait_at_least(&sy->sel[r & 1], P * (r >> 1) + n_pods, sy)) sh_stop = 1;
      __syncthreads();
    }
    if (sh_stop) return;  // the evaluation side failed: give up, the host reports it
    const uint64_t t_entry = (dbg && t == 0) ? stamp() : 0;
    const int32_t mp = sh_mp;
    if (!preloaded) load_round(r, p0, n_pods, lk, lpod, pre, prenr, pre_node, t, RES_THREADS);
    for (int32_t x = t; x < RES_HASH; x += RES_THREADS) hnode[x] = -1;
    if (t == 0) {
      sh_done = 0;
      sh_chain = 0;
    }
    __syncthreads();
    if (t < mp) {  // M' hash: node -> slot, linear probing, lock-free inserts
      const int32_t nd = pnode[t];
      uint32_t h = res_hash(nd);
      while (atomicCAS(&hnode[h], -1, nd) != -1) h = (h + 1) & (RES_HASH - 1);
      hslot[h] = t;
    }
    __syncthreads();
    const uint64_t t_a = (dbg && t == 0) ? stamp() : 0;
    // list-head rows of M' nodes: the M' slots hold their current rows (a
    // prefetch made while the previous round ran is stale), and a commit to
    // an M' node must go through its slot (moved[]): drop those slots
    if (mp > 0 && t < RES_PRE) {
      const int32_t nd = pre_node[t];
      if (nd >= 0 && prev_slot(nd) >= 0) pre_node[t] = -1;
    }
    // ---- 1. every pod's staged decision: eight lanes per pod walk its first
    //         RES_WE entries; M' entries (X = M' now) are evaluated on their
    //         current rows, the first entry outside M' (exact) ends the walk
    for (int32_t base = 0; base < n_pods * RES_WE; base += RES_THREADS) {
      const int32_t x = base + t;
      const int32_t l = x / RES_WE, q = x - l * RES_WE;
      const bool live = l < n_pods;
      const uint64_t e = (live && q < kp) ? lk[l * kp + q] : 0ull;
      const int32_t nd = e ? key_node(e) : -1;
      const bool inx = e != 0 && xbit(modmap, nd);
      const int g = lane & ~(RES_WE - 1);
      const uint32_t bx = (uint32_t)(__ballot(live && e != 0 && !inx) >> g) & 0xFFu;
      const uint32_t bz = (uint32_t)(__ballot(live && e == 0) >> g) & 0xFFu;
      const int f = bx ? __builtin_ctz(bx) : RES_WE, z = bz ? __builtin_ctz(bz) : RES_WE;
      const bool general = f == RES_WE && z == RES_WE;  // RES_WE M' entries in a row
      const bool walked = live && !general && (q < min(f, z) || (q == f && f < z));
      uint64_t key = 0;
      int32_t ms = -1;
      if (walked) {
        if (q < min(f, z)) {  // an M' entry: its exact key on the current row
          ms = prev_slot(nd);
          const DevPod pod = lpod[l];
          key = make_key(eval_row<NM>(pod, slot_row(prow[ms]), pnr[ms], cls, c), nd);
        } else {
          key = e;
        }
      }
      uint64_t mx = key;
#pragma unroll
      for (int m = 1; m < RES_WE; m <<= 1) {
        const uint64_t o = shfl_xor_u64(mx, m);
        mx = o > mx ? o : mx;
      }
      if (live) {
        dec_e[l * RES_WE + q] = walked ? nd : -1;
        // ---- (2) the staged winner's row, by the lane that walked it: its M'
        //          slot (src < 0), its list-head prefetch slot (entry q < HP:
        //          slot l HP + q), or one HBM load into the pod's first head
        //          slot (entries before it were M' entries: that slot is free)
        if (walked && key == mx && mx != 0) {
          int32_t src;
          if (ms >= 0) {
            src = -ms - 1;
          } else if (q < HP && pre_node[l * HP + q] == nd) {
            src = l * HP + q;
          } else {
            src = l * HP;
            if (dbg) n_p2++;
            NV v;
            load_row(v, nodes(), nd);
            pre[src] = v;
            if constexpr (NUMA) {
              NR nr;
              load_side_row<NM>(nr, nodes(), nd);
              prenr[src] = nr;
            }
            pre_node[src] = nd;
          }
          dec_src[l] = src;
        }
        if (q == 0) {
          const int32_t dn = general ? -1 : (f < z ? f + 1 : z);
          dec_key[l] = mx;
          dec_n[l] = dn;
          if (mx == 0 || dn < 0) dec_src[l] = 0;
          // "slow" pods always take the general path: a non-monotone configuration,
          // NUMA cpuset pods (Allocate at Reserve; required-policy feasibility is
          // not monotone), a walk longer than RES_WE entries
          const uint32_t fl = lpod[l].flags;
          bool slow = !monotone || dn < 0;
          // a device pod: its node comes from k_ext_final (general path)
          if constexpr (NM == 0) slow = slow || (fl & KH_POD_EXT) != 0u;
          if constexpr (NUMA) {
            // (with topology-policy nodes every NUMA pod: its zone hint can move
            // to emptier zones as a node fills, so its score is not monotone)
            slow = slow || (numa_on(c) && ((fl & KOORDHIP_POD_CPUSET) || c.zones) &&
                            !(fl & (KOORDHIP_POD_NUMA_SKIP | KOORDHIP_POD_NUMA_ERROR)));
          }
          if constexpr (NM >= 3) {
            // a pod some reservation may match: committing into a reservation raises
            // its (MostAllocated) reservation score elsewhere -- not monotone
            slow = slow || lpod[l].resv_match != 0ull;
          }
          dec_c[l] = slow ? 2 : 0;
          // claims for the conflict check: staged winner -> first pod (linear probing)
          if (!slow && mx != 0) {
            const int32_t sw = key_node(mx);
            uint32_t h = res_hash(sw);
            for (;;) {
              const int32_t prev = atomicCAS(&ckey[h], -1, sw);
              if (prev == -1 || prev == sw) {
                atomicMin(&cval[h], l);
                break;
              }
              h = (h + 1) & (RES_HASH - 1);
            }
          }
        }
      }
    }
    const uint64_t t_p1 = (dbg && t == 0) ? stamp() : 0;
    __syncthreads();
    const uint64_t t_p2 = (dbg && t == 0) ? stamp() : 0;
    // ---- 2b. conflicts among the staged decisions (one walked entry per
    //          thread): pod l's walk met the staged winner of an earlier pod
    for (int32_t x = t; x < n_pods * RES_WE; x += RES_THREADS) {
      const int32_t l = x / RES_WE;
      const int32_t y = dec_e[x];
      if (y >= 0 && !(dec_c[l] & 2)) {
        uint32_t h = res_hash(y);
        for (;;) {
          const int32_t xk = ckey[h];
          if (xk == y) {
            if (cval[h] < l) atomicOr(&dec_c[l], 1);
            break;
          }
          if (xk < 0) break;
          h = (h + 1) & (RES_HASH - 1);
        }
      }
    }
    __syncthreads();
    uint64_t *dep = ofs.dep >= 0 ? reinterpret_cast<uint64_t *>(lds + ofs.dep) : nullptr;
    if (dep)
      for (int32_t x = t; x < n_pods; x += RES_THREADS) dep[x] = 0ull;
    if (dbg && t == 0) {
      const uint64_t t_p3 = stamp();
      c_hash += t_a - t_entry;
      c_pro += t_p3 - t_a;
      c_wait += t_entry - t_w0;
      c_p[0] += t_p1 - t_a;
      c_p[1] += t_p2 - t_p1;
      c_p[2] += t_p3 - t_p2;
    }
    if (t < 64) {  // ---- 3. the sequential greedy over the round (wave 0)
      __builtin_amdgcn_s_setprio(3);
      // ---- 2c. chained decisions (monotone configurations, monotone bit 1),
      //      wave 0 alone (no workgroup barrier: wave 1 loads the next round
      //      meanwhile; the helper waves wait for sh_chain): a conflicting pod
      //      re-walks its list with the staged winners of the earlier VALID
      //      pods as modified entries -- each evaluated on its claimer's source
      //      row + the claimer's Reserve delta -- up to the first unmodified
      //      entry (exact).  Its decision then assumes those claimers' commits
      //      (dep: a claimer voided later voids it too).  A pod whose new winner
      //      is a valid claimer's node, or whose walk needs more than RES_WE
      //      entries, stays on the general path.  Each pass re-checks the valid
      //      pods against the valid claims and closes the dependencies in pod
      //      order; up to RES_CHAIN_PASSES passes, eight pods per lane group.
      if (chain_on) {
        const uint64_t t_c0 = dbg ? stamp() : 0;
        auto wsync = [&]() {
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        };
        // the claims of the valid (dec_c == 0) pods: staged winner -> first pod
        auto claims = [&]() {
          for (int32_t x = lane; x < RES_HASH; x += 64) {
            ckey[x] = -1;
            cval[x] = 64;
          }
          wsync();
          if (lane < n_pods && dec_c[lane] == 0 && dec_key[lane] != 0ull) {
            const int32_t sw2 = key_node(dec_key[lane]);
            uint32_t h = res_hash(sw2);
            for (;;) {
              const int32_t prev = atomicCAS(&ckey[h], -1, sw2);
              if (prev == -1 || prev == sw2) {
                atomicMin(&cval[h], lane);
                break;
              }
              h = (h + 1) & (RES_HASH - 1);
            }
          }
          wsync();
        };
        auto claimer_of = [&](int32_t y) -> int32_t {
          uint32_t q = res_hash(y);
          for (;;) {
            const int32_t xk = ckey[q];
            if (xk == y) return cval[q];
            if (xk == -1) return 64;  // (-2: a removed claim, probe on)
            q = (q + 1) & (RES_HASH - 1);
          }
        };
        // the first pass's claims from 2b's table (every non-slow pod's staged
        // winner -> its first claimer): drop the nodes whose first claimer
        // conflicts -- every later claimer of such a node met that claim on its
        // own walk (its winner is a walked entry), so it conflicts too, and the
        // table then holds exactly the valid pods' claims (a tombstone, -2,
        // keeps the probe chains)
        auto drop_conflicting = [&]() {
          if (lane < n_pods && dec_c[lane] == 1 && dec_key[lane] != 0ull) {
            const int32_t y = key_node(dec_key[lane]);
            uint32_t q = res_hash(y);
            for (;;) {
              const int32_t xk = ckey[q];
              if (xk == y) {
                if (cval[q] == lane) ckey[q] = -2;
                break;
              }
              if (xk == -1) break;
              q = (q + 1) & (RES_HASH - 1);
            }
          }
          wsync();
        };
        // passes: monotone bits 2-3 (KOORDHIP_CHAIN_PASSES), else RES_CHAIN_PASSES;
        // fresh: ckey / cval hold exactly the valid pods' claims
        const int npass = ((monotone >> 2) & 3) ? ((monotone >> 2) & 3) : RES_CHAIN_PASSES;
        bool fresh = false;
        uint64_t tc = dbg ? stamp() : 0;
        auto clap = [&](int ph) {
          if (dbg) {
            const uint64_t x = stamp();
            c_ch[ph] += x - tc;
            tc = x;
          }
        };
        for (int pass = 0; pass < npass; pass++) {
          if (!fresh) {
            if (pass == 0)
              drop_conflicting();
            else
              claims();
          }
          fresh = true;
          clap(0);
          uint64_t conf = __ballot(lane < n_pods && dec_c[lane] == 1);
          if (!conf) break;
          bool resolved = false;
          if (lane == 0) sh_rsv = 0ull;
          wsync();
          while (conf) {  // eight conflicting pods at a time, eight lanes (entries) each
            const uint64_t t_g = dbg ? stamp() : 0;
            bool hbm = false;
            const int gq = lane >> 3, q = lane & 7;
            uint64_t cm = conf;
            for (int k = 0; k < gq && cm; k++) cm &= cm - 1ull;
            const int32_t l = cm ? (int32_t)__builtin_ctzll(cm) : -1;
            for (int k = 0; k < 8 && conf; k++) conf &= conf - 1ull;
            const bool live = l >= 0;
            const uint64_t e = (live && q < kp) ? lk[l * kp + q] : 0ull;
            const int32_t nd = e ? key_node(e) : -1;
            const bool inm = e != 0 && xbit(modmap, nd);
            const int32_t cl = e != 0 ? claimer_of(nd) : 64;
            const bool clv = live && cl < l;
            const bool mod = inm || clv;
            const int g8 = lane & ~7;
            const uint32_t bx = (uint32_t)(__ballot(live && e != 0 && !mod) >> g8) & 0xFFu;
            const uint32_t bz = (uint32_t)(__ballot(live && e == 0) >> g8) & 0xFFu;
            const int f = bx ? __builtin_ctz(bx) : RES_WE, z = bz ? __builtin_ctz(bz) : RES_WE;
            const bool general = f == RES_WE && z == RES_WE;
            const bool walked = live && !general && (q < min(f, z) || (q == f && f < z));
            const uint64_t t_wk = dbg ? stamp() : 0;
            uint64_t key = 0;
            if (walked) {
              if (q < min(f, z)) {  // a modified entry: its key on the row it will have
                NV v;
                NR nr;
                if (clv) {
                  const int32_t src = dec_src[cl];
                  v = src >= 0 ? pre[src] : prow[-src - 1];
                  if constexpr (NUMA) nr = src >= 0 ? prenr[src] : pnr[-src - 1];
                  apply_delta(v, lpod[cl], +1);
                } else {
                  const int32_t ms = prev_slot(nd);
                  v = slot_row(prow[ms]);
                  if constexpr (NUMA) nr = pnr[ms];
                }
                key = make_key(eval_row<NM>(lpod[l], v, nr, cls, c), nd);
              } else {
                key = e;
              }
            }
            if (dbg) {  // (every lane's key done)
              asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
              const uint64_t t_ev = stamp();
              c_rw[2] += t_wk - t_g;
              c_rw[3] += t_ev - t_wk;
            }
            uint64_t mx = key, dm = (walked && clv) ? (1ull << cl) : 0ull;
#pragma unroll
            for (int m = 1; m < RES_WE; m <<= 1) {
              const uint64_t o = shfl_xor_u64(mx, m);
              mx = o > mx ? o : mx;
              dm |= shfl_xor_u64(dm, m);
            }
            const uint64_t t_k = dbg ? stamp() : 0;
            const bool win = walked && key == mx && mx != 0;
            // the new winner is a valid claimer's node: two commits to one node (general path)
            const bool rep = ((uint32_t)(__ballot(win && clv) >> g8) & 0xFFu) != 0u;
            const bool ok2 = live && !general && !rep;
            if (ok2) {
              dec_e[l * RES_WE + q] = walked ? nd : -1;
              if (win) {  // the winner's row source, as in phase 2
                int32_t src;
                if (inm) {
                  src = -prev_slot(nd) - 1;
                } else if (q < HP && pre_node[l * HP + q] == nd) {
                  src = l * HP + q;
                } else {
                  src = l * HP;
                  hbm = true;
                  NV v;
                  load_row(v, nodes(), nd);
                  pre[src] = v;
                  if constexpr (NUMA) {
                    NR nr;
                    load_side_row<NM>(nr, nodes(), nd);
                    prenr[src] = nr;
                  }
                  pre_node[src] = nd;
                }
                dec_src[l] = src;
              }
              if (q == 0) {
                dec_key[l] = mx;
                dec_n[l] = f < z ? f + 1 : z;
                if (mx == 0) dec_src[l] = 0;
                dep[l] = dm;
                dec_c[l] = 0;
                atomicOr((unsigned long long *)&sh_rsv, (unsigned long long)(1ull << l));
                if (dbg) atomicAdd((unsigned long long *)&dbg[63], 1ull);
              }
            }
            resolved = resolved || (__ballot(ok2) != 0ull);
            wsync();
            if (dbg) {
              const uint64_t t_s = stamp();
              c_rw[0] += t_k - t_g;
              c_rw[1] += t_s - t_k;
              n_chbm += __popcll(__ballot(hbm));
            }
          }
          clap(1);
          if (!resolved) break;
          // re-check: a valid pod whose walk meets the new winner of a pod
          // resolved in this pass that it did not assume -- the only claims
          // that changed: every other valid walk met no earlier claim in 2b,
          // and a re-walk assumed every valid claimer it met.  (Where two pods
          // resolved in one pass took one node, both are checked, not only the
          // first: at most an extra general-path pod, never another placement.)
          bool inv = false;
          for (uint64_t rm = sh_rsv; rm; rm &= rm - 1ull) {
            const int32_t r = (int32_t)__builtin_ctzll(rm);
            const uint64_t kr = dec_key[r];
            if (kr == 0ull) continue;
            const int32_t wr = key_node(kr);
            for (int32_t x0 = (r + 1) * RES_WE; x0 < n_pods * RES_WE; x0 += 64) {
              const int32_t x = x0 + lane, l2 = x / RES_WE;
              const bool bad = x < n_pods * RES_WE && dec_e[x] == wr && dec_c[l2] == 0 && !((dep[l2] >> r) & 1ull);
              if (bad) atomicOr(&dec_c[l2], 1);
              inv = inv || __ballot(bad) != 0ull;
            }
            wsync();
          }
          {  // closure in pod order: a pod assuming an invalid pod's commit is invalid
            const bool lv = lane < n_pods;
            const uint64_t dl = lv ? dep[lane] : 0ull;
            uint64_t valid = __ballot(lv && dec_c[lane] == 0);
            for (;;) {
              const uint64_t bad = __ballot(((valid >> lane) & 1ull) && (dl & ~valid) != 0ull);
              if (!bad) break;
              inv = true;
              valid &= ~bad;
              if ((bad >> lane) & 1ull) dec_c[lane] = 1;
            }
          }
          wsync();
          fresh = false;  // (the resolved pods' new claims are not in the table)
          clap(2);
        }
        if (!fresh) claims();  // the loop's claimer(): the valid pods' winners
        clap(3);
        if (lane == 0) __hip_atomic_store(&sh_chain, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (dbg) c_chain += stamp() - t_c0;
      }
      const uint64_t t_loop = dbg ? stamp() : 0;
      int32_t nm = 0;  // |M| (wave-uniform)
      my_node = -1;
      const int32_t pn0 = pre_node[lane], pn1 = pre_node[lane + 64];
      // ---- lane l = pod l: its staged decision in registers
      const bool live = lane < n_pods;
      uint32_t fl = 0;
      int32_t sw = -1, ssrc = 0;
      int32_t se[RES_WE];
#pragma unroll
      for (int q = 0; q < RES_WE; q++) se[q] = -1;
      if (live) {
        fl = lpod[lane].flags;
        const uint64_t kk = dec_key[lane];
        sw = kk ? key_node(kk) : -1;
        ssrc = dec_src[lane];
#pragma unroll
        for (int q = 0; q < RES_WE; q++) se[q] = dec_e[lane * RES_WE + q];
      }
      const uint64_t prodmask = __ballot(live && (fl & KOORDHIP_POD_PROD));
      const uint64_t mydep = (dep && live) ? dep[lane] : 0ull;  // the staged commits this pod's chained decision assumed
      // general-path-only pods and conflicts: from the prologue (phase 2 / 2b)
      const int32_t dc = live ? dec_c[lane] : 2;
      const bool slow = (dc & 2) != 0;
      const bool conflict = (dc & 1) != 0;
      uint64_t ok = __ballot(live && !slow && !conflict);  // staged decisions still valid
      uint64_t cstaged = 0;                                 // pods committed with their staged decision
      // Lazy staged rows: a bulk commit only records (slot, pod); the row is
      // materialised when a general commit hits it, before a non-monotone
      // pass over all M rows, and at the write-back.  my_node (node of slot
      // lane s) is valid for the slots of gvalid (general commits and
      // materialised slots); lane l of a staged pod holds its slot (pslot_r).
      uint64_t lazy = 0, gvalid = 0;
      int32_t pslot_r = -1;
      const uint64_t slowmask = __ballot(live && slow);
      if (dbg) {
        n_conf += __popcll(__ballot(live && !slow && conflict));
        n_slowc += __popcll(slowmask);
      }
      // materialise lazy slot s (uniform): its staged pod's source row + Reserve
      // delta, word-parallel (over-commit flags left to slot_row), and its side row
      auto materialize = [&](int32_t s) {
        const int32_t pi = seg_p[s];
        const int32_t src = dec_src[pi];
        const int32_t nd = seg_w[s];
        if (lane < RES_WORDS) {
          const uint64_t *srow = reinterpret_cast<const uint64_t *>(src >= 0 ? &pre[src] : &prow[-src - 1]);
          uint64_t x = srow[lane];
          if (doff >= 0 && (lane < 16 || ((prodmask >> pi) & 1ull))) {
            const double dq = *reinterpret_cast<const double *>(reinterpret_cast<const char *>(&lpod[pi]) + doff);
            x = (uint64_t)__double_as_longlong(__longlong_as_double((long long)x) + dq);
          }
          if (lane == 18) x += 1ull << 32;
          reinterpret_cast<uint64_t *>(&mrow[s])[lane] = x;
        }
        if constexpr (NUMA) {
          constexpr int NRW = (int)(sizeof(NR) / 8);
          const uint64_t *sn = reinterpret_cast<const uint64_t *>(src >= 0 ? &prenr[src] : &pnr[-src - 1]);
          for (int32_t w = lane; w < NRW; w += 64) reinterpret_cast<uint64_t *>(&mnr[s])[w] = sn[w];
        }
        if (lane == s) my_node = nd;
        lazy &= ~(1ull << s);
        gvalid |= 1ull << s;
      };
      // the first pod whose staged winner is node y (64: none)
      auto claimer = [&](int32_t y) -> int32_t {
        uint32_t q = res_hash(y);
        for (;;) {
          const int32_t xk = ckey[q];
          if (xk == y) return cval[q];
          if (xk == -1) return 64;  // (-2: a claim the chained decisions dropped)
          q = (q + 1) & (RES_HASH - 1);
        }
      };
      int32_t j = 0;
      if (dbg) c_l[0] += stamp() - t_loop;
      while (j < n_pods) {
        uint64_t ts = dbg ? stamp() : 0;
        auto lap = [&](int ph) {
          if (dbg) {
            const uint64_t x = stamp();
            c_l[ph] += x - ts;
            ts = x;
          }
        };
        // ---- the next general-path pod g; pods [j, g) commit their staged
        //      decisions together (distinct winners: a shared winner is a conflict)
        const uint64_t from_j = ~0ull << j;
        const uint64_t gen = ~ok & from_j & (n_pods < 64 ? ((1ull << n_pods) - 1ull) : ~0ull);
        const int32_t g = gen ? (int32_t)__builtin_ctzll(gen) : n_pods;
        if (g > j) {
          const bool mine = lane >= j && lane < g;
          const bool com = mine && sw >= 0;
          const uint64_t cb = __ballot(com);
          const int32_t slot = nm + __popcll(cb & ((1ull << lane) - 1ull));
          if (com) {
            if (ssrc < 0) moved[-ssrc - 1] = 1;
            atomicOr(&modmap[sw >> 5], 1u << (sw & 31));
            seg_w[slot] = sw;
            seg_p[slot] = lane;
            pslot_r = slot;
          }
          if (mine) {
            // write-through: the class lists read the placements as the commit log
            st_wt(&out_node[p0 + lane], (int32_t)(com ? sw : KOORDHIP_UNSCHEDULABLE));
            if (out_cpus) {
#pragma unroll
              for (int q = 0; q < NW; q++) out_cpus[(size_t)(p0 + lane) * NW + q] = 0ull;
            }
          }
          const int32_t nc = __popcll(cb);
          lazy |= (nc >= 64 ? ~0ull : ((1ull << nc) - 1ull)) << nm;
          nm += nc;
          cstaged |= cb;
          n_staged += g - j;
          n_bulk++;
        }
        lap(1);
        if (g >= n_pods) break;
        // ---- general path: pod g alone -- c, then every M and M' row's current key
        n_slow++;
        const DevPod pod = lpod[g];  // VGPR copy: SGPRs are the scarce register file here (uniform_pod measured slower)
        // A device pod (KH_POD_EXT, plain build): k_ext_final places it on the
        // exact state -- every commit so far written back first (M rows,
        // write-through, drained) and X exported, then the hand-off; its node (or
        // UNSCHEDULABLE / RESERVE_FAILED) comes back through out_node, and the
        // Fit / LoadAware delta is committed below like any general-path pod's.
        bool ext_pod = false;
        int32_t ext_res = KOORDHIP_UNSCHEDULABLE;
        if constexpr (NM == 0) ext_pod = (__builtin_amdgcn_readfirstlane(pod.flags) & KH_POD_EXT) != 0u;
        if (ext_pod) {
          const uint64_t t_x = dbg ? stamp() : 0;
          while (lazy) materialize((int32_t)__builtin_ctzll(lazy));
          if (lane < nm) {
            const NV v = slot_row(mrow[lane]);
            mrow[lane] = v;
            store_row_wt(v, nodes(), my_node);
          }
          {  // X = M' + this round's M so far: the nodes the worker evaluates again
            int32_t *xl = pipe_xlist(sy);
            if (lane < mp) st_wt(&xl[1 + lane], pnode[lane]);
            if (lane < nm) st_wt(&xl[1 + mp + lane], my_node);
            if (lane == 0) st_wt(&xl[0], mp + nm);
          }
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          int32_t xr = KOORDHIP_UNSCHEDULABLE;
          if (lane == 0) {
            __hip_atomic_store(&sy->ext_req, p0 + g + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (wait_at_least(&sy->ext_done, p0 + g + 1, sy))
              xr = __hip_atomic_load(&out_node[p0 + g], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
          ext_res = __builtin_amdgcn_readfirstlane(xr);
          if (dbg) {
            c_ext += stamp() - t_x;
            n_ext++;
          }
        }
        const uint64_t *L = lk + (size_t)g * kp;
        const uint64_t e0 = lane < kp ? L[lane] : 0ull;
        const uint64_t e1 = (two && 64 + lane < kp) ? L[64 + lane] : 0ull;
        const bool x0 = e0 != 0 && xbit(modmap, key_node(e0));
        const bool x1 = e1 != 0 && xbit(modmap, key_node(e1));
        const uint64_t f0 = __ballot(e0 != 0 && !x0), f1 = __ballot(e1 != 0 && !x1);
        uint64_t best = f0 ? readlane_u64(e0, __builtin_ctzll(f0)) : (f1 ? readlane_u64(e1, __builtin_ctzll(f1)) : 0ull);
        if (ext_pod) best = ext_res >= 0 ? make_key(0, ext_res) : 0ull;
        // (NM 5) how many nodes are feasible now: the list's entries outside X
        // are exact, the X rows are all evaluated below (these pods are never
        // monotone), and a list that was not full held every node feasible at
        // its evaluation (feasibility only shrinks).  One: upstream returns it
        // without PreScore, so no reservation is nominated for the Reserve.
        int32_t nfeas = __popcll(f0) + __popcll(f1);
        const bool lfull = (k <= 64 ? readlane_u64(e0, k - 1) : readlane_u64(e1, k - 65)) != 0ull;
        // A monotone pod: only the X entries ranked above c can win.  Each one's
        // current key: from the helper waves' key tables when they are ready
        // (kpre: the row its staged claimer committed to; ktab: an M' row no
        // commit touched), else one evaluation on its current row -- a
        // materialised M slot (a general commit changed it), its staged
        // claimer's lazy row, or its M' row.
        const bool mono_g = monotone && !((slowmask >> g) & 1ull);  // (device pods are slow: no keys to take)
        if (dbg) c_cand += stamp() - ts;
        if (mono_g) {
          const bool tabs = have_tables && __hip_atomic_load(&ready[g], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != 0;
          if (dbg) n_tready += tabs;
          const int first = f0 ? __builtin_ctzll(f0) : (f1 ? 64 + __builtin_ctzll(f1) : 128);
          bool used = false;
#pragma unroll
          for (int h = 0; h < 2; h++) {
            const uint64_t e = h ? e1 : e0;
            const bool xh = (h ? x1 : x0) && 64 * h + lane < first;
            if (__ballot(xh)) {
              uint64_t kv = 0;
              if (xh) {
                const int32_t y = key_node(e);
                const bool gb = xbit(gbits, y);
                const int32_t cl = gb ? 64 : claimer(y);
                const bool st = cl < 64 && ((cstaged >> cl) & 1ull);
                const int32_t sl = (gb || st || mp == 0) ? -1 : prev_slot(y);
                bool have = false;
                if (tabs && !gb) {
                  if (st) {
                    kv = ktab_key(kget(kpre, g * RES_MAXP_ROUND + cl), y);
                    have = true;
                  } else if (sl >= 0) {
                    kv = ktab_key(kget(ktab, g * RES_MAXP_ROUND + sl), y);
                    have = true;
                  }
                }
                if (dbg && __ballot(!have) != 0ull && lane == (int)__builtin_ctzll(__ballot(true))) n_evpass++;
                if (!have) {
                  NV v;
                  NR nr;
                  if (gb) {
                    int32_t ms = 0;
                    for (uint64_t gm = gvalid; gm; gm &= gm - 1ull) {
                      const int sx = __builtin_ctzll(gm);
                      if (__builtin_amdgcn_readlane(my_node, sx) == y) ms = sx;
                    }
                    v = slot_row(mrow[ms]);
                    if constexpr (NUMA) nr = mnr[ms];
                  } else if (st) {
                    const int32_t src = dec_src[cl];
                    v = src >= 0 ? pre[src] : prow[-src - 1];
                    if constexpr (NUMA) nr = src >= 0 ? prenr[src] : pnr[-src - 1];
                    apply_delta(v, lpod[cl], +1);
                  } else {
                    v = slot_row(prow[sl]);
                    if constexpr (NUMA) nr = pnr[sl];
                  }
                  kv = make_key(eval_row<NM>(pod, v, nr, cls, c), y);
                }
                used = used || have;
              }
              kv = wave_max_u64_dpp(kv);
              best = kv > best ? kv : best;
            }
          }
          n_tab += __ballot(used) != 0;
        }
        if (dbg) {
          const uint64_t x = stamp();
          c_g[0] += x - ts;
          ts = x;
        }
        const int32_t nrows = (mono_g || ext_pod) ? 0 : nm + mp;
        const uint64_t t_rows = dbg ? stamp() : 0;
        if (nrows > 0)  // a pass over every M row: materialise the lazy ones first
          while (lazy) materialize((int32_t)__builtin_ctzll(lazy));
        for (int32_t b0 = 0; b0 < nrows; b0 += 64) {  // rows: M slots, then the M' slots not moved into M
          const int32_t s = b0 + lane;
          uint64_t kv = 0;
          if (s < nm) {
            NR nr;
            if constexpr (NUMA) nr = mnr[s];
            kv = make_key(eval_row<NM>(pod, slot_row(mrow[s]), nr, cls, c), my_node);
          } else if (s < nrows && !moved[s - nm]) {
            NR nr;
            if constexpr (NUMA) nr = pnr[s - nm];
            kv = make_key(eval_row<NM>(pod, slot_row(prow[s - nm]), nr, cls, c), pnode[s - nm]);
          }
          if (dbg) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            c_g[1] += stamp() - ts;
          }
          if constexpr (NM == 5) nfeas += __popcll(__ballot(kv != 0ull));
          kv = wave_max_u64_dpp(kv);
          best = kv > best ? kv : best;
        }
        const bool single = !mono_g && !lfull && nfeas == 1;  // (mono_g: the X rows were not all evaluated)
        (void)single;
        if (dbg && NUMA && nrows > 0) {
          const int b = KOORDHIP_NUMA_REQUIRED(pod.numa_policy) == KOORDHIP_CPUBIND_SPREAD_BY_PCPUS ? 4 : 6;
          c_nx[b] += stamp() - t_rows;
          c_nx[b + 1]++;
        }
        lap(2);
        uint64_t cpus[NW] = {0, 0, 0, 0};
        int32_t result = ext_pod ? ext_res : KOORDHIP_UNSCHEDULABLE;
        uint64_t t_gc = dbg ? stamp() : 0;
        auto gclap = [&](int ph) {
          if (dbg) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            const uint64_t x = stamp();
            c_gc[ph] += x - t_gc;
            t_gc = x;
          }
        };
        if (best != 0) {
          const int32_t w = key_node(best);
          // w's M slot (a staged pod's, materialised now if lazy, or a general
          // commit's); its current row: the slot itself, else (new this round)
          // a prefetched list-head row, an M' row, or HBM (rare)
          const uint64_t hit_s = __ballot(lane < n_pods && ((cstaged >> lane) & 1ull) && sw == w);
          int32_t rw = nm;
          if (hit_s) {
            rw = __builtin_amdgcn_readlane(pslot_r, __builtin_ctzll(hit_s));
            if ((lazy >> rw) & 1ull) materialize(rw);
          } else {
            const uint64_t hit_g = __ballot(((gvalid >> lane) & 1ull) && my_node == w);
            if (hit_g) rw = __builtin_ctzll(hit_g);
          }
          const bool hit = rw < nm;
          if (dbg) n_ghit += hit;
          const NV *srow = &mrow[rw];
          const NR *snr = &mnr[rw];
          int32_t from_prev = -1;
          if (!hit) {
            const uint64_t pm0 = __ballot(pn0 == w), pm1 = __ballot(pn1 == w);
            const int src = pm0 ? __builtin_ctzll(pm0) : (pm1 ? 64 + __builtin_ctzll(pm1) : -1);
            const int32_t sl = (src < 0 && mp > 0) ? prev_slot(w) : -1;
            if (src >= 0) {
              srow = &pre[src];
              snr = &prenr[src];
            } else if (sl >= 0) {
              srow = &prow[sl];
              snr = &pnr[sl];
              from_prev = sl;
            } else {
              n_miss++;
              if (lane == 0) {
                NV v;
                load_row(v, nodes(), w);
                mrow[rw] = v;
                if constexpr (NUMA) {
                  NR nr;
                  load_side_row<NM>(nr, nodes(), w);
                  mnr[rw] = nr;
                }
              }
            }
          }
          gclap(0);
          bool okr = true;
          if constexpr (NUMA) {
            if (numa_on(c) && numa_active(pod, c)) {
              // NodeNUMAResource Reserve: lane 0 replays the accumulator (and the
              // zone hint) on the row, the chosen CPUs are broadcast to the wave
              uint64_t mc[NW] = {0, 0, 0, 0};
              int okl = 0;
              const uint64_t t_acc = dbg ? stamp() : 0;
              {  // every lane: the accumulator's id-ordered takes run lane-parallel
                NR nr = *snr;
                if constexpr (NM == 5) {  // the nominated reservation's reserved CPUs first
                  uint64_t pref[NW];
                  resv_pref_cpus(nr, pod,
                                 ((c.score & KOORDHIP_PLUGIN_RESERVATION) && !single) ? resv_matched(nr, pod) : 0u, pref);
                  okl = numa_reserve<ZONES, true>(cls, nr, pod, mc, pref);
                } else {
                  okl = numa_reserve<ZONES, true>(cls, nr, pod, mc);
                }
                if (okl && lane == 0) mnr[rw] = nr;
              }
              if (dbg) {
                const int b = KOORDHIP_NUMA_PREFERRED(pod.numa_policy) == KOORDHIP_CPUBIND_SPREAD_BY_PCPUS ? 2 : 0;
                c_nx[b] += stamp() - t_acc;
                c_nx[b + 1]++;
              }
              okr = __builtin_amdgcn_readfirstlane(okl) != 0;
#pragma unroll
              for (int q = 0; q < NW; q++) cpus[q] = readlane_u64(mc[q], 0);
            } else if (!hit && lane < (int)(sizeof(NR) / 8)) {
              reinterpret_cast<uint64_t *>(&mnr[rw])[lane] = reinterpret_cast<const uint64_t *>(snr)[lane];
            }
          }
          if constexpr (NM >= 3) {
            // Reservation Reserve: assumePod into the node's nominated reservation
            if (okr && c.resv && pod.resv_match != 0ull && lane == 0) {
              NR nr = mnr[rw];
              resv_assume(nr, pod, cpus);
              mnr[rw] = nr;
            }
          }
          if (!okr) {
            result = KOORDHIP_RESERVE_FAILED;  // nothing is committed
          } else {
            result = w;
            // Reserve delta, lane q on word q (flags: slot_row() on read)
            const uint64_t xw = lane < RES_WORDS ? reinterpret_cast<const uint64_t *>(srow)[lane] : 0ull;
            const double dq = (doff >= 0 && (lane < 16 || ((prodmask >> g) & 1ull)))
                                  ? *reinterpret_cast<const double *>(reinterpret_cast<const char *>(&lpod[g]) + doff)
                                  : 0.0;
            uint64_t x = xw;
            if (lane < 18) x = (uint64_t)__double_as_longlong(__longlong_as_double((long long)xw) + dq);
            if (lane == 18) x += 1ull << 32;
            if (lane < RES_WORDS) reinterpret_cast<uint64_t *>(&mrow[rw])[lane] = x;
            if (lane == 0) atomicOr(&gbits[w >> 5], 1u << (w & 31));
            if (!hit) {
              if (lane == rw) my_node = w;
              gvalid |= 1ull << rw;
              if (lane == 0) {
                atomicOr(&modmap[w >> 5], 1u << (w & 31));
                if (from_prev >= 0) moved[from_prev] = 1;
              }
              nm++;
            }
            gclap(1);
            // later staged decisions that walked w are void
            bool met = false;
#pragma unroll
            for (int q = 0; q < RES_WE; q++) met = met || se[q] == w;
            uint64_t voided = __ballot(lane > g && met);
            // ... and the chained decisions that assumed a voided pod's commit
            for (;;) {
              const uint64_t nx = __ballot(lane > g && ((ok >> lane) & 1ull) && !((voided >> lane) & 1ull) &&
                                           (mydep & voided) != 0ull);
              if (!nx) break;
              voided |= nx;
            }
            if (dbg) n_void += __popcll(ok & voided);
            ok &= ~voided;
          }
        }
        if (lane == 0) st_wt(&out_node[p0 + g], result);
        if (out_cpus && lane < NW)
          out_cpus[(size_t)(p0 + g) * NW + lane] =
              lane == 0 ? cpus[0] : (lane == 1 ? cpus[1] : (lane == 2 ? cpus[2] : cpus[3]));
        gclap(2);
        lap(3);
        j = g + 1;
      }
      // ---- 4. write M back; M becomes the next round's M' (rows stay in LDS)
      const uint64_t t_wb = dbg ? stamp() : 0;
      if (lane < nm && ((lazy >> lane) & 1ull)) {  // a lazy staged row: materialised here, word by word
        const int32_t pi = seg_p[lane];
        my_node = seg_w[lane];
        const int32_t src = dec_src[pi];
        const uint64_t *sr = reinterpret_cast<const uint64_t *>(src >= 0 ? &pre[src] : &prow[-src - 1]);
        uint64_t *dr = reinterpret_cast<uint64_t *>(&mrow[lane]);
        const char *pp = reinterpret_cast<const char *>(&lpod[pi]);
        const bool prod = ((prodmask >> pi) & 1ull) != 0;
        // two halves, each loaded whole before its stores (LDS pointers may
        // alias for the compiler: word-by-word would serialise 20 round trips)
#pragma unroll
        for (int h = 0; h < 2; h++) {
          uint64_t x[RES_WORDS / 2];
          double dq[RES_WORDS / 2];
#pragma unroll
          for (int u = 0; u < RES_WORDS / 2; u++) {
            const int q = h * (RES_WORDS / 2) + u;
            const int32_t o = word_doff(q);
            x[u] = sr[q];
            dq[u] = (o >= 0 && (q < 16 || prod)) ? *reinterpret_cast<const double *>(pp + o) : 0.0;
          }
#pragma unroll
          for (int u = 0; u < RES_WORDS / 2; u++) {
            const int q = h * (RES_WORDS / 2) + u;
            uint64_t y = x[u];
            if (word_doff(q) >= 0) y = (uint64_t)__double_as_longlong(__longlong_as_double((long long)y) + dq[u]);
            if (q == 18) y += 1ull << 32;
            dr[q] = y;
          }
        }
        if constexpr (NUMA) {
          const uint64_t *sn = reinterpret_cast<const uint64_t *>(src >= 0 ? &prenr[src] : &pnr[-src - 1]);
          uint64_t *dn2 = reinterpret_cast<uint64_t *>(&mnr[lane]);
#pragma unroll 4
          for (int w = 0; w < (int)(sizeof(NR) / 8); w++) dn2[w] = sn[w];
        }
      }
      if (lane < nm) {
        const NV v = slot_row(mrow[lane]);
        mrow[lane] = v;
#ifdef KH_PUBLISH_RELEASE
        store_row(v, nodes(), my_node);
#else
        store_row_wt(v, nodes(), my_node);  // write-through: no L2 write-back fence at the publish
#endif
        if constexpr (NUMA) {
          const NR nr = mnr[lane];
#ifdef KH_PUBLISH_RELEASE
          store_side_row<NM>(nr, nodes(), my_node);
#else
          store_side_row_wt<NM>(nr, nodes(), my_node);
#endif
        }
      }
      if (lane == 0) __hip_atomic_store(&sh_done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);  // helpers stop
      // lag 2: the next round's lists were evaluated before this round and the
      // previous one, so the M' slots the previous round committed to (and this
      // one did not) stay in X: their current rows follow M's in the M region
      const bool surv = lag > 1 && lane < mp && pgen[lane] == r - 1 && !moved[lane];
      const uint64_t sbm = __ballot(surv);
      const int32_t ns = __popcll(sbm);
      const int32_t sidx = nm + __popcll(sbm & ((1ull << lane) - 1ull));
      int32_t snode = -1;
      if (surv) {
        snode = pnode[lane];
        mrow[sidx] = prow[lane];
        if constexpr (NUMA) mnr[sidx] = pnr[lane];
      }
      // X of the next round = M (+ those): clear the words of M' and M (every
      // bit set in them is X's), then set the next X's bits; M's and the general
      // pods' bitmaps are cleared (both are subsets of M), and the staged-winner claims
      if (lane < mp) modmap[pnode[lane] >> 5] = 0;
      if (lane < nm) {
        modmap[my_node >> 5] = 0;
        gbits[my_node >> 5] = 0;
      }
      for (int32_t x = lane; x < RES_HASH; x += 64) {
        ckey[x] = -1;
        cval[x] = 64;
      }
      if (lane < nm) {
        atomicOr(&modmap[my_node >> 5], 1u << (my_node & 31));
        pnode[lane] = my_node;
        pgen[lane] = r;
      }
      if (surv) {
        atomicOr(&modmap[snode >> 5], 1u << (snode & 31));
        pnode[sidx] = snode;
        pgen[sidx] = r - 1;
      }
      moved[lane] = 0;
      const uint64_t t_rel = dbg ? stamp() : 0;
      if (dbg) c_wb += t_rel - t_wb;
      if (lane == 0) {
        sh_mp = nm + ns;
        // the rows were stored write-through: drain them, then the relaxed
        // agent-scope flag (Guideline 16 R1; the evaluation side acquires)
#ifdef KH_PUBLISH_RELEASE
        store_release(&sy->res_round, r + 1);
#else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(&sy->res_round, r + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
      }
      if (dbg) {
        const uint64_t t_end = stamp();
        c_rel += t_end - t_rel;
        c_loop += t_end - t_loop;
      }
    } else if (t < 64 * (1 + res_loaders<NM>())) {
      if (ofs.overlap && r + 1 < r_end && p0 + P < total) {
        // ---- waves 1..: the next round's lists, pods and head rows, meanwhile
        //      (each waits for the lists itself: no barrier without wave 0)
        const int32_t np2 = min(P, total - (p0 + P));
        int ok = 1;
        const uint64_t t1 = dbg ? stamp() : 0;
        if (lane == 0) ok = wait_at_least(&sy->sel[(r + 1) & 1], P * ((r + 1) >> 1) + np2, sy) ? 1 : 0;
        const uint64_t t2 = dbg ? stamp() : 0;
        if (__builtin_amdgcn_readfirstlane(ok)) {
          load_round(r + 1, p0 + P, np2, lk2, lpod2, pre2, prenr2, pre_node2, t - 64, 64 * res_loaders<NM>());
          if (dbg) {
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            c_w1load += stamp() - t2;
          }
        } else if (lane == 0) {
          sh_stop = 1;
        }
        if (dbg) c_w1wait += t2 - t1;
      }
    } else {
      // ---- waves 2..: key tables for the general path, pod by pod (one pod
      //      per wave: its record is wave-uniform), lanes over the rows --
      //      kpre[l][i] on staged pod i's committed row, ktab[l][s] on M' row s
      //      Only the pods whose staged decision conflicts use them (general
      //      path, monotone): those pods are dealt round-robin to the waves.
      const int hw = __builtin_amdgcn_readfirstlane((t >> 6) - 1 - res_loaders<NM>()),
                nh = RES_THREADS / 64 - 1 - res_loaders<NM>();
      if (chain_on)  // wave 0's chained decisions first (they rewrite the staged decisions)
        while (!__hip_atomic_load(&sh_chain, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) __builtin_amdgcn_s_sleep(1);
      uint64_t todo = __ballot(lane < n_pods && dec_c[lane] == 1);
      for (int32_t x = 0; x < hw && todo; x++) todo &= todo - 1ull;
      for (; have_tables && todo;) {
        const int32_t l = (int32_t)__builtin_ctzll(todo);
        for (int32_t x = 0; x < nh && todo; x++) todo &= todo - 1ull;
        if (__hip_atomic_load(&sh_done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) break;
        const DevPod pod = uniform_pod(lpod[l]);
        for (int32_t b0 = 0; b0 < l + mp; b0 += 64) {
          const int32_t x = b0 + lane;
          int32_t v = 0;
          if (x < l) {  // staged pod i = x
            const uint64_t kk = dec_key[x];
            if (kk != 0 && dec_n[x] >= 0) {
              const int32_t src = dec_src[x];
              NV row = src >= 0 ? pre[src] : prow[-src - 1];
              NR nr;
              if constexpr (NUMA) nr = src >= 0 ? prenr[src] : pnr[-src - 1];
              const DevPod pi = lpod[x];
              apply_delta(row, pi, +1);
              v = eval_row<NM>(pod, row, nr, cls, c) + 1;
            }
            kput(kpre, l * RES_MAXP_ROUND + x, (uint32_t)v);
          } else if (x < l + mp) {  // M' slot s
            const int32_t sl = x - l;
            NR nr;
            if constexpr (NUMA) nr = pnr[sl];
            v = eval_row<NM>(pod, slot_row(prow[sl]), nr, cls, c) + 1;
            kput(ktab, l * RES_MAXP_ROUND + sl, (uint32_t)v);
          }
        }
        if (lane == 0) __hip_atomic_store(&ready[l], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
    const uint64_t t_bar = (dbg && t == 0) ? stamp() : 0;
    __syncthreads();
    if (dbg && t == 0) c_bar += stamp() - t_bar;
    for (int32_t x = t; x < RES_MAXP_ROUND; x += RES_THREADS) ready[x] = 0;
    if (ofs.overlap) {  // the next round's inputs become current
      uint64_t *a = lk;
      lk = lk2;
      lk2 = a;
      DevPod *b = lpod;
      lpod = lpod2;
      lpod2 = b;
      NV *c2 = pre;
      pre = pre2;
      pre2 = c2;
      NR *d2 = prenr;
      prenr = prenr2;
      prenr2 = d2;
      int32_t *e2 = pre_node;
      pre_node = pre_node2;
      pre_node2 = e2;
    }
    {  // M's rows become the next round's M' rows
      NV *x = prow;
      prow = mrow;
      mrow = x;
      NR *y = pnr;
      pnr = mnr;
      mnr = y;
    }
  }
  if (t <= RES_MAXP_ROUND && t <= sh_mp) mbuf[t] = t == 0 ? sh_mp : pnode[t - 1];  // hand M' on
  if (dbg && n_p2) atomicAdd((unsigned long long *)&dbg[51], (unsigned long long)n_p2);
  if (dbg && n_evpass) atomicAdd((unsigned long long *)&dbg[57], (unsigned long long)n_evpass);
  if (dbg && t == 64) {
    atomicAdd((unsigned long long *)&dbg[27], (unsigned long long)c_w1wait);
    atomicAdd((unsigned long long *)&dbg[28], (unsigned long long)c_w1load);
  }
  if (dbg && t == 0) {
    atomicAdd((unsigned long long *)&dbg[0], (unsigned long long)c_pro);
    atomicAdd((unsigned long long *)&dbg[1], (unsigned long long)c_wait);
    atomicAdd((unsigned long long *)&dbg[2], (unsigned long long)c_hash);
    atomicAdd((unsigned long long *)&dbg[4], (unsigned long long)c_loop);
    atomicAdd((unsigned long long *)&dbg[5], (unsigned long long)n_slow);
    atomicAdd((unsigned long long *)&dbg[6], (unsigned long long)n_miss);
    atomicAdd((unsigned long long *)&dbg[7], (unsigned long long)total);
    atomicAdd((unsigned long long *)&dbg[14], (unsigned long long)c_rel);
    atomicAdd((unsigned long long *)&dbg[25], (unsigned long long)c_wb);
    atomicAdd((unsigned long long *)&dbg[26], (unsigned long long)(stamp() - t_kernel));
    atomicAdd((unsigned long long *)&dbg[29], (unsigned long long)c_bar);
    for (int q = 0; q < 8; q++) atomicAdd((unsigned long long *)&dbg[32 + q], (unsigned long long)c_nx[q]);
    for (int q = 0; q < 4; q++) atomicAdd((unsigned long long *)&dbg[16 + q], (unsigned long long)c_l[q]);
    atomicAdd((unsigned long long *)&dbg[20], (unsigned long long)n_bulk);
    atomicAdd((unsigned long long *)&dbg[21], (unsigned long long)n_staged);
    atomicAdd((unsigned long long *)&dbg[22], (unsigned long long)c_g[0]);
    atomicAdd((unsigned long long *)&dbg[24], (unsigned long long)n_tab);
    atomicAdd((unsigned long long *)&dbg[23], (unsigned long long)c_g[1]);
    for (int q = 0; q < 3; q++) atomicAdd((unsigned long long *)&dbg[48 + q], (unsigned long long)c_p[q]);
    atomicAdd((unsigned long long *)&dbg[52], (unsigned long long)n_conf);
    atomicAdd((unsigned long long *)&dbg[53], (unsigned long long)n_slowc);
    atomicAdd((unsigned long long *)&dbg[54], (unsigned long long)n_void);
    atomicAdd((unsigned long long *)&dbg[55], (unsigned long long)c_cand);
    atomicAdd((unsigned long long *)&dbg[56], (unsigned long long)n_tready);
    atomicAdd((unsigned long long *)&dbg[58], (unsigned long long)c_gc[0]);
    atomicAdd((unsigned long long *)&dbg[59], (unsigned long long)c_gc[1]);
    atomicAdd((unsigned long long *)&dbg[60], (unsigned long long)c_gc[2]);
    atomicAdd((unsigned long long *)&dbg[61], (unsigned long long)n_ghit);
    atomicAdd((unsigned long long *)&dbg[62], (unsigned long long)c_chain);
    for (int q = 0; q < 4; q++) atomicAdd((unsigned long long *)&dbg[90 + q], (unsigned long long)c_ch[q]);
    atomicAdd((unsigned long long *)&dbg[107], (unsigned long long)c_rw[0]);
    atomicAdd((unsigned long long *)&dbg[108], (unsigned long long)c_rw[1]);
    atomicAdd((unsigned long long *)&dbg[109], (unsigned long long)n_chbm);
    atomicAdd((unsigned long long *)&dbg[112], (unsigned long long)c_rw[2]);
    atomicAdd((unsigned long long *)&dbg[113], (unsigned long long)c_rw[3]);
    atomicAdd((unsigned long long *)&dbg[30], (unsigned long long)c_ext);
    atomicAdd((unsigned long long *)&dbg[31], (unsigned long long)n_ext);
  }
}

// ---------------------------------------------------------------------------
// single-pod commit / uncommit (Reserve / Unreserve from the host)

__global__ void k_commit(DevCfg c, DevNodes d, const DevPod *__restrict__ pod, int32_t node, int32_t sign,
                         uint64_t *__restrict__ cpus, int32_t *__restrict__ rc) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const DevPod p = *pod;
  *rc = 0;
  NumaRowR8 rv{};
  if (c.resv) {
    load_resv(rv, d.rv, node);
    // Unreserve: whether the Reserve went into one of the node's reservations
    // (state.assumed, reservation/plugin.go:591-597) is not passed back
    if (sign < 0 && resv_matchable(rv, p)) {
      *rc = KOORDHIP_EINVAL;
      return;
    }
  }
  uint64_t m[NW] = {0, 0, 0, 0};
  if (numa_on(c) && numa_active(p, c)) {
    NumaRow r;
    load_numa_row(r, d, node);
    if (sign > 0) {
      uint64_t pref[NW];
      resv_pref_cpus(rv, p, (c.resv && (c.score & KOORDHIP_PLUGIN_RESERVATION)) ? resv_matched(rv, p) : 0u, pref);
      if (!numa_reserve<true>(d.nu.cls, r, p, m, pref)) {
        *rc = KOORDHIP_ERESERVE;  // Reserve fails: nothing is committed
        return;
      }
    } else if (topo_policy(r.nflags) != 0) {
      *rc = KOORDHIP_EINVAL;  // the zone amounts of the Reserve are not passed back
      return;
    } else if (is_cpuset(p)) {
      for (int w = 0; w < NW; w++) m[w] = cpus[w];
      numa_apply(r, p, m, sign);
    }
    store_numa_row(r, d, node);
    if (sign > 0)
      for (int w = 0; w < NW; w++) cpus[w] = m[w];
  } else if (sign > 0) {
    for (int w = 0; w < NW; w++) cpus[w] = 0;
  }
  if (c.resv && sign > 0) {  // Reservation Reserve: assumePod into the nominated reservation
    resv_assume(rv, p, m);
    store_resv(rv, d.rv, node);
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
template hipError_t launch_scatter<ZoneRow>(ZoneRow *, const ZoneRow *, const int32_t *, int32_t, hipStream_t);
template hipError_t launch_scatter<uint32_t>(uint32_t *, const uint32_t *, const int32_t *, int32_t, hipStream_t);
template hipError_t launch_scatter<uint16_t>(uint16_t *, const uint16_t *, const int32_t *, int32_t, hipStream_t);

// rows of `bytes` (a multiple of 4) per node: row j of src -> row idx[j] of dst
__global__ void k_scatter_rows(uint32_t *__restrict__ dst, const uint32_t *__restrict__ src,
                               const int32_t *__restrict__ idx, int32_t m, int32_t words) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)m * words) return;
  const int32_t j = (int32_t)(t / words), w = (int32_t)(t - (int64_t)j * words);
  dst[(size_t)idx[j] * words + w] = src[t];
}

hipError_t launch_scatter_rows(void *dst, const void *src, const int32_t *idx, int32_t m, int32_t bytes, hipStream_t s) {
  if (m <= 0) return hipSuccess;
  if (bytes % 4) return hipErrorInvalidValue;
  const int32_t words = bytes / 4;
  const int64_t tot = (int64_t)m * words;
  hipLaunchKernelGGL(k_scatter_rows, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, static_cast<uint32_t *>(dst),
                     static_cast<const uint32_t *>(src), idx, m, words);
  return hipGetLastError();
}
template hipError_t launch_scatter<double>(double *, const double *, const int32_t *, int32_t, hipStream_t);

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

// the template instantiation of the last evaluation / resolve launch of this
// host thread, spelled as rocprofv3 names it (bench.py matches the committed
// PMC summary against it)
static thread_local char g_eval_name[64], g_resolve_name[64];
template <typename... A>
static inline void note_kernel(char *dst, const char *fmt, A... a) {
  std::snprintf(dst, 64, fmt, a...);
}
const char *last_eval_kernel() { return g_eval_name; }
const char *last_resolve_kernel() { return g_resolve_name; }

int32_t scan_chunks(int R, int32_t lo, int32_t hi) { return hi > lo ? (hi - lo + 64 * R - 1) / (64 * R) : 0; }

int32_t scan_ppw(int R, int32_t lo, int32_t hi, int32_t n_pods) {
  const int32_t nq = (scan_chunks(R, lo, hi) + 3) / 4;
  if (nq <= 0 || n_pods <= 0) return 1;
  // ~2048 waves (2 per SIMD) over nq chunk quads x 4 waves
  const int32_t groups = std::max(1, std::min(n_pods, (2048 + 4 * nq - 1) / (4 * nq)));
  return (n_pods + groups - 1) / groups;
}

hipError_t launch_scan(int R, const DevCfg &c, const DevNodes &d, const DevPod *pods, int32_t n_pods, int32_t lo,
                       int32_t hi, uint16_t *S, int64_t s_stride, uint16_t *Mx, int32_t m_stride, int32_t ppw,
                       hipStream_t s) {
  if (n_pods <= 0 || hi <= lo) return hipSuccess;
  const int nm = side_mode(c);
  const bool numa = nm != 0;
  const int32_t nchunks = scan_chunks(R, lo, hi);
  const size_t lds = (numa && d.nu.ncls <= NUMA_LDS_CLASSES) ? (size_t)d.nu.ncls * sizeof(DevNumaClass) : 0;
  if (ppw > 0 && R <= 2 && nm < 4) {  // node-major (k_scan_nm)
    const int32_t cqx = ((nchunks + 3) / 4 + 7) / 8;
    const int32_t nblocks = 8 * cqx * ((n_pods + ppw - 1) / ppw);
#define KH_SCAN_NM(RR, NN)                                                                                          \
  note_kernel(g_eval_name, "kh::k_scan_nm<%d, %d>", RR, NN);                                                        \
  hipLaunchKernelGGL((k_scan_nm<RR, NN>), dim3(nblocks), dim3(256), lds, s, c, d, pods, n_pods, lo, hi, nchunks, cqx, \
                     ppw, S, s_stride, Mx, m_stride)
    switch (nm * 2 + (R - 1)) {
      case 0: KH_SCAN_NM(1, 0); break;
      case 1: KH_SCAN_NM(2, 0); break;
      case 2: KH_SCAN_NM(1, 1); break;
      case 3: KH_SCAN_NM(2, 1); break;
      case 4: KH_SCAN_NM(1, 2); break;
      case 5: KH_SCAN_NM(2, 2); break;
      case 6: KH_SCAN_NM(1, 3); break;
      case 7: KH_SCAN_NM(2, 3); break;
      default: return hipErrorInvalidValue;
    }
#undef KH_SCAN_NM
    return hipGetLastError();
  }
  const int32_t cpx = (nchunks + 7) / 8;
  const int32_t blocks = 8 * cpx * ((n_pods + 3) / 4);
  // pod-group-fastest block order once an XCD's eighth of the shard outgrows
  // what its L2 keeps across a sweep (measured: neutral at 50k nodes, +5 % at 200k)
  const int32_t pfast = (hi - lo) > kScanPodFastNodes ? 1 : 0;
#define KH_SCAN(RR, NN)                                                                                            \
  do {                                                                                                        \
    note_kernel(g_eval_name, "kh::k_scan<%d, %d>", RR, NN);                                                      \
    hipLaunchKernelGGL((k_scan<RR, NN>), dim3(blocks), dim3(256), lds, s, c, d, pods, n_pods, lo, hi, nchunks,  \
                       cpx, pfast, S, s_stride, Mx, m_stride);                                                  \
  } while (0)
  if (nm == 5) {
    switch (R) {
      case 4: KH_SCAN(4, 5); break;
      default: return hipErrorInvalidValue;
    }
  } else if (nm == 4) {
    switch (R) {
      case 4: KH_SCAN(4, 4); break;
      default: return hipErrorInvalidValue;
    }
  } else if (nm == 3) {
    switch (R) {
      case 1: KH_SCAN(1, 3); break;
      case 2: KH_SCAN(2, 3); break;
      case 4: KH_SCAN(4, 3); break;
      default: return hipErrorInvalidValue;
    }
  } else if (nm == 2) {
    switch (R) {
      case 1: KH_SCAN(1, 2); break;
      case 2: KH_SCAN(2, 2); break;
      case 4: KH_SCAN(4, 2); break;
      default: return hipErrorInvalidValue;
    }
  } else if (numa) {
    switch (R) {
      case 1: KH_SCAN(1, 1); break;
      case 2: KH_SCAN(2, 1); break;
      case 4: KH_SCAN(4, 1); break;
      default: return hipErrorInvalidValue;
    }
  } else {
    switch (R) {
      case 1: KH_SCAN(1, 0); break;
      case 2: KH_SCAN(2, 0); break;
      case 4: KH_SCAN(4, 0); break;
      case 8: KH_SCAN(8, 0); break;
      default: return hipErrorInvalidValue;
    }
  }
#undef KH_SCAN
  return hipGetLastError();
}

hipError_t launch_select(const uint16_t *S, int64_t s_stride, int32_t lo, int32_t m, int32_t n_pods, int32_t k,
                         int32_t nbins, const uint16_t *Mx, int32_t m_stride, int32_t nchunks, uint64_t *out,
                         uint64_t *dbg, hipStream_t s) {
  if (n_pods <= 0) return hipSuccess;
  if (k < 1 || k > RES_MAXP || nbins < 2 || nbins > 32768) return hipErrorInvalidValue;
  if (nchunks > 65535) nchunks = 0;  // no lower bound: histogram the whole row
  size_t lds = (size_t)nbins * sizeof(uint32_t);
  if (lds + (size_t)((nbins + 1) / 2) * sizeof(uint32_t) > 128 * 1024)
    nchunks = 0;  // chunk-max histogram does not fit beside the score histogram
  if (nchunks >= k) lds += (size_t)((nbins + 1) / 2) * sizeof(uint32_t);
  static bool attr = false;
  if (!attr) {
    const hipError_t e = hipFuncSetAttribute((const void *)k_select, hipFuncAttributeMaxDynamicSharedMemorySize, 131072);
    if (e != hipSuccess) return e;
    attr = true;
  }
  hipLaunchKernelGGL(k_select, dim3(n_pods), dim3(SEL_THREADS), lds, s, S, s_stride, lo, m, k, nbins, Mx, m_stride,
                     nchunks, out, dbg);
  return hipGetLastError();
}

int32_t select_split_groups(int32_t m, int32_t G) {
  const int32_t ntiles = std::max<int32_t>(1, (m + SPL_TILE - 1) / SPL_TILE);
  G = std::max<int32_t>(1, std::min<int32_t>(std::min<int32_t>(G, SPL_GMAX), ntiles));
  const int32_t per = (ntiles + G - 1) / G;
  return (ntiles + per - 1) / per;  // no workgroup without a tile
}

hipError_t launch_select_split(const uint16_t *S, int64_t s_stride, int32_t lo, int32_t m, int32_t n_pods, int32_t k,
                               int32_t nbins, const uint16_t *Mx, int32_t m_stride, int32_t nchunks, int32_t G,
                               uint64_t *part, uint32_t *cnt, uint64_t *out, PipeSync *sync, int32_t sel_par,
                               int32_t res_wait, hipStream_t s) {
  if (n_pods <= 0) return hipSuccess;
  if (k < 1 || k > RES_MAXP || nbins < 2 || nbins > 32768 || n_pods > kSelMaxPods) return hipErrorInvalidValue;
  const int32_t ntiles = std::max<int32_t>(1, (m + SPL_TILE - 1) / SPL_TILE);
  // large score ranges (Reservation ranking totals): u16-packed score bins,
  // with slices short enough that a count stays below 2^16
  const bool pk = nbins > 8192;
  if (pk)
    while (G < SPL_GMAX && (int64_t)((ntiles + G - 1) / G) * SPL_TILE >= 65536) G++;
  G = select_split_groups(m, G);
  const int32_t per = (ntiles + G - 1) / G;
  if (pk && (int64_t)per * SPL_TILE >= 65536) return hipErrorInvalidValue;
  if (nchunks > 65535) nchunks = 0;  // no lower bound: histogram the slices whole
  size_t hb = (size_t)(pk ? (nbins + 1) / 2 : nbins) * sizeof(uint32_t);
  if (hb + (size_t)((nbins + 1) / 2) * sizeof(uint32_t) > 136 * 1024) nchunks = 0;
  if (nchunks >= k) hb += (size_t)((nbins + 1) / 2) * sizeof(uint32_t);
  const size_t lds = (size_t)SPL_HDR + (((size_t)G * k * sizeof(uint64_t) + 15) & ~(size_t)15) + hb + 16;
  static bool attr[2] = {false, false};
  const void *fn = pk ? (const void *)k_select_split<true> : (const void *)k_select_split<false>;
  if (!attr[pk]) {
    const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr[pk] = true;
  }
  if (pk)
    hipLaunchKernelGGL(k_select_split<true>, dim3(G, n_pods), dim3(SPL_THREADS), lds, s, S, s_stride, lo, m, k, nbins,
                       Mx, m_stride, nchunks, G, per, part, cnt, out, sync, sel_par, res_wait);
  else
    hipLaunchKernelGGL(k_select_split<false>, dim3(G, n_pods), dim3(SPL_THREADS), lds, s, S, s_stride, lo, m, k, nbins,
                       Mx, m_stride, nchunks, G, per, part, cnt, out, sync, sel_par, res_wait);
  return hipGetLastError();
}

__global__ void k_empty_lists(uint64_t *out, int32_t n, PipeSync *sy, int32_t par, int32_t pods) {
  for (int32_t j = threadIdx.x; j < n; j += blockDim.x) st_wt(&out[j], (uint64_t)0);
  if (sy) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      __hip_atomic_fetch_add(&sy->sel[par], pods, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // stores sc1 + drained
    }
  }
}

int32_t eval_topk_slices(int VT, int32_t lo, int32_t hi) {
  const int32_t sl = ETK_THREADS * VT;
  return hi > lo ? (hi - lo + sl - 1) / sl : 0;
}

int eval_topk_vt(int nm, int32_t n_cu, int32_t n_pods, int32_t lo, int32_t hi, int32_t k) {
  if (const char *e = std::getenv("KOORDHIP_ETK_VT")) {
    const int v = std::atoi(e);
    if (v == 8 || v == 16 || v == 32) return eval_topk_slices(v, lo, hi) <= ETK_MAX_SLICES ? v : 32;
  }
  (void)nm;
  (void)n_cu;
  (void)n_pods;
  // the narrowest slices (most workgroups, shortest evaluation chains) whose
  // lists the merge still stages in LDS
  for (int v : {8, 16})
    if (eval_topk_slices(v, lo, hi) <= ETK_MAX_SLICES && (int64_t)eval_topk_slices(v, lo, hi) * k <= ETK_MERGE_KEYS)
      return v;
  return 32;
}

hipError_t launch_eval_topk(const DevCfg &c, const DevNodes &d, const DevPod *pods, int32_t n_pods, int32_t lo,
                            int32_t hi, int32_t k, int VT, uint64_t *part, int32_t *pcnt, uint32_t *arrive,
                            uint64_t *out, PipeSync *sync, int32_t sel_par, int32_t res_wait, uint64_t *dbg,
                            hipStream_t s) {
  if (n_pods <= 0) return hipSuccess;
  if (k < 1 || k > RES_MAXP || n_pods > kSelMaxPods) return hipErrorInvalidValue;
  const int32_t nslices = eval_topk_slices(VT, lo, hi);
  if (nslices > ETK_MAX_SLICES) return hipErrorInvalidValue;
  if (nslices == 0) {  // an empty shard: empty lists (and the pods counted in, like a merge would)
    hipLaunchKernelGGL(k_empty_lists, dim3(1), dim3(256), 0, s, out, n_pods * k, sync, sel_par, n_pods);
    return hipGetLastError();
  }
  const int nm = side_mode(c);
  // pods per workgroup (KOORDHIP_ETK_G: 1, 2 or 4; built for the plain, NUMA
  // and one-reservation plugin sets at 8 / 16 nodes per thread)
  int G = 1;
  if (const char *e = std::getenv("KOORDHIP_ETK_G")) G = std::atoi(e);
  if (!(G == 2 || G == 4) || VT == 32 || !(nm == 0 || nm == 1 || nm == 3)) G = 1;
  const int32_t sl = ETK_THREADS * VT;
  // merge staging: as many candidates as the slice lists can hold, up to ETK_MERGE_KEYS
  const int32_t stage_cap = (int32_t)std::min<int64_t>((int64_t)nslices * k, ETK_MERGE_KEYS);
  const size_t vbytes = (size_t)std::max<int32_t>(G * sl * 4, stage_cap * 8);
  const size_t lds = (size_t)ETK_HDR + vbytes +
                     ((nm != 0 && d.nu.ncls <= NUMA_LDS_CLASSES) ? (size_t)d.nu.ncls * sizeof(DevNumaClass) : 0);
  const int32_t spx = (nslices + 7) / 8;
  const int32_t blocks = 8 * spx * ((n_pods + G - 1) / G);
  static bool attr[6][3][5] = {};
  const int vi = VT == 8 ? 0 : (VT == 16 ? 1 : 2);
#define KH_ETK(NN, VV, RR, GG)                                                                                      \
  do {                                                                                                              \
    if (!attr[NN][vi][GG]) {                                                                                        \
      const hipError_t e = hipFuncSetAttribute((const void *)k_eval_topk<NN, VV, RR, GG>,                          \
                                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);             \
      if (e != hipSuccess) return e;                                                                                \
      attr[NN][vi][GG] = true;                                                                                      \
    }                                                                                                               \
    note_kernel(g_eval_name, "kh::k_eval_topk<%d, %d, %d, %d>", NN, VV, RR, GG);                                  \
    hipLaunchKernelGGL((k_eval_topk<NN, VV, RR, GG>), dim3(blocks), dim3(ETK_THREADS), lds, s, c, d, pods, n_pods,   \
                       lo, hi, nslices, spx, k, part, pcnt, arrive, out, sync, sel_par, res_wait, stage_cap, dbg);  \
  } while (0)
#define KH_ETK_G(NN, VV, RR)       \
  do {                             \
    if (G == 4)                    \
      KH_ETK(NN, VV, RR, 4);       \
    else if (G == 2)               \
      KH_ETK(NN, VV, RR, 2);       \
    else                           \
      KH_ETK(NN, VV, RR, 1);       \
  } while (0)
  // R: evaluations in flight per thread (all of a slice's for the plain plugin
  // set; the NUMA / Reservation rows are large: two or four at a time)
  switch (nm * 4 + vi) {
    case 0: KH_ETK_G(0, 8, 8); break;
    case 1: KH_ETK_G(0, 16, 8); break;
    case 2: KH_ETK(0, 32, 8, 1); break;
    case 4: KH_ETK_G(1, 8, 2); break;
    case 5: KH_ETK_G(1, 16, 2); break;
    case 6: KH_ETK(1, 32, 2, 1); break;
    case 8: KH_ETK(2, 8, 2, 1); break;
    case 9: KH_ETK(2, 16, 2, 1); break;
    case 10: KH_ETK(2, 32, 2, 1); break;
    case 12: KH_ETK_G(3, 8, ETK_R3); break;
    case 13: KH_ETK_G(3, 16, ETK_R3); break;
    case 14: KH_ETK(3, 32, ETK_R3, 1); break;
    case 16: KH_ETK(4, 8, 4, 1); break;
    case 17: KH_ETK(4, 16, 4, 1); break;
    case 18: KH_ETK(4, 32, 4, 1); break;
    case 20: KH_ETK(5, 8, 4, 1); break;
    case 21: KH_ETK(5, 16, 4, 1); break;
    case 22: KH_ETK(5, 32, 4, 1); break;
    default: return hipErrorInvalidValue;
  }
#undef KH_ETK_G
#undef KH_ETK
  return hipGetLastError();
}

hipError_t launch_topk_merge(const uint64_t *in, int64_t pod_stride, int64_t list_stride, int32_t n_pods, int32_t L,
                             int32_t k, int32_t score_bits, uint64_t *out, PipeSync *sync, int32_t sel_par,
                             hipStream_t s) {
  if (score_bits > 31 || L > MERGE_MAXL || k < 1) return hipErrorInvalidValue;
  const int32_t total = L * k;
  const size_t lds = L == 1 ? 0 : (size_t)(total <= MERGE_STAGE ? ((total * 8 + 1023) & ~1023) : 0) + (size_t)L * 4;
  static bool attr = false;
  if (!attr) {
    const hipError_t e = hipFuncSetAttribute((const void *)k_topk_merge, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
    if (e != hipSuccess) return e;
    attr = true;
  }
  hipLaunchKernelGGL(k_topk_merge, dim3(n_pods), dim3(MERGE_THREADS), lds, s, in, pod_stride, list_stride, L, k,
                     score_bits, out, sync, sel_par);
  return hipGetLastError();
}

// LDS list stride: k rounded up to 8 entries (zero padded)
static inline int32_t list_stride(int32_t k) { return (k + 7) & ~7; }

int side_mode(const DevCfg &c) {
  if (c.resv) return c.resv_cpus ? 5 : (c.resv_slots > 1 ? 4 : 3);
  if (!((c.filt | c.score) & KOORDHIP_PLUGIN_NUMA)) return 0;
  return c.zones ? 2 : 1;
}

static int32_t side_row_bytes(int nm) {
  return nm >= 4 ? (int32_t)sizeof(NumaRowR4) : nm == 3 ? (int32_t)sizeof(NumaRowR) : (nm ? (int32_t)sizeof(NumaRow) : 0);
}

int32_t resolve_lds_bytes(int32_t n_pods_max, int32_t k, int32_t n_nodes, int nm, int32_t lag) {
  const int32_t kp = list_stride(k);
  return res_lds(n_pods_max, kp, n_nodes, side_row_bytes(nm), false, false, lag, false, nm <= 2).total;
}

hipError_t launch_resolve(const DevCfg &c, const DevNodes &d, const DevNodes *d_desc, const DevPod *pods, int32_t total, int32_t P, int32_t k,
                          int32_t r_begin, int32_t r_end, const uint64_t *lists0, int64_t list_buf, int32_t monotone,
                          int32_t lag, PipeSync *sync, int32_t *mbuf, int32_t *out_node, uint64_t *out_cpus, uint64_t *dbg,
                          int32_t trace, hipStream_t s) {
  if (total <= 0 || r_end <= r_begin) return hipSuccess;
  if (P > RES_MAXP_ROUND || P < 1 || k > RES_MAXP || k < 1) return hipErrorInvalidValue;
  // lag 2 (one persistent launch): M' spans two rounds, lists hold >= 3P entries
  if (lag < 1 || lag > 2 || lag * P > RES_MAXP_ROUND || (lag > 1 && (k < 3 * P || r_begin != 0)))
    return hipErrorInvalidValue;
  const int32_t kp = list_stride(k);
  const int nm = side_mode(c);
  const int32_t nrow = side_row_bytes(nm);
  // a persistent launch preloads round r+1 during round r when both copies fit
  // the largest layout that fits: key tables and the next round's preload,
  // then without the preload, then without the tables
  const bool pre = r_end - r_begin > 1 && !std::getenv("KOORDHIP_NO_PRELOAD");
  const bool tab = !std::getenv("KOORDHIP_NO_KEY_TABLES");
  const bool wide = c.wide_keys != 0;
  const bool chain = nm <= 2;
  ResLds o = res_lds(P, kp, d.n, nrow, pre, tab, lag, wide, chain);
  if (o.total > RES_LDS_MAX) o = res_lds(P, kp, d.n, nrow, false, tab, lag, wide, chain);
  if (o.total > RES_LDS_MAX) o = res_lds(P, kp, d.n, nrow, pre, false, lag, wide, chain);
  if (o.total > RES_LDS_MAX) o = res_lds(P, kp, d.n, nrow, false, false, lag, wide, chain);
  static bool attr[12] = {};
  const int ai = nm * 2 + (dbg ? 1 : 0);
  if (!attr[ai]) {
    const void *f = dbg ? (nm == 5   ? (const void *)k_resolve<5, true>
                           : nm == 4 ? (const void *)k_resolve<4, true>
                           : nm == 3 ? (const void *)k_resolve<3, true>
                           : nm == 2 ? (const void *)k_resolve<2, true>
                                     : (nm == 1 ? (const void *)k_resolve<1, true> : (const void *)k_resolve<0, true>))
                        : (nm == 5   ? (const void *)k_resolve<5, false>
                           : nm == 4 ? (const void *)k_resolve<4, false>
                           : nm == 3 ? (const void *)k_resolve<3, false>
                           : nm == 2 ? (const void *)k_resolve<2, false>
                                     : (nm == 1 ? (const void *)k_resolve<1, false> : (const void *)k_resolve<0, false>));
    const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, RES_LDS_MAX);
    if (e != hipSuccess) return e;
    attr[ai] = true;
  }
  if (o.total > RES_LDS_MAX) return hipErrorInvalidValue;
#define KH_RESOLVE_D(NN, DD)                                                                                  \
  do {                                                                                                        \
    note_kernel(g_resolve_name, DD ? "kh::k_resolve<%d, true>" : "kh::k_resolve<%d, false>", NN);                \
    hipLaunchKernelGGL((k_resolve<NN, DD>), dim3(1), dim3(res_threads<NN>()), o.total, s, c, d_desc, d.n, d.nu.cls, \
                       pods, total, P, k, kp, r_begin, r_end, mbuf, lists0, list_buf, monotone, lag, sync, o, out_node, \
                       out_cpus, dbg, trace);                                                                   \
  } while (0)
#define KH_RESOLVE(NN)       \
  if (dbg)                   \
    KH_RESOLVE_D(NN, true);  \
  else                       \
    KH_RESOLVE_D(NN, false)
  if (nm == 5)
    KH_RESOLVE(5);
  else if (nm == 4)
    KH_RESOLVE(4);
  else if (nm == 3)
    KH_RESOLVE(3);
  else if (nm == 2)
    KH_RESOLVE(2);
  else if (nm == 1)
    KH_RESOLVE(1);
  else
    KH_RESOLVE(0);
#undef KH_RESOLVE
#undef KH_RESOLVE_D
  return hipGetLastError();
}

hipError_t launch_wait_resolved(PipeSync *sync, int32_t rounds, hipStream_t s) {
  hipLaunchKernelGGL(k_wait_resolved, dim3(1), dim3(64), 0, s, sync, rounds);
  return hipGetLastError();
}

hipError_t launch_signal_lists(PipeSync *sync, int32_t par, int32_t pods, hipStream_t s) {
  hipLaunchKernelGGL(k_signal_lists, dim3(1), dim3(64), 0, s, sync, par, pods);
  return hipGetLastError();
}

hipError_t launch_commit(const DevCfg &c, const DevNodes &d, const DevPod *pod, int32_t node, int32_t sign,
                         uint64_t *cpus, int32_t *rc, hipStream_t s) {
  hipLaunchKernelGGL(k_commit, dim3(1), dim3(64), 0, s, c, d, pod, node, sign, cpus, rc);
  return hipGetLastError();
}

}  // namespace kh
