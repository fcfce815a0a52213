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

__global__ void k_eval_full(DevCfg c, DevNodes d, const koordhip_pod *__restrict__ pods, int32_t n_pods,
                            uint8_t *__restrict__ status, int32_t *__restrict__ scores) {
  int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  int32_t p = blockIdx.y;
  if (i >= d.n || p >= n_pods) return;
  const koordhip_pod pod = pods[p];
  NV v{};
  load_node(v, d, i, need_all(c), c);
  if (status) {
    uint8_t b = 0;
    if ((c.filt & KOORDHIP_PLUGIN_FIT) && !fit_filter(pod, v)) b |= KOORDHIP_ST_FIT_FAIL;
    if ((c.filt & KOORDHIP_PLUGIN_LOADAWARE) && !la_filter(pod, v)) b |= KOORDHIP_ST_LA_FAIL;
    status[(size_t)p * d.n + i] = b;
  }
  if (scores) {
    int32_t *row = scores + (size_t)p * KOORDHIP_NPLUGINS * d.n;
    row[i] = (c.score & KOORDHIP_PLUGIN_FIT) ? fit_score(pod, v, c) : 0;
    row[(size_t)d.n + i] = (c.score & KOORDHIP_PLUGIN_LOADAWARE) ? la_score(pod, v, c) : 0;
    row[2 * (size_t)d.n + i] = 0;
  }
}

// ---------------------------------------------------------------------------
// k_topk_partial

__global__ __launch_bounds__(256) void k_topk_partial(DevCfg c, DevNodes d, const koordhip_pod *__restrict__ pods,
                                                      int32_t n_pods, int32_t lo, int32_t hi, int32_t chunk,
                                                      int32_t k, uint64_t *__restrict__ out) {
  const int lane = lane_id();
  const int wave = threadIdx.x >> 6;
  const int32_t p = blockIdx.y * (blockDim.x >> 6) + wave;
  if (p >= n_pods) return;  // wave-uniform
  const int32_t c0 = lo + blockIdx.x * chunk;
  const int32_t c1 = min(hi, c0 + chunk);
  const koordhip_pod pod = pods[p];
  const Need need = pod_needs(pod, c);
  uint64_t list = 0;  // rank `lane` of this chunk's running top-k (0 = empty)
  uint64_t thr = 0;   // current k-th key
  for (int32_t base = c0; base < c1; base += 64) {
    const int32_t i = base + lane;
    uint64_t key = 0;
    if (i < c1) {
      NV v;
      load_node(v, d, i, need, c);
      key = make_key(eval_total(pod, v, c), i);
    }
    uint64_t cand = __ballot(key > thr);
    while (cand) {  // rank-insert every key that beats the k-th
      const int src = __builtin_ctzll(cand);
      cand &= cand - 1;
      const uint64_t x = shfl_u64(key, src);
      if (x <= thr) continue;  // wave-uniform
      const int pos = __popcll(__ballot(list > x));
      const uint64_t up = shfl_up_u64(list, 1);
      if (lane > pos) list = up;
      if (lane == pos) list = x;
      if (lane >= k) list = 0;
      thr = shfl_u64(list, k - 1);
    }
  }
  if (lane < k) out[((size_t)p * gridDim.x + blockIdx.x) * k + lane] = list;
}

// ---------------------------------------------------------------------------
// k_topk_merge: per pod, exact top-k of L sorted lists of k keys.

constexpr int MERGE_THREADS = 256;
constexpr int MERGE_CAP = 2048;

__device__ __forceinline__ uint64_t block_max_u64(uint64_t v, uint64_t *red) {
  v = wave_max_u64(v);
  const int w = threadIdx.x >> 6;
  if (lane_id() == 0) red[w] = v;
  __syncthreads();
  uint64_t r = 0;
  for (int j = 0; j < (int)(blockDim.x >> 6); j++) r = red[j] > r ? red[j] : r;
  __syncthreads();
  return r;
}

__global__ __launch_bounds__(MERGE_THREADS) void k_topk_merge(const uint64_t *__restrict__ in, int64_t pod_stride,
                                                              int64_t list_stride, int32_t L, int32_t k,
                                                              uint64_t *__restrict__ out) {
  __shared__ uint64_t buf[MERGE_CAP];
  __shared__ uint64_t red[MERGE_THREADS / 64];
  __shared__ int32_t cnt;
  const int32_t p = blockIdx.x;
  const uint64_t *lists = in + (size_t)p * pod_stride;
  // 1. tau = max over lists of the k-th key: the global k-th key is >= tau.
  uint64_t t = 0;
  for (int32_t l = threadIdx.x; l < L; l += blockDim.x) {
    uint64_t x = lists[(size_t)l * list_stride + (k - 1)];
    t = x > t ? x : t;
  }
  const uint64_t tau = block_max_u64(t, red);
  if (threadIdx.x == 0) cnt = 0;
  __syncthreads();
  // 2. collect every key >= tau (and > 0)
  const int32_t total = L * k;
  for (int32_t j = threadIdx.x; j < total; j += blockDim.x) {
    uint64_t x = lists[(size_t)(j / k) * list_stride + (j % k)];
    if (x != 0 && x >= tau) {
      int32_t s = atomicAdd(&cnt, 1);
      if (s < MERGE_CAP) buf[s] = x;
    }
  }
  __syncthreads();
  const int32_t m = cnt;
  uint64_t *o = out + (size_t)p * k;
  if (m <= MERGE_CAP) {
    // 3. rank sort (keys are unique): rank = #keys greater
    for (int32_t j = threadIdx.x; j < m; j += blockDim.x) {
      const uint64_t x = buf[j];
      int32_t rank = 0;
      for (int32_t q = 0; q < m; q++) rank += buf[q] > x;
      if (rank < k) o[rank] = x;
    }
    for (int32_t j = m + threadIdx.x; j < k; j += blockDim.x) o[j] = 0;
  } else {
    // overflow: k rounds of "largest key below the previous one" over all keys
    uint64_t prev = ~0ull;
    for (int32_t r = 0; r < k; r++) {
      uint64_t b = 0;
      for (int32_t j = threadIdx.x; j < total; j += blockDim.x) {
        uint64_t x = lists[(size_t)(j / k) * list_stride + (j % k)];
        if (x < prev && x > b) b = x;
      }
      b = block_max_u64(b, red);
      if (threadIdx.x == 0) o[r] = b;
      prev = b;
    }
  }
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

constexpr int RES_MAXP = 64;
constexpr int RES_HASH = 256;

__device__ __forceinline__ int hash_find(const int32_t *ht_node, const int8_t *ht_row, int32_t node) {
  uint32_t h = ((uint32_t)node * 2654435761u) >> 24;  // 256 slots
  for (int probe = 0; probe < RES_HASH; probe++) {
    const int32_t x = ht_node[h];
    if (x == node) return ht_row[h];
    if (x < 0) return -1;
    h = (h + 1) & (RES_HASH - 1);
  }
  return -1;
}

__global__ __launch_bounds__(64) void k_resolve(DevCfg c, DevNodes d, const koordhip_pod *__restrict__ pods,
                                                int32_t n_pods, int32_t k, const uint64_t *__restrict__ lists,
                                                int32_t monotone, int32_t *__restrict__ out_node) {
  __shared__ NV rows[RES_MAXP];
  __shared__ int32_t row_node[RES_MAXP];
  __shared__ uint64_t lk[RES_MAXP * RES_MAXP];
  __shared__ koordhip_pod lp[RES_MAXP];
  __shared__ int32_t ht_node[RES_HASH];
  __shared__ int8_t ht_row[RES_HASH];
  const int lane = lane_id();
  for (int32_t j = lane; j < n_pods * k; j += 64) lk[j] = lists[j];
  {
    const uint64_t *src = reinterpret_cast<const uint64_t *>(pods);
    uint64_t *dst = reinterpret_cast<uint64_t *>(lp);
    const int32_t words = n_pods * (int32_t)(sizeof(koordhip_pod) / 8);
    for (int32_t j = lane; j < words; j += 64) dst[j] = src[j];
  }
  for (int32_t j = lane; j < RES_HASH; j += 64) ht_node[j] = -1;
  __syncthreads();
  int32_t nm = 0;  // modified rows this round (wave-uniform)
  for (int32_t j = 0; j < n_pods; j++) {
    const koordhip_pod pod = lp[j];
    const uint64_t e = lane < k ? lk[j * k + lane] : 0;
    bool mod = false;
    if (e != 0 && nm > 0) mod = hash_find(ht_node, ht_row, key_node(e)) >= 0;
    const uint64_t free_mask = __ballot(e != 0 && !mod);
    const int first = free_mask ? __builtin_ctzll(free_mask) : 64;
    uint64_t best = free_mask ? shfl_u64(e, first) : 0;
    const bool prefix_modified = __ballot(e != 0 && mod && lane < first) != 0;
    if (nm > 0 && (!monotone || prefix_modified)) {
      uint64_t key = 0;
      if (lane < nm) {
        const NV v = rows[lane];
        key = make_key(eval_total(pod, v, c), row_node[lane]);
      }
      key = wave_max_u64(key);
      best = key > best ? key : best;
    }
    if (best == 0) {
      if (lane == 0) out_node[j] = KOORDHIP_UNSCHEDULABLE;
      continue;
    }
    const int32_t w = key_node(best);
    if (lane == 0) out_node[j] = w;
    int32_t r = nm > 0 ? hash_find(ht_node, ht_row, w) : -1;  // uniform
    if (r < 0) {
      r = nm++;
      if (lane == 0) {
        NV v;
        load_row(v, d, w);
        rows[r] = v;
        row_node[r] = w;
        uint32_t h = ((uint32_t)w * 2654435761u) >> 24;
        while (ht_node[h] >= 0) h = (h + 1) & (RES_HASH - 1);
        ht_node[h] = w;
        ht_row[h] = (int8_t)r;
      }
    }
    if (lane == 0) {
      NV v = rows[r];
      apply_delta(v, pod, +1);
      rows[r] = v;
    }
    __syncthreads();
  }
  if (lane < nm) store_row(rows[lane], d, row_node[lane]);
}

// ---------------------------------------------------------------------------
// single-pod commit / uncommit (Reserve / Unreserve from the host)

__global__ void k_commit(DevNodes d, const koordhip_pod *__restrict__ pod, int32_t node, int32_t sign) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  NV v;
  load_row(v, d, node);
  apply_delta(v, *pod, sign);
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

hipError_t launch_eval_full(const DevCfg &c, const DevNodes &d, const koordhip_pod *pods, int32_t n_pods,
                            uint8_t *status, int32_t *scores, hipStream_t s) {
  if (n_pods <= 0 || d.n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_eval_full, dim3((d.n + 255) / 256, n_pods), dim3(256), 0, s, c, d, pods, n_pods, status,
                     scores);
  return hipGetLastError();
}

hipError_t launch_topk_partial(const DevCfg &c, const DevNodes &d, const koordhip_pod *pods, int32_t n_pods,
                               int32_t lo, int32_t hi, int32_t chunk, int32_t nchunks, int32_t k, uint64_t *out,
                               hipStream_t s) {
  dim3 grid(nchunks, (n_pods + 3) / 4);
  hipLaunchKernelGGL(k_topk_partial, grid, dim3(256), 0, s, c, d, pods, n_pods, lo, hi, chunk, k, out);
  return hipGetLastError();
}

hipError_t launch_topk_merge(const uint64_t *in, int64_t pod_stride, int64_t list_stride, int32_t n_pods, int32_t L,
                             int32_t k, uint64_t *out, hipStream_t s) {
  hipLaunchKernelGGL(k_topk_merge, dim3(n_pods), dim3(MERGE_THREADS), 0, s, in, pod_stride, list_stride, L, k, out);
  return hipGetLastError();
}

hipError_t launch_resolve(const DevCfg &c, const DevNodes &d, const koordhip_pod *pods, int32_t n_pods, int32_t k,
                          const uint64_t *lists, int32_t monotone, int32_t *out_node, hipStream_t s) {
  hipLaunchKernelGGL(k_resolve, dim3(1), dim3(64), 0, s, c, d, pods, n_pods, k, lists, monotone, out_node);
  return hipGetLastError();
}

hipError_t launch_commit(const DevNodes &d, const koordhip_pod *pod, int32_t node, int32_t sign, hipStream_t s) {
  hipLaunchKernelGGL(k_commit, dim3(1), dim3(64), 0, s, d, pod, node, sign);
  return hipGetLastError();
}

}  // namespace kh
