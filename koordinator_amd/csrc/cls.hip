// cls.hip -- class-incremental candidate lists: the pipelined greedy's
// evaluation when the staged pods fall into few classes.
//
// Pods whose device records are byte-identical (a ReplicaSet's replicas; in
// config 4 the 80 request / QoS shapes of the stream) rank every node the
// same way, and between two rounds a node's key changes only when the resolve
// commits a pod to it (every pipelined plugin's Filter / Score is a function
// of the node's own row: koord-scheduler's NodeResourcesFit, LoadAware,
// NodeNUMAResource and Reservation read no other node).  So instead of
// evaluating every node for every pod of every round (k_scan + k_select_split:
// P x n evaluations per round), each class keeps a buffer of its best keys:
//
//   build (k_scan of the class record + k_cls_collect, off the critical path
//   on the second stream): the best kClsTarget keys of the class on the state
//   after round tb - 1, sorted; every other node's key <= the boundary.
//   lists (k_cls_lists, one workgroup per class of round r): the commits of
//   the rounds the resolve finished since the buffer's base (its out_node log)
//   are re-evaluated for the class on their current rows -- a buffer key takes
//   the node's new value, a node outside whose key now exceeds the boundary is
//   inserted (a non-monotone Score can rise) -- the buffer is re-sorted by one
//   merge of the untouched run with the touched keys, and its first k keys are
//   the round's list for every pod of the class.
//
// Exactness: a node outside the buffer either was never committed since the
// build (key unchanged, <= boundary) or was re-evaluated from the log
// (inserted if above the boundary), so the buffer holds EVERY node whose key
// exceeds the boundary, with its key on the state the lists must reflect, and
// its sorted prefix is the exact top-k (ties: lowest node index, the key's low
// word).  The host schedules builds so that at most kClsTarget - k keys can
// leave the valid range (one per committed node) between a build and its last
// use; an underflow anyway (fewer than k keys above a nonzero boundary) stops
// the pipeline (sync->err = 2) instead of handing out a short list.
// Nodes the resolve is committing while a list is built (rounds >= r - lag)
// are its X set: their list keys are re-evaluated there, as with k_scan's.
#include <hip/hip_runtime.h>

#include "cls.h"
#include "pipe.hpp"
#include "rows.hpp"

namespace kh {

constexpr int CLS_THREADS = 512;
constexpr int CLS_WAVES = CLS_THREADS / 64;
constexpr int CLS_BUILD_THREADS = 1024;
constexpr int CLS_BUILD_WAVES = CLS_BUILD_THREADS / 64;

// block-wide exclusive prefix sum of v (every thread); *total = the sum
template <int WAVES>
__device__ __forceinline__ int32_t cls_scan(int32_t v, int32_t *wsum, int32_t *total) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  int32_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int32_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  int32_t off = 0, all = 0;
#pragma unroll
  for (int q = 0; q < WAVES; q++) {
    const int32_t s = wsum[q];
    off += q < w ? s : 0;
    all += s;
  }
  __syncthreads();  // wsum is reused by the next scan
  *total = all;
  return off + x - v;
}

// bitonic sort of a[0, n2) descending (n2 a power of two), all threads
template <int THREADS>
__device__ __forceinline__ void cls_sort_desc(uint64_t *a, int32_t n2) {
  for (int32_t k = 2; k <= n2; k <<= 1) {
    for (int32_t j = k >> 1; j > 0; j >>= 1) {
      for (int32_t i = threadIdx.x; i < n2; i += THREADS) {
        const int32_t x = i ^ j;
        if (x > i) {
          const uint64_t u = a[i], v = a[x];
          const bool down = (i & k) == 0;  // this run descending
          if (down ? (u < v) : (u > v)) {
            a[i] = v;
            a[x] = u;
          }
        }
      }
      __syncthreads();
    }
  }
}

// KOORDHIP_STAMPS: workgroup 0's phase cycles, accumulated per launch
struct ClsStamp {
  uint64_t *dbg;
  uint64_t t;
  __device__ __forceinline__ void lap(int q) {
    if (dbg && blockIdx.x == 0 && threadIdx.x == 0) {
      const uint64_t x = stamp();
      atomicAdd((unsigned long long *)&dbg[q], (unsigned long long)(x - t));
      t = x;
    }
  }
};

__device__ __forceinline__ uint64_t cls_key(uint32_t v, int32_t i) {
  return ((uint64_t)v << 32) | (uint64_t)(0xFFFFFFFFu - (uint32_t)i);
}

// one thread: spin (relaxed polls, s_sleep) until *p >= v, then ONE agent
// acquire; false when the pipeline's watchdog fires or it reported an error
__device__ __forceinline__ bool cls_wait_ge(const int32_t *p, int32_t v, PipeSync *sy) {
  const uint64_t t0 = stamp();
  while (__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < v) {
    if (__hip_atomic_load(&sy->err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return false;
    if (stamp() - t0 > PIPE_WATCHDOG) {
      __hip_atomic_store(&sy->err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    __builtin_amdgcn_s_sleep(4);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  return true;
}

// ---------------------------------------------------------------------------
// k_cls_collect: one workgroup per class of the build.  The row holds total + 1
// per node (0 = infeasible, < 2^15).  Thread t holds nodes i0 + 8t .. + 7 of
// every 8192-node tile, the first CLS_CT tiles in registers.  The threshold
// value v* = the largest v with at least `target` nodes >= v is found by a
// binary search of counting passes (ballot-free, atomic-free: ranking totals
// concentrate in a few values, where histogram atomics serialise); the buffer
// takes every key above v* (fewer than the target: block-scanned slots, then
// a bitonic sort) and the lowest-index ties at v* up to the target (in node
// order: one block scan per tile); the boundary is the largest key it leaves
// out.
constexpr int CLS_VPT = 8;
constexpr int32_t CLS_TILE = CLS_BUILD_THREADS * CLS_VPT;
constexpr int CLS_CT = 8;  // tiles held in registers (65536 nodes; larger rows re-read the rest per pass)

__device__ __forceinline__ uint4 cls_tile_load(const uint16_t *row, int32_t n, int32_t g) {
  const int32_t i = g * CLS_TILE + (int32_t)threadIdx.x * CLS_VPT;
  if (i + CLS_VPT <= n) return *reinterpret_cast<const uint4 *>(row + i);
  uint32_t w[4] = {0u, 0u, 0u, 0u};
  for (int u = 0; u < CLS_VPT; u++)
    if (i + u < n) w[u >> 1] |= (uint32_t)row[i + u] << (16 * (u & 1));
  return make_uint4(w[0], w[1], w[2], w[3]);
}
__device__ __forceinline__ uint32_t cls_val(const uint4 &q, int u) {
  const uint32_t w = u < 2 ? q.x : (u < 4 ? q.y : (u < 6 ? q.z : q.w));
  return (u & 1) ? (w >> 16) : (w & 0xFFFFu);
}

// f(tile g, its 8 values): every tile of the row, cached ones from registers
template <typename F>
__device__ __forceinline__ void cls_each_tile(const uint4 (&qc)[CLS_CT], const uint16_t *row, int32_t n, int32_t ntiles,
                                              F f) {
#pragma unroll
  for (int g = 0; g < CLS_CT; g++)
    if (g < ntiles) f(g, qc[g]);
  for (int32_t g = CLS_CT; g < ntiles; g++) f(g, cls_tile_load(row, n, g));
}

// bitonic sort of a[0, n2) descending, one compare-exchange pair per thread per
// step (n2 a power of two <= 2 * THREADS)
template <int THREADS>
__device__ __forceinline__ void cls_sort_pairs(uint64_t *a, int32_t n2) {
  const int32_t p = threadIdx.x;
  for (int32_t k = 2; k <= n2; k <<= 1) {
    for (int32_t j = k >> 1; j > 0; j >>= 1) {
      if (p < (n2 >> 1)) {
        const int32_t i = (p / j) * 2 * j + (p % j), x = i + j;
        const uint64_t u = a[i], v = a[x];
        const bool down = (i & k) == 0;
        if (down ? (u < v) : (u > v)) {
          a[i] = v;
          a[x] = u;
        }
      }
      __syncthreads();
    }
  }
}

__global__ __launch_bounds__(CLS_BUILD_THREADS) void k_cls_collect(const uint16_t *__restrict__ S, int64_t s_stride,
                                                                   int32_t n, const int32_t *__restrict__ ent,
                                                                   const int32_t *__restrict__ bm,
                                                                   const int32_t *__restrict__ bw, int32_t tb,
                                                                   uint64_t *__restrict__ bufs,
                                                                   ClsMeta *__restrict__ metas, ClsSync cs,
                                                                   uint64_t *dbg) {
  __shared__ uint64_t keys[kClsTarget];
  __shared__ uint64_t tie[kClsTarget];
  __shared__ int32_t wsum[CLS_BUILD_WAVES];
  __shared__ int32_t s_last;
  const int t = threadIdx.x;
  const int32_t e = ent[blockIdx.x];
  const int32_t slot = (e >> 1) * 2 + (e & 1);
  const uint16_t *row = S + (size_t)blockIdx.x * s_stride;
  ClsStamp st{dbg, dbg ? stamp() : 0};
  const int32_t ntiles = (n + CLS_TILE - 1) / CLS_TILE;
  uint4 qc[CLS_CT];
#pragma unroll
  for (int g = 0; g < CLS_CT; g++) qc[g] = g < ntiles ? cls_tile_load(row, n, g) : make_uint4(0u, 0u, 0u, 0u);
  if (t == 0) s_last = -1;
  // ---- the largest value and the feasible count
  uint32_t mx = 0;
  int32_t nf = 0;
  cls_each_tile(qc, row, n, ntiles, [&](int32_t, const uint4 &q) {
#pragma unroll
    for (int u = 0; u < CLS_VPT; u++) {
      const uint32_t v = cls_val(q, u);
      mx = v > mx ? v : mx;
      nf += v != 0u;
    }
  });
  int32_t feas;
  (void)cls_scan<CLS_BUILD_WAVES>(nf, wsum, &feas);
  int32_t vmax;
  {
    int32_t m = (int32_t)mx;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) m = max(m, __shfl_xor(m, d, 64));
    if ((t & 63) == 0) wsum[t >> 6] = m;
    __syncthreads();
    vmax = 0;
#pragma unroll
    for (int q = 0; q < CLS_BUILD_WAVES; q++) vmax = max(vmax, wsum[q]);
    __syncthreads();
  }
  st.lap(8);
  // ---- v*: the largest v with count(>= v) >= target (every feasible node when there are fewer)
  const int32_t tgt = kClsTarget;
  const bool all = feas <= tgt;  // block-uniform
  auto count_ge = [&](uint32_t x) -> int32_t {
    int32_t c = 0;
    cls_each_tile(qc, row, n, ntiles, [&](int32_t, const uint4 &q) {
#pragma unroll
      for (int u = 0; u < CLS_VPT; u++) c += cls_val(q, u) >= x;
    });
    int32_t tot;
    (void)cls_scan<CLS_BUILD_WAVES>(c, wsum, &tot);
    return tot;
  };
  uint32_t vstar = 0;
  int32_t G = feas;
  if (!all) {
    int32_t lo = 1, hi = vmax;  // count(>= lo) >= tgt holds
    while (lo < hi) {
      const int32_t mid = (lo + hi + 1) >> 1;
      if (count_ge((uint32_t)mid) >= tgt)
        lo = mid;
      else
        hi = mid - 1;
    }
    vstar = (uint32_t)lo;
    G = count_ge(vstar + 1u);
  }
  const int32_t need = all ? 0 : tgt - G;
  st.lap(9);
  // ---- keys above v*: block-scanned slots
  {
    int32_t c = 0;
    cls_each_tile(qc, row, n, ntiles, [&](int32_t, const uint4 &q) {
#pragma unroll
      for (int u = 0; u < CLS_VPT; u++) c += cls_val(q, u) > vstar;
    });
    int32_t tot;
    int32_t pos = cls_scan<CLS_BUILD_WAVES>(c, wsum, &tot);
    cls_each_tile(qc, row, n, ntiles, [&](int32_t g, const uint4 &q) {
#pragma unroll
      for (int u = 0; u < CLS_VPT; u++) {
        const uint32_t v = cls_val(q, u);
        if (v > vstar) keys[pos++] = cls_key(v, g * CLS_TILE + t * CLS_VPT + u);
      }
    });
  }
  // ---- the lowest-index ties at v*, in node order
  int32_t ties = 0;  // block-uniform
  cls_each_tile(qc, row, n, ntiles, [&](int32_t g, const uint4 &q) {
    if (ties >= need) return;
    int32_t c = 0;
#pragma unroll
    for (int u = 0; u < CLS_VPT; u++) c += (cls_val(q, u) == vstar && vstar != 0u) ? 1 : 0;
    int32_t tot;
    int32_t pos = ties + cls_scan<CLS_BUILD_WAVES>(c, wsum, &tot);
    int32_t last = -1;
#pragma unroll
    for (int u = 0; u < CLS_VPT; u++) {
      if (cls_val(q, u) == vstar && vstar != 0u) {
        const int32_t i = g * CLS_TILE + t * CLS_VPT + u;
        if (pos < need) {
          tie[pos] = cls_key(vstar, i);
          last = i;
        }
        pos++;
      }
    }
    if (last >= 0) atomicMax(&s_last, last);
    ties += tot;
  });
  int32_t n2 = 1;
  while (n2 < G) n2 <<= 1;
  for (int32_t j = G + t; j < n2; j += CLS_BUILD_THREADS) keys[j] = 0ull;
  __syncthreads();
  st.lap(10);
  cls_sort_pairs<CLS_BUILD_THREADS>(keys, n2);
  st.lap(11);
  const int32_t cnt = all ? feas : tgt;
  // the slot's previous build: its class's workgroup must have copied it into
  // its LDS (it reads a slot only when it switches to it) -- bw[b] switches
  if (t == 0) {
    if (bw[blockIdx.x] > 0 && !cls_wait_ge(cs.sw + (e >> 1), bw[blockIdx.x], cs.sy)) wsum[0] = -1;
  }
  __syncthreads();
  if (wsum[0] == -1) return;  // the pipeline gave up
  uint64_t *gb = bufs + (size_t)slot * kClsCap;
  for (int32_t j = t; j < cnt; j += CLS_BUILD_THREADS) gb[j] = j < G ? keys[j] : tie[j - G];
  if (t == 0) {
    ClsMeta m;
    m.boundary = all ? 0ull : ((uint64_t)vstar << 32) | (uint64_t)(0xFFFFFFFFu - (uint32_t)(s_last + 1));
    m.cnt = cnt;
    m.base = tb;
    metas[slot] = m;
  }
  // publish (Guideline 16, release form): every storing wave drains, then one
  // agent release and the class's build counter
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(cs.done + (e >> 1), bm[blockIdx.x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  st.lap(12);
  if (dbg && blockIdx.x == 0 && t == 0) atomicAdd((unsigned long long *)&dbg[15], 1ull);
}

// ---------------------------------------------------------------------------
// k_cls_run: one persistent workgroup per class (see cls.h).  Dynamic LDS:
// bk[kClsCap] (the buffer, resident for the whole call), ob[kClsCap] (the
// untouched run; scratch), chg[kClsCap] (touched flags), the log bitmap and,
// for a non-monotone configuration, the buffer's node bitmap.
struct ClsLds {
  int32_t ins, over, stop, cnt, base;
  uint64_t bnd;
  int32_t wsum[CLS_WAVES];
};

template <int NM>
__global__ __launch_bounds__(CLS_THREADS) void k_cls_run(DevCfg c, DevNodes d, const DevPod *__restrict__ cls_pod,
                                                         const int32_t *__restrict__ coff,
                                                         const int32_t *__restrict__ csched,
                                                         const int32_t *__restrict__ csm,
                                                         const int32_t *__restrict__ pod_cls,
                                                         const int32_t *__restrict__ out_node, int32_t lag, int32_t P,
                                                         int32_t total, const uint64_t *__restrict__ bufs,
                                                         const ClsMeta *__restrict__ metas, int32_t k, int32_t monotone,
                                                         uint64_t *__restrict__ lists0, int64_t list_buf, ClsSync cs,
                                                         uint64_t *dbg) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  __shared__ ClsLds h;
  uint64_t *bk = reinterpret_cast<uint64_t *>(lds);
  uint64_t *ob = bk + kClsCap;
  uint8_t *chg = reinterpret_cast<uint8_t *>(ob + kClsCap);
  uint32_t *lg = reinterpret_cast<uint32_t *>(chg + kClsCap);
  const int32_t words = (d.n + 31) >> 5;
  uint32_t *mb = lg + words;
  const int t = threadIdx.x;
  constexpr int PER = kClsCap / CLS_THREADS;  // 8 consecutive entries per thread
  PipeSync *sy = cs.sy;
  const int32_t cl = blockIdx.x;
  const DevPod pod = cls_pod[cl];
  const DevNumaClass *ncls = d.nu.cls;
  auto eval_key = [&](int32_t y) -> uint64_t {
    NV v;
    load_row(v, d, y);
    side_row_t<NM> nr;
    if constexpr (NM != 0) load_side_row<NM>(nr, d, y);
    return make_key(eval_row<NM>(pod, v, nr, ncls, c), y);
  };
  for (int32_t w = t; w < words; w += CLS_THREADS) {
    lg[w] = 0u;
    if (!monotone) mb[w] = 0u;
  }
  if (t == 0) atomicAdd(cs.rcnt + kClsRoundRing, 1);  // workgroups started (diagnostics: api.hip pipe_status)
  int32_t nsw = 0;  // switches to a new build so far
  uint32_t nev = 0;  // evaluations from the commit log (counted into cs.evc at the end)
  for (int32_t ix = coff[cl]; ix < coff[cl + 1]; ix++) {
    const int32_t ent = csched[ix];
    const int32_t u = ent & 0x7FFFFFFF;
    ClsStamp st{dbg, dbg ? stamp() : 0};
    if (ent < 0) {  // ---- switch to build csm[ix]: wait for it, copy it into LDS
      const int32_t m = csm[ix];
      const int32_t slot = cl * 2 + ((m - 1) & 1);
      if (t == 0) {
        cs.rcnt[kClsRoundRing + 1 + cl] = (u << 4) | 1;  // (diagnostics: where each workgroup waits)
        h.stop = cls_wait_ge(cs.done + cl, m, sy) ? 0 : 1;
      }
      __syncthreads();
      if (h.stop) return;
      const ClsMeta mt = metas[slot];
      const int32_t cnt = mt.cnt;
      const uint4 *g4 = reinterpret_cast<const uint4 *>(bufs + (size_t)slot * kClsCap);
      constexpr int LP = kClsCap / 2 / CLS_THREADS;
      const int32_t c16 = (cnt + 1) >> 1;
      uint4 q[LP];
#pragma unroll
      for (int v = 0; v < LP; v++) {
        const int32_t x = t + v * CLS_THREADS;
        if (x < c16) q[v] = g4[x];
      }
#pragma unroll
      for (int v = 0; v < LP; v++) {
        const int32_t x = t + v * CLS_THREADS;
        if (x < c16) {
          bk[2 * x] = ((uint64_t)q[v].y << 32) | q[v].x;
          if (2 * x + 1 < cnt) bk[2 * x + 1] = ((uint64_t)q[v].w << 32) | q[v].z;
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      nsw++;
      if (t == 0) {
        h.cnt = cnt;
        h.base = mt.base;
        h.bnd = mt.boundary;
        // the slot may be rebuilt now (k_cls_collect waits for this count)
        __hip_atomic_store(cs.sw + cl, nsw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    if (t == 0) {
      h.ins = 0;
      h.over = 0;
      h.stop = 0;
      // round u's lists reflect the commits of the rounds < u - lag (one agent
      // acquire after the poll, then the barrier, before any wave reads the log or a row)
      cs.rcnt[kClsRoundRing + 1 + cl] = (u << 4) | 2;
      if (u > lag && !wait_at_least(&sy->res_round, u - lag, sy)) h.stop = 1;
    }
    __syncthreads();
    if (h.stop) return;  // the pipeline gave up (watchdog / error): the host reports it
    const int32_t cnt = h.cnt, base = h.base;
    const uint64_t bnd = h.bnd;
    for (int32_t j = t; j < cnt; j += CLS_THREADS) chg[j] = 0;
    st.lap(0);
    // ---- the log: the nodes committed in rounds [base, u - lag)
    const int32_t plo = base * P, phi = min(total, (u - lag) * P);
    int32_t touched = 0;
    for (int32_t p0 = plo + t; p0 < phi; p0 += 4 * CLS_THREADS) {  // four loads in flight
      int32_t y[4];
#pragma unroll
      for (int v = 0; v < 4; v++) y[v] = p0 + v * CLS_THREADS < phi ? out_node[p0 + v * CLS_THREADS] : -1;
#pragma unroll
      for (int v = 0; v < 4; v++)
        if (y[v] >= 0) {
          atomicOr(&lg[y[v] >> 5], 1u << (y[v] & 31));
          touched = 1;
        }
    }
    if (!monotone)
      for (int32_t j = t; j < cnt; j += CLS_THREADS) {
        const int32_t y = key_node(bk[j]);
        atomicOr(&mb[y >> 5], 1u << (y & 31));
      }
    bool any = __syncthreads_or(touched) != 0;  // the log touched the buffer's rounds
    st.lap(1);
    int32_t ntot = cnt;
    if (any) {
      int32_t moved = 0;
      // ---- touched buffer keys, gathered first (then one evaluation per thread:
      //      the touched rows' loads are one round trip)
      int32_t *tj = reinterpret_cast<int32_t *>(ob);  // scratch until the compaction
      {
        int32_t myc = 0;
        uint32_t hitm = 0u;
  #pragma unroll
        for (int q = 0; q < PER; q++) {
          const int32_t j = t * PER + q;
          if (j < cnt) {
            const int32_t y = key_node(bk[j]);
            if ((lg[y >> 5] >> (y & 31)) & 1u) {
              hitm |= 1u << q;
              myc++;
            }
          }
        }
        int32_t ntouch;
        int32_t pos = cls_scan<CLS_WAVES>(myc, h.wsum, &ntouch);
  #pragma unroll
        for (int q = 0; q < PER; q++)
          if ((hitm >> q) & 1u) tj[pos++] = t * PER + q;
        __syncthreads();
        for (int32_t x = t; x < ntouch; x += CLS_THREADS) {
          const int32_t j = tj[x];
          bk[j] = eval_key(key_node(bk[j]));
          chg[j] = 1;
        }
        nev += (uint32_t)ntouch * (t == 0);
        moved = ntouch > 0 ? 1 : 0;
      }
      // ---- (non-monotone) committed nodes outside the buffer whose key rose above the boundary
      if (!monotone) {
        for (int32_t w = t; w < words; w += CLS_THREADS) {
          uint32_t bits = lg[w] & ~mb[w];
          while (bits) {
            const int32_t y = w * 32 + __builtin_ctz(bits);
            bits &= bits - 1u;
            const uint64_t key = eval_key(y);
            nev++;
            if (key > bnd) {
              const int32_t pos = cnt + atomicAdd(&h.ins, 1);
              moved = 1;
              if (pos < kClsCap) {
                bk[pos] = key;
                chg[pos] = 1;
              } else {
                h.over = 1;
              }
            }
          }
        }
      }
      any = __syncthreads_or(moved) != 0;
      st.lap(2);
    }
    if (any) {  // some key moved: re-sort
      ntot = min(kClsCap, cnt + h.ins);
      // ---- re-sort: the untouched keys keep their order (ob[0, na)); the touched
      //      ones still above the boundary (U) are compacted to bk[0, nu), sorted,
      //      and merged back in: every key's rank = its rank in its own run + the
      //      keys of the other run above it (keys are unique)
      // each thread holds 8 consecutive entries; one block scan of the packed
      // (untouched, touched-and-valid) counts places them in index order
      uint64_t xv[PER];
      uint32_t am = 0u, um = 0u;
      int32_t ca = 0, cu = 0;
  #pragma unroll
      for (int q = 0; q < PER; q++) {
        const int32_t j = t * PER + q;
        xv[q] = j < ntot ? bk[j] : 0ull;
        const bool isa = j < ntot && !chg[j];
        const bool isu = j < ntot && chg[j] && xv[q] > bnd;
        am |= (isa ? 1u : 0u) << q;
        um |= (isu ? 1u : 0u) << q;
        ca += isa;
        cu += isu;
      }
      int32_t tot;
      const int32_t pp = cls_scan<CLS_WAVES>(ca | (cu << 16), h.wsum, &tot);  // (every read of bk precedes its barriers)
      int32_t pa = pp & 0xFFFF, pu = pp >> 16;
  #pragma unroll
      for (int q = 0; q < PER; q++) {
        if ((am >> q) & 1u) ob[pa++] = xv[q];
        if ((um >> q) & 1u) bk[pu++] = xv[q];
      }
      __syncthreads();
      const int32_t runa = tot & 0xFFFF, runu = tot >> 16;
      const int32_t na = runa, nu = runu;
      st.lap(3);
      if (nu > 0) {
        int32_t n2 = 1;
        while (n2 < nu) n2 <<= 1;
        for (int32_t j = nu + t; j < n2; j += CLS_THREADS) bk[j] = 0ull;
        __syncthreads();
        cls_sort_desc<CLS_THREADS>(bk, n2);
        st.lap(4);
        // rank of x among the keys of a sorted-descending run s[0, len): keys above x
        auto above = [](const uint64_t *s, int32_t len, uint64_t x) -> int32_t {
          int32_t lo = 0, hi = len;
          while (lo < hi) {
            const int32_t mid = (lo + hi) >> 1;
            if (s[mid] > x)
              lo = mid + 1;
            else
              hi = mid;
          }
          return lo;
        };
        uint64_t xa[PER], xu[PER];
        int32_t ia[PER], iu[PER];
  #pragma unroll
        for (int q = 0; q < PER; q++) {
          const int32_t j = t + q * CLS_THREADS;
          xa[q] = j < na ? ob[j] : 0ull;
          ia[q] = j < na ? j + above(bk, nu, xa[q]) : -1;
          xu[q] = j < nu ? bk[j] : 0ull;
          iu[q] = j < nu ? j + above(ob, na, xu[q]) : -1;
        }
        __syncthreads();
  #pragma unroll
        for (int q = 0; q < PER; q++) {
          if (ia[q] >= 0) bk[ia[q]] = xa[q];
          if (iu[q] >= 0) bk[iu[q]] = xu[q];
        }
      } else {
        for (int32_t j = t; j < na; j += CLS_THREADS) bk[j] = ob[j];
      }
      ntot = na + nu;
      __syncthreads();
      st.lap(5);
    }

    // ---- clear the log's bits (and the buffer's, non-monotone) for the next appearance
    for (int32_t p0 = plo + t; p0 < phi; p0 += CLS_THREADS) {
      const int32_t y = out_node[p0];
      if (y >= 0) lg[y >> 5] = 0u;
    }
    if (!monotone)
      for (int32_t w = t; w < words; w += CLS_THREADS) mb[w] = 0u;
    // ---- round u's lists: the first k keys, for every pod of the class
    const bool under = ntot < k && bnd != 0ull;
    uint64_t *lists = lists0 + (size_t)(u & (2 * lag - 1)) * list_buf;
    const int32_t p0 = u * P, np = min(P, total - p0);
    int32_t mine = 0;
    for (int32_t j = 0; j < np; j++) {
      if (pod_cls[p0 + j] != cl) continue;  // uniform
      mine++;
      for (int32_t q = t; q < k; q += CLS_THREADS) st_wt(&lists[(size_t)j * k + q], (uint64_t)(q < ntot ? bk[q] : 0ull));
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) {
      if (under || h.over) {
        __hip_atomic_store(&sy->err, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else if (mine) {
        // the resolve counts finished lists per round parity, cumulatively: a
        // round is added only as a whole, by its last class, and only after the
        // previous round of its parity (classes run ahead of each other)
        int32_t *rc = cs.rcnt + (u & (kClsRoundRing - 1));
        const int32_t old = __hip_atomic_fetch_add(rc, mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old + mine == np) {
          __hip_atomic_store(rc, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          cs.rcnt[kClsRoundRing + 1 + cl] = (u << 4) | 3;
          if (!cls_wait_ge(&sy->sel[u & 1], P * (u >> 1), sy)) h.stop = 1;
          else __hip_atomic_fetch_add(&sy->sel[u & 1], np, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      h.cnt = ntot;
      h.base = max(base, u - lag);
      cs.rcnt[kClsRoundRing + 1 + cl] = (u << 4) | 4;  // round u published
    }
    __syncthreads();
    if (under || h.over || h.stop) return;
    st.lap(6);
    if (dbg && cl == 0 && t == 0) atomicAdd((unsigned long long *)&dbg[7], 1ull);
  }
  if (nev) atomicAdd(cs.evc, nev);
}

hipError_t launch_cls_collect(const uint16_t *S, int64_t s_stride, int32_t n, const int32_t *ent, const int32_t *bm,
                              const int32_t *bw, int32_t nb, int32_t tb, uint64_t *bufs, ClsMeta *metas,
                              const ClsSync &cs, uint64_t *dbg, hipStream_t s) {
  if (nb <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_cls_collect, dim3(nb), dim3(CLS_BUILD_THREADS), 0, s, S, s_stride, n, ent, bm, bw, tb, bufs, metas,
                     cs, dbg);
  return hipGetLastError();
}

size_t cls_run_lds(int32_t n, int32_t monotone) {
  const size_t words = ((size_t)n + 31) / 32;
  return (size_t)kClsCap * (8 + 8 + 1) + words * 4 * (monotone ? 1 : 2);
}

hipError_t launch_cls_run(const DevCfg &c, const DevNodes &d, const DevPod *cls_pod, int32_t n_cls, const int32_t *coff,
                          const int32_t *csched, const int32_t *csm, const int32_t *pod_cls, const int32_t *out_node,
                          int32_t lag, int32_t P, int32_t total, const uint64_t *bufs, const ClsMeta *metas, int32_t k,
                          int32_t monotone, uint64_t *lists0, int64_t list_buf, const ClsSync &cs, uint64_t *dbg,
                          hipStream_t s) {
  if (n_cls <= 0) return hipSuccess;
  const size_t lds = cls_run_lds(d.n, monotone);
  if (lds > 150 * 1024) return hipErrorInvalidValue;
  const int nm = side_mode(c);
#define KH_CLS(NN)                                                                                                   \
  do {                                                                                                               \
    static bool attr = false;                                                                                        \
    if (!attr) {                                                                                                     \
      if (hipError_t e = hipFuncSetAttribute((const void *)k_cls_run<NN>,                                            \
                                             hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024))                \
        return e;                                                                                                    \
      attr = true;                                                                                                   \
    }                                                                                                                \
    hipLaunchKernelGGL(k_cls_run<NN>, dim3(n_cls), dim3(CLS_THREADS), lds, s, c, d, cls_pod, coff, csched, csm,      \
                       pod_cls, out_node, lag, P, total, bufs, metas, k, monotone, lists0, list_buf, cs, dbg);      \
  } while (0)
  switch (nm) {
    case 0: KH_CLS(0); break;
    case 1: KH_CLS(1); break;
    case 2: KH_CLS(2); break;
    case 3: KH_CLS(3); break;
    case 4: KH_CLS(4); break;
    case 5: KH_CLS(5); break;
    default: return hipErrorInvalidValue;
  }
#undef KH_CLS
  return hipGetLastError();
}

const char *cls_run_kernel_name(const DevCfg &c) {
  static const char *names[6] = {"kh::k_cls_run<0>", "kh::k_cls_run<1>", "kh::k_cls_run<2>",
                                 "kh::k_cls_run<3>", "kh::k_cls_run<4>", "kh::k_cls_run<5>"};
  const int nm = side_mode(c);
  return names[nm >= 0 && nm < 6 ? nm : 0];
}

}  // namespace kh
