// pts.hpp -- upstream PodTopologySpread (k8s v1.24 pkg/scheduler/framework/
// plugins/podtopologyspread; not vendored in the reference) for the
// sequential cycle (seq.hip).  Restated in oracle/pts_oracle.c, which is the
// checker; koordinator_amd/topologyspread.py builds the columns.
//
// Device model.  Domains are small integers per topology key (< 64; the
// node itself for kubernetes.io/hostname).  Every workgroup keeps, in LDS, a
// replica of the cluster-wide pair counters the plugin sums over ALL nodes:
//   fsum[c][d]     matching pods of table constraint c in domain d (Filter:
//                  calPreFilterState counts every node of a present pair)
//   ssum[s][c][d]  ... over the nodes soft-eligible for spread class s (Score:
//                  processAllNode counts the nodes matching the pod's required
//                  affinity that carry every soft key)
//   fpres[s][k]    the domains of key k holding a node hard-eligible for class
//                  s (the pairs of TpPairToMatchNum)
// built once per launch from the columns and advanced identically by every
// workgroup on every commit (the winner, its domains and eligibility bits are
// known to all: no cross-workgroup reads).  Hostname pairs are per node: the
// node's own count column, read only by its owner workgroup; their minimum
// (criticalPaths) is a grid reduction of its own.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dev.hpp"

namespace kh {

constexpr int PD = KOORDHIP_PTS_DOMAINS, PK = KOORDHIP_PTS_KEYS, PC = KOORDHIP_PTS_CONS, PS = KOORDHIP_PTS_CLASSES,
              PP = KOORDHIP_PTS_POD;

struct PtsArgs {
  const int32_t *dom;    // [keys][n]
  int32_t *cnt;          // [cons][n] (advanced by the owner's Reserve)
  const uint16_t *elig;  // [n]
  int32_t keys, cons, classes;
  uint32_t host;         // bit k: key k is kubernetes.io/hostname
  int32_t filt, score;   // the plugin's Filter / Score are enabled (and the snapshot has tables)
  int32_t w;             // Score weight
  int32_t cons_key[PC];
};

struct PtsLds {
  int32_t fsum[PC][PD];
  int32_t ssum[PS][PC][PD];
  uint32_t fpres[PS][PK][2];
  int32_t fmatch[PK][PD];   // per pod: the pair counters of its hard keys
  int32_t fmin[PK];
  int32_t smatch[PK][PD];   // per pod: the pair counters of its soft keys
  uint32_t smask[PK][2];    // per pod: domains of this workgroup's feasible, non-ignored nodes
  int32_t nfni;             // ... and their count
  int32_t red[2];           // min / max scratch
};

// One pod's constraints in its own order (wave-uniform).  Every loop over
// them runs j = 0 .. PP-1 unrolled under the hard / soft masks: with static
// indices the arrays stay in registers (a dynamically indexed array lives in
// scratch, one memory round trip per access).
struct PtsPod {
  int32_t cls, nh, ns;
  int32_t c[PP], k[PP], skew[PP], self[PP];
  uint32_t hard, soft;  // bit j: constraint j is a DoNotSchedule / ScheduleAnyway one the plugin evaluates
  uint32_t hkeys, skeys;
  bool on, hhost;
};

__device__ __forceinline__ PtsPod pts_pod(const PtsArgs &pa, const DevPodX &x) {
  PtsPod q{};
  q.on = (pa.filt || pa.score) && pa.keys > 0 && x.pts_n > 0;
  if (!q.on) return q;
  q.cls = x.pts_class;
#pragma unroll
  for (int j = 0; j < PP; j++) {
    if (j >= x.pts_n) continue;
    const int c = x.pts_c[j], k = pa.cons_key[c];
    q.c[j] = c;
    q.k[j] = k;
    q.skew[j] = x.pts_skew[j];
    q.self[j] = (x.pts_fl[j] & KOORDHIP_PTS_SELF) ? 1 : 0;
    if (x.pts_fl[j] & KOORDHIP_PTS_HARD) {
      if (!pa.filt) continue;
      q.hard |= 1u << j;
      q.hkeys |= 1u << k;
      q.hhost |= ((pa.host >> k) & 1u) != 0;
      q.nh++;
    } else {
      if (!pa.score) continue;
      q.soft |= 1u << j;
      q.skeys |= 1u << k;
      q.ns++;
    }
  }
  return q;
}

__device__ __forceinline__ bool pts_bit(const uint32_t (&m)[2], int32_t d) { return (m[d >> 5] >> (d & 31)) & 1u; }

// The launch's replicated counters (every thread of the workgroup takes part).
__device__ __forceinline__ void pts_init(const PtsArgs &pa, int32_t n, PtsLds &L, int t, int nt) {
  for (int x = t; x < PC * PD; x += nt) (&L.fsum[0][0])[x] = 0;
  for (int x = t; x < PS * PC * PD; x += nt) (&L.ssum[0][0][0])[x] = 0;
  for (int x = t; x < PS * PK * 2; x += nt) (&L.fpres[0][0][0])[x] = 0u;
  __syncthreads();
  for (int32_t i = t; i < n; i += nt) {
    const uint32_t el = pa.elig[i];
    for (int k = 0; k < pa.keys; k++) {
      if ((pa.host >> k) & 1u) continue;
      const int32_t d = pa.dom[(size_t)k * n + i];
      if (d < 0) continue;
      for (int s = 0; s < pa.classes; s++)
        if ((el >> (2 * s)) & 1u) atomicOr(&L.fpres[s][k][d >> 5], 1u << (d & 31));
    }
    for (int c = 0; c < pa.cons; c++) {
      const int k = pa.cons_key[c];
      if ((pa.host >> k) & 1u) continue;
      const int32_t d = pa.dom[(size_t)k * n + i];
      const int32_t v = pa.cnt[(size_t)c * n + i];
      if (d < 0 || v == 0) continue;
      atomicAdd(&L.fsum[c][d], v);
      for (int s = 0; s < pa.classes; s++)
        if ((el >> (2 * s + 1)) & 1u) atomicAdd(&L.ssum[s][c][d], v);
    }
  }
  __syncthreads();
}

__device__ __forceinline__ int32_t pts_wave_min(int32_t v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v = min(v, __shfl_xor(v, m));
  return v;
}
__device__ __forceinline__ int32_t pts_wave_max(int32_t v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v = max(v, __shfl_xor(v, m));
  return v;
}
__device__ __forceinline__ uint32_t pts_wave_or(uint32_t v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v |= __shfl_xor(v, m);
  return v;
}
__device__ __forceinline__ int32_t pts_wave_sum(int32_t v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m);
  return v;
}
// A per-thread (min, max) folded into LDS: wave reductions, then one atomic
// per wave (256 threads' atomics on one LDS word serialise)
__device__ __forceinline__ void wave_fold_minmax(int32_t mn, int32_t mx, int32_t *dmin, int32_t *dmax) {
  mn = pts_wave_min(mn);
  mx = pts_wave_max(mx);
  if ((threadIdx.x & 63) == 0) {
    atomicMin(dmin, mn);
    atomicMax(dmax, mx);
  }
}

// Per pod: the pair counters of its keys and the hard keys' minima (wave w =
// key w, lane = domain; requires 256 threads), the phase-A accumulators reset.
__device__ __forceinline__ void pts_prep(const PtsArgs &pa, const PtsPod &q, PtsLds &L, int t) {
  const int k = t >> 6, dd = t & 63;
  if (k < PK && !((pa.host >> k) & 1u)) {
    if ((q.hkeys >> k) & 1u) {
      int32_t m = 0;
#pragma unroll
      for (int j = 0; j < PP; j++)
        if (((q.hard >> j) & 1u) && q.k[j] == k) m += L.fsum[q.c[j]][dd];
      L.fmatch[k][dd] = m;
      const int32_t mn = pts_wave_min(pts_bit(L.fpres[q.cls][k], dd) ? m : INT32_MAX);
      if (dd == 0) L.fmin[k] = mn;
    }
    if ((q.skeys >> k) & 1u) {
      int32_t m = 0;
#pragma unroll
      for (int j = 0; j < PP; j++)
        if (((q.soft >> j) & 1u) && q.k[j] == k) m += L.ssum[q.cls][q.c[j]][dd];
      L.smatch[k][dd] = m;
    }
  }
  if (t < PK * 2) (&L.smask[0][0])[t] = 0u;
  if (t == 0) {
    L.nfni = 0;
    L.red[0] = INT32_MAX;
    L.red[1] = 0;
  }
  __syncthreads();
}

// A hostname key's pair counter on node i: the node's own counts of the pod's
// hard constraints on that key (0 when the node is not hard-eligible: no pair)
__device__ __forceinline__ int32_t pts_host_match(const PtsArgs &pa, const PtsPod &q, int k, int32_t n, int32_t i) {
  if (!((pa.elig[i] >> (2 * q.cls)) & 1u)) return -1;
  int32_t m = 0;
#pragma unroll
  for (int j = 0; j < PP; j++)
    if (((q.hard >> j) & 1u) && q.k[j] == k) m += pa.cnt[(size_t)q.c[j] * n + i];
  return m;
}

// Filter, filtering.go: every hard key on the node; matchNum + self - min <= maxSkew.
__device__ __forceinline__ bool pts_filter(const PtsArgs &pa, const PtsPod &q, const PtsLds &L, int32_t hmin, int32_t n,
                                           int32_t i) {
#pragma unroll
  for (int j = 0; j < PP; j++) {
    if (!((q.hard >> j) & 1u)) continue;
    const int k = q.k[j];
    const int32_t d = pa.dom[(size_t)k * n + i];
    if (d < 0) return false;
    int64_t match, mn;
    if ((pa.host >> k) & 1u) {
      const int32_t m = pts_host_match(pa, q, k, n, i);
      match = m < 0 ? 0 : m;
      mn = hmin;
    } else {
      match = pts_bit(L.fpres[q.cls][k], d) ? L.fmatch[k][d] : 0;
      mn = L.fmin[k];
    }
    if (match + q.self[j] - mn > q.skew[j]) return false;
  }
  return true;
}

// A feasible node: false = an IgnoredNode (lacks a soft key); else its
// domains go into the thread's masks (PreScore's pairs) and count, folded
// into the workgroup's by pts_soft_fold.
__device__ __forceinline__ bool pts_soft_mark(const PtsArgs &pa, const PtsPod &q, int32_t n, int32_t i,
                                              uint32_t (&m)[PK][2], int32_t &cnt) {
#pragma unroll
  for (int j = 0; j < PP; j++)
    if (((q.soft >> j) & 1u) && pa.dom[(size_t)q.k[j] * n + i] < 0) return false;
#pragma unroll
  for (int j = 0; j < PP; j++) {
    if (!((q.soft >> j) & 1u)) continue;
    const int k = q.k[j];
    if ((pa.host >> k) & 1u) continue;
    const int32_t d = pa.dom[(size_t)k * n + i];
#pragma unroll
    for (int kk = 0; kk < PK; kk++)
      if (kk == k) {
        if (d < 32)
          m[kk][0] |= 1u << d;
        else
          m[kk][1] |= 1u << (d - 32);
      }
  }
  cnt++;
  return true;
}

// the threads' soft masks and counts into L.smask / L.nfni (zeroed before)
__device__ __forceinline__ void pts_soft_fold(PtsLds &L, const uint32_t (&m)[PK][2], int32_t cnt) {
  const bool l0 = (threadIdx.x & 63) == 0;
#pragma unroll
  for (int k = 0; k < PK; k++)
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const uint32_t v = pts_wave_or(m[k][h]);
      if (l0 && v) atomicOr(&L.smask[k][h], v);
    }
  cnt = pts_wave_sum(cnt);
  if (l0 && cnt) atomicAdd(&L.nfni, cnt);
}

// topologyNormalizingWeight of each soft constraint from the grid's masks
// (topoSize credited to the first soft constraint of each key) and the
// feasible non-ignored count (hostname)
__device__ __forceinline__ void pts_weights(const PtsArgs &pa, const PtsPod &q, const uint32_t (&mask)[PK][2],
                                            int32_t nfni, double (&w)[PP]) {
  uint32_t seen = 0;
#pragma unroll
  for (int j = 0; j < PP; j++) {
    w[j] = 0.0;
    if (!((q.soft >> j) & 1u)) continue;
    const int k = q.k[j];
    int64_t sz;
    if ((pa.host >> k) & 1u) {
      sz = nfni;
    } else {
      int32_t pc = 0;  // (static indices into mask: no scratch)
#pragma unroll
      for (int kk = 0; kk < PK; kk++)
        if (kk == k) pc = __popc(mask[kk][0]) + __popc(mask[kk][1]);
      sz = ((seen >> k) & 1u) ? 0 : (int64_t)pc;
      seen |= 1u << k;
    }
    w[j] = log((double)(sz + 2));
  }
}

// Score, scoring.go: round(sum of cnt * weight + (maxSkew - 1)) on a non-ignored feasible node
__device__ __forceinline__ int32_t pts_raw(const PtsArgs &pa, const PtsPod &q, const PtsLds &L, const double (&w)[PP],
                                           int32_t n, int32_t i) {
  double s = 0.0;
#pragma unroll
  for (int j = 0; j < PP; j++) {
    if (!((q.soft >> j) & 1u)) continue;
    const int k = q.k[j];
    const int32_t d = pa.dom[(size_t)k * n + i];
    const int64_t cnt = ((pa.host >> k) & 1u) ? (int64_t)pa.cnt[(size_t)q.c[j] * n + i] : (int64_t)L.smatch[k][d];
    s += (double)cnt * w[j] + (double)(q.skew[j] - 1);
  }
  return (int32_t)round(s);
}

// NormalizeScore: ignored (raw < 0) -> 0; max 0 -> 100; else 100 (max + min - s) / max
__device__ __forceinline__ int32_t pts_norm(int32_t raw, int32_t mn, int32_t mx) {
  if (raw < 0) return 0;
  if (mx == 0) return 100;
  return (int32_t)((int64_t)100 * ((int64_t)mx + mn - raw) / mx);
}

// The commit of a pod matching table constraints `match` on node w: every
// workgroup advances its replicas (thread 0); the owner advances w's counts.
__device__ __forceinline__ void pts_commit_tables(const PtsArgs &pa, PtsLds &L, uint32_t match, int32_t n, int32_t w) {
  const uint32_t el = pa.elig[w];
  for (int c = 0; c < pa.cons; c++) {
    if (!((match >> c) & 1u)) continue;
    const int k = pa.cons_key[c];
    if ((pa.host >> k) & 1u) continue;
    const int32_t d = pa.dom[(size_t)k * n + w];
    if (d < 0) continue;
    L.fsum[c][d] += 1;
    for (int s = 0; s < pa.classes; s++)
      if ((el >> (2 * s + 1)) & 1u) L.ssum[s][c][d] += 1;
  }
}

}  // namespace kh
