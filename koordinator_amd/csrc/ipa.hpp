// ipa.hpp -- upstream InterPodAffinity (k8s v1.24 pkg/scheduler/framework/
// plugins/interpodaffinity; not vendored in the reference) for the
// sequential cycle (seq.hip).  Restated in oracle/ipa_oracle.c, which is the
// checker; koordinator_amd/interpodaffinity.py builds the count entries.
//
// Device model.  Every count the plugin reads is the sum, over the nodes of a
// (topology key, value) pair, of one count entry's per-node column ipa_cnt[e]
// (the pods a term matches, or the pods carrying a term).  Per launch one
// kernel (k_ipa_sums) sums each entry per domain of its key; every workgroup
// copies the sums into LDS and advances them on every commit exactly like
// PodTopologySpread's replicas (pts.hpp): the winner's domains and the pod's
// ipa_inc are known to every workgroup, so nobody reads another's counts.  A
// hostname entry's pair is the node itself: its own column, read by its
// owner.  The pod's Filter reads the entries of its masks, its raw Score the
// weighted entries; the min-max NormalizeScore needs the grid's min / max of
// the raw scores over the feasible nodes (two more words in phase A's
// granule), nothing else crosses workgroups.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dev.hpp"
#include "pts.hpp"

namespace kh {

constexpr int IE = KOORDHIP_IPA_ENTRIES;
constexpr int IPA_SUMS = IE * PD + IE;  // k_ipa_sums' output: [IE][PD] domain sums, then [IE] totals

struct IpaArgs {
  const int32_t *dom;  // the topology keys' domains [keys][n] (the pts_* columns)
  int32_t *cnt;        // [ents][n] (advanced by the owner's Reserve)
  int32_t *sums;       // IPA_SUMS ints, written by k_ipa_sums at each launch
  int32_t ents;
  uint32_t host;       // bit k: key k is kubernetes.io/hostname
  int32_t filt, score; // the plugin's Filter / Score are enabled (and the snapshot has entries)
  int32_t w;           // Score weight
  int32_t ent_key[IE];
};

struct IpaLds {
  int32_t dsum[IE][PD];  // entry e's pods in domain d of its key (non-hostname keys)
  int32_t tot[IE];       // ... over every node carrying the key (len(affinityCounts) == 0)
  int32_t mm[2];         // the workgroup's raw Score min / max
};

__device__ __forceinline__ int ipa_next(uint32_t &m) {
  const int e = __ffs(m) - 1;
  m &= m - 1u;
  return e;
}

__device__ __forceinline__ void ipa_load(const IpaArgs &a, IpaLds &L, int t, int nt) {
  for (int x = t; x < IE * PD; x += nt) (&L.dsum[0][0])[x] = a.sums[x];
  for (int x = t; x < IE; x += nt) L.tot[x] = a.sums[IE * PD + x];
  __syncthreads();
}

// Entry e's count at node i's pair, -1 when the node lacks the key
__device__ __forceinline__ int32_t ipa_count(const IpaArgs &a, const IpaLds &L, int e, int32_t n, int32_t i) {
  const int k = a.ent_key[e];
  const int32_t d = a.dom[(size_t)k * n + i];
  if (d < 0) return -1;
  return ((a.host >> k) & 1u) ? a.cnt[(size_t)e * n + i] : L.dsum[e][d];
}

// Filter, filtering.go: satisfyPodAffinity (every term's key on the node and
// its pair counted; else only the first pod of a series: no pair counted
// anywhere and the pod matching its own terms), satisfyPodAntiAffinity +
// satisfyExistingPodsAntiAffinity (no counted pair at the node's values).
__device__ __forceinline__ bool ipa_filter(const IpaArgs &a, const IpaLds &L, const DevPodX &x, int32_t n, int32_t i) {
  uint32_t m = x.ipa_anti;
  while (m) {
    const int e = ipa_next(m);
    if (ipa_count(a, L, e, n, i) > 0) return false;
  }
  if (x.ipa_aff) {
    bool exist = true;
    m = x.ipa_aff;
    while (m) {
      const int e = ipa_next(m);
      const int32_t c = ipa_count(a, L, e, n, i);
      if (c < 0) return false;
      if (c <= 0) exist = false;
    }
    if (!exist) {
      if (!(x.ipa_flags & KOORDHIP_IPA_SELF)) return false;
      m = x.ipa_aff;
      while (m)
        if (L.tot[ipa_next(m)] != 0) return false;
    }
  }
  return true;
}

// Score, scoring.go: the node's topologyScore = sum of w[e] x entry e's pair count
__device__ __forceinline__ int32_t ipa_raw(const IpaArgs &a, const IpaLds &L, uint32_t score, const int32_t *w,
                                           int32_t n, int32_t i) {
  int64_t s = 0;
  while (score) {
    const int e = ipa_next(score);
    const int32_t c = ipa_count(a, L, e, n, i);
    if (c > 0) s += (int64_t)w[e] * c;
  }
  return (int32_t)s;
}

// NormalizeScore: int64(MaxNodeScore x float64(s - min) / float64(max - min)), 0 when max == min
__device__ __forceinline__ int32_t ipa_norm(int32_t raw, int32_t mn, int32_t mx) {
  if (mx <= mn) return 0;
  const double f = 100.0 * ((double)((int64_t)raw - mn) / (double)((int64_t)mx - mn));
  return (int32_t)f;
}

// The commit of a pod counted by entries `inc` on node w: every workgroup
// advances its sums (thread 0); the owner advances w's columns.
__device__ __forceinline__ void ipa_commit_tables(const IpaArgs &a, IpaLds &L, uint32_t inc, int32_t n, int32_t w) {
  while (inc) {
    const int e = ipa_next(inc);
    const int k = a.ent_key[e];
    const int32_t d = a.dom[(size_t)k * n + w];
    if (d < 0) continue;
    L.tot[e] += 1;
    if (!((a.host >> k) & 1u)) L.dsum[e][d] += 1;
  }
}

__device__ __forceinline__ void ipa_commit_cols(const IpaArgs &a, uint32_t inc, int32_t n, int32_t w) {
  while (inc) {
    const int e = ipa_next(inc);
    a.cnt[(size_t)e * n + w] += 1;
  }
}

}  // namespace kh
