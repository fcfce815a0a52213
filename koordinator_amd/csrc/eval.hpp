// eval.hpp -- the per-(pod,node) Filter+Score arithmetic on CDNA4, shared by
// every kernel of libkoordhip.so (stream top-k, resolve, parity eval).
//
// Exactness: the reference computes in int64.  On device every resource
// quantity (node columns and pod records) is held as an f64 that IS that
// integer: the host rejects magnitudes >= 2^45 (KH_EXACT_LIMIT), so sums,
// differences, the x100 of leastRequestedScore and the division remainders
// below are all integers < 2^53 and therefore exact in binary64.  The only
// divisions are quotients in [0, 101] (leastRequestedScore, weighted
// averages): a reciprocal estimate, then one exact remainder fix-up in each
// direction, equals Go's truncating int64 division bit for bit (lrs,
// div_weights).  f64 is native on CDNA4's VALU, where int64 multiply/convert
// are multi-instruction sequences.  The LoadAware threshold mask uses IEEE
// f64 division + round-half-away exactly like math.Round in
// load_aware.go:214,248 (compiled with -ffp-contract=off).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/koordhip.h"
#include "numa.hpp"

namespace kh {

// Write-through (sc1) stores: the row reaches the coherence point without an
// agent release fence, i.e. without a write-back of the whole XCD L2
// (cdna_hip_programming.md Guideline 16 R1; MI355X_MICROARCH.md fence table).
template <typename T>
__device__ __forceinline__ void st_wt(T *p, T v) {
  if constexpr (sizeof(T) == 8) {
    __hip_atomic_store(reinterpret_cast<uint64_t *>(p), __builtin_bit_cast(uint64_t, v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  } else if constexpr (sizeof(T) == 4) {
    __hip_atomic_store(reinterpret_cast<uint32_t *>(p), __builtin_bit_cast(uint32_t, v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  } else {
    __hip_atomic_store(reinterpret_cast<uint8_t *>(p), __builtin_bit_cast(uint8_t, v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
}

// device-side node flag bits (flags column, maintained on device)
enum : uint32_t {
  NF_LA_OK_NONPROD = 1u,  // LoadAware Filter passes for non-prod pods
  NF_LA_OK_PROD = 2u,     // ... for prod pods
  NF_LA_SCORE_ZERO = 4u,  // LoadAware Score is 0 (missing / expired NodeMetric)
  NF_OVER_CPU = 8u,       // Requested.cpu > Allocatable.cpu (fitsRequest with a 0 request fails)
  NF_OVER_MEM = 16u,
  NF_OVER_EPH = 32u,
};

struct DevCfg {
  uint32_t filt, score;
  int32_t w_fit, w_la, w_numa, w_bal;
  int32_t fit_w[KOORDHIP_NRES];
  int32_t la_w_cpu, la_w_mem;
  int32_t according;  // ScoreAccordingProdUsage
  int32_t la_alias;   // la_alloc columns equal alloc cpu/mem columns (loaded once)
  int32_t numa_w_cpu, numa_w_mem;  // NodeNUMAResourceArgs scoring weights
  int32_t numa_most;               // NodeNUMAResource MostAllocated scoring strategy
  int32_t zones;                   // some node has a NUMA topology policy (zone columns loaded)
  int32_t amp;                     // some node has a CPU amplification ratio > 1
  int32_t resv;                    // Reservation enabled and the snapshot carries reservation columns
  int32_t resv_slots;              // reservation slots per node (the NM 4 build when > 1)
  int32_t resv_cpus;               // some reservation holds CPUs (resv_cpus columns; the NM 4 build)
  int32_t resv_b1;                 // 1 + the other plugins' maximum weighted total (resv.hpp ranking total)
  int32_t wide_keys;               // ranking totals + 1 exceed 16 bits (the resolve's key tables hold u32)
  // the normalized-score plugins (the sequential cycle, seq.hip)
  int32_t w_ext[KOORDHIP_NEXT_PLUGINS];  // DeviceShare, NodeAffinity, TaintToleration score weights
  int32_t dev_most;                      // DeviceShare MostAllocated scorer
  int32_t dev_w[5];                      // DeviceShare scorer weights: gpu-core, ratio, memory, rdma, fpga
};

// DeviceShare devices, NodeResourcesFit extended scalars and the upstream
// static Score columns (koordhip_node_soa ABI 9; read by the sequential cycle)
struct DevDev {
  int32_t slots;              // minors per type per node (0: no device columns)
  const uint8_t *present;     // [n] nodeDevice entry exists
  const int32_t *minor;       // [n][TYPES][slots], -1 = empty
  const int64_t *total;       // [n][TYPES][slots][RES]
  int64_t *used;              // [n][TYPES][slots][RES]
  const int64_t *xalloc;      // [NXRES][n] (NULL: 0)
  int64_t *xreq;              // [NXRES][n] Requested of the extended scalars
  const uint16_t *sscore[2];  // [MAX_STATIC_CLASSES][n] NodeAffinity / TaintToleration raw scores (NULL: 0)
  // the node's one reservation holding devices (koordhip_node_soa.resv_dev_*;
  // NULL: none): its slot [n] (-1 none) and [n][2][TYPES][slots][RES] its
  // allocatable / allocated (the allocated half advanced by Reserve)
  const int32_t *rslot;
  int64_t *rdev;
  // ABI 14: that reservation's extended scalars [NXRES][n], its Allocatable
  // (the reserve pod's scalar requests) and Allocated (advanced by Reserve);
  // NULL: none (the sequential cycle's Reservation rules read them, resv.hpp ResvXS)
  const int64_t *rxa;
  int64_t *rxd;
};

// Columnar node state in HBM.  Static columns are const; the mutable ones are
// advanced by the resolve kernel (Reserve delta) and by commit/uncommit.
struct DevNodes {
  const double *alloc[KOORDHIP_NRES];
  const int32_t *alloc_pods;
  double *requested[KOORDHIP_NRES];
  double *nz_cpu, *nz_mem;
  int32_t *npods;
  const double *la_alloc_cpu, *la_alloc_mem;
  double *la_used_cpu, *la_used_mem, *la_used_prod_cpu, *la_used_prod_mem;
  uint8_t *flags;
  const uint32_t *sallow;  // KOORDHIP_PLUGIN_NODE_STATIC: allowed pod static classes (NULL = all)
  int32_t n;
  DevNuma nu;  // NodeNUMAResource columns (unused unless the plugin is enabled)
  DevResv rv;  // Reservation columns (NM == 3 builds)
  DevDev dv;   // DeviceShare / extended scalars / static scores (the sequential cycle)
};

// One node's values as the evaluation consumes them (registers or an LDS row).
struct NV {
  double a[KOORDHIP_NRES];
  double r[KOORDHIP_NRES];
  double nz_cpu, nz_mem;
  double la_a_cpu, la_a_mem, la_u_cpu, la_u_mem, la_up_cpu, la_up_mem;
  int32_t a_pods, npods;
  uint32_t flags;
  uint32_t sa;  // static_allow (the row's last word: static, copied along, never written back)
};

// What one pod's evaluation needs from the node columns (wave-uniform).
struct Need {
  bool pods, r_cpu, r_mem, eph, bcpu, bmem, a_cpu, a_mem, nz_cpu, nz_mem, la, la_nonprod, la_prod;
  bool numa, numa_masks;  // NUMA class (+ the cpuset masks for a cpuset pod)
  bool zones;             // node flags + NUMA zones (topology-policy nodes)
  bool amp;               // the CPU amplification ratio + allocated cpuset count
  bool resv;              // the reservation columns (the restore rewrites Requested / NonZero / pods)
  bool sa;                // the static-filter allow mask
};

__device__ __forceinline__ bool numa_on(const DevCfg &c) {
  return ((c.filt | c.score) & KOORDHIP_PLUGIN_NUMA) != 0;
}
__device__ __forceinline__ bool is_cpuset(const DevPod &p) {
  return (p.flags & KOORDHIP_POD_CPUSET) && !(p.flags & (KOORDHIP_POD_NUMA_SKIP | KOORDHIP_POD_NUMA_ERROR));
}
// NodeNUMAResource acts on this pod at Filter / Reserve on some node: a cpuset
// pod, or any pod with requests once a node has a topology policy
__device__ __forceinline__ bool numa_active(const DevPod &p, const DevCfg &c) {
  return is_cpuset(p) || (c.zones && !(p.flags & (KOORDHIP_POD_NUMA_SKIP | KOORDHIP_POD_NUMA_ERROR)));
}

__device__ __forceinline__ Need pod_needs(const DevPod &p, const DevCfg &c) {
  Need n{};
  const bool ff = c.filt & KOORDHIP_PLUGIN_FIT;
  const bool fs = c.score & KOORDHIP_PLUGIN_FIT;
  const bool hr = p.flags & KOORDHIP_POD_HAS_REQ;
  n.pods = ff;
  n.r_cpu = ff && hr && p.req[KOORDHIP_RES_CPU] != 0.0;
  n.r_mem = ff && hr && p.req[KOORDHIP_RES_MEM] != 0.0;
  n.eph = (ff && hr && p.req[KOORDHIP_RES_EPH] != 0.0) || (fs && c.fit_w[KOORDHIP_RES_EPH] != 0);
  n.bcpu = (ff && (p.flags & KOORDHIP_POD_REQ_BCPU)) ||
           (fs && c.fit_w[KOORDHIP_RES_BCPU] != 0 && p.req[KOORDHIP_RES_BCPU] != 0.0);
  n.bmem = (ff && (p.flags & KOORDHIP_POD_REQ_BMEM)) ||
           (fs && c.fit_w[KOORDHIP_RES_BMEM] != 0 && p.req[KOORDHIP_RES_BMEM] != 0.0);
  n.nz_cpu = fs && c.fit_w[KOORDHIP_RES_CPU] != 0;
  n.nz_mem = fs && c.fit_w[KOORDHIP_RES_MEM] != 0;
  n.la = c.score & KOORDHIP_PLUGIN_LOADAWARE;
  n.la_prod = n.la && c.according && (p.flags & KOORDHIP_POD_PROD);
  n.la_nonprod = n.la && !n.la_prod;
  // NodeNUMAResource: Score reads Requested cpu/memory + Allocatable (scoring.go:104-106, :161-166)
  const bool ns = (c.score & KOORDHIP_PLUGIN_NUMA) && !(p.flags & (KOORDHIP_POD_NUMA_SKIP | KOORDHIP_POD_NUMA_ERROR));
  n.numa = ns || ((c.filt & KOORDHIP_PLUGIN_NUMA) && numa_active(p, c));
  n.numa_masks = numa_on(c) && is_cpuset(p);
  n.zones = n.numa && c.zones && !(p.flags & (KOORDHIP_POD_NUMA_SKIP | KOORDHIP_POD_NUMA_ERROR));
  // filterAmplifiedCPUs / the amplified scores read Requested + Allocatable cpu,
  // the allocated cpuset count and the ratio (plugin.go:326-363, scoring.go:95-168)
  n.amp = c.amp && numa_on(c) && p.req[KOORDHIP_RES_CPU] != 0.0 &&
          !(p.flags & (KOORDHIP_POD_NUMA_SKIP | KOORDHIP_POD_NUMA_ERROR));
  if (n.amp) {
    n.numa = true;
    n.r_cpu = n.a_cpu = true;
  }
  if (ns) {
    n.r_cpu |= !is_cpuset(p);
    n.r_mem = true;
    n.a_cpu = n.a_mem = true;
  }
  // NodeResourcesBalancedAllocation: Requested + Allocatable cpu / memory
  if (c.score & KOORDHIP_PLUGIN_BALANCED) n.r_cpu = n.r_mem = n.a_cpu = n.a_mem = true;
  n.sa = (c.filt & KOORDHIP_PLUGIN_NODE_STATIC) != 0;
  if (c.resv) {
    // the restore rewrites Requested (the over-commit bits are re-derived from
    // it), NonZeroRequested and the pod count; a matched reservation's Aligned /
    // Restricted filter reads ephemeral storage too
    n.resv = true;
    n.r_cpu = n.r_mem = n.pods = true;
    n.eph |= (c.filt & KOORDHIP_PLUGIN_RESERVATION) && p.resv_match != 0ull;
  }
  n.a_cpu = n.a_cpu || n.r_cpu || n.nz_cpu || (n.la && c.la_alias);
  n.a_mem = n.a_mem || n.r_mem || n.nz_mem || (n.la && c.la_alias);
  return n;
}

__device__ __forceinline__ void need_or(Need &a, const Need &b) {
  a.pods |= b.pods;
  a.r_cpu |= b.r_cpu;
  a.r_mem |= b.r_mem;
  a.eph |= b.eph;
  a.bcpu |= b.bcpu;
  a.bmem |= b.bmem;
  a.a_cpu |= b.a_cpu;
  a.a_mem |= b.a_mem;
  a.nz_cpu |= b.nz_cpu;
  a.nz_mem |= b.nz_mem;
  a.la |= b.la;
  a.la_nonprod |= b.la_nonprod;
  a.la_prod |= b.la_prod;
  a.numa |= b.numa;
  a.numa_masks |= b.numa_masks;
  a.zones |= b.zones;
  a.amp |= b.amp;
  a.resv |= b.resv;
}

__device__ __forceinline__ Need need_all(const DevCfg &c) {
  Need n{};
  n.pods = n.r_cpu = n.r_mem = n.eph = n.bcpu = n.bmem = n.a_cpu = n.a_mem = n.nz_cpu = n.nz_mem = true;
  n.la = true;
  n.la_nonprod = true;
  n.la_prod = c.according != 0;
  n.numa = n.numa_masks = numa_on(c);
  n.zones = n.numa && c.zones;
  n.amp = n.numa && c.amp;
  n.resv = c.resv != 0;
  n.sa = true;
  return n;
}

// NodeNUMAResource columns of node i.
__device__ __forceinline__ void load_zones(NumaRow &r, const DevNodes &d, int32_t i) {
  const double *zu = d.nu.zu + (size_t)i * 2 * ZMAX;
  r.za = d.nu.za + (size_t)i * 2 * ZMAX;  // static: read in place by the zone code
#pragma unroll
  for (int q = 0; q < ZMAX; q++) {
    r.zu[0][q] = zu[q];
    r.zu[1][q] = zu[ZMAX + q];
  }
}

template <bool Z>
__device__ __forceinline__ void load_numa(NumaRow &r, const DevNodes &d, int32_t i, const Need &n) {
  r.cls = -1;
  r.nflags = 0;
  r.amp = 1.0;
  if (!n.numa) return;
  r.cls = d.nu.node_cls[i];
  if (n.amp) {
    r.amp = d.nu.amp[i];
    r.cnt = d.nu.cnt[i];
  }
  if (n.numa_masks || (Z && n.zones)) r.nflags = d.nu.nflags[i];
  if constexpr (Z) {
    if (n.zones && topo_policy(r.nflags) != 0) load_zones(r, d, i);
  }
  if (n.numa_masks) {
    r.cnt = d.nu.cnt[i];
#pragma unroll
    for (int w = 0; w < NW; w++) {
      r.fr[w] = d.nu.fr[w][i];
      r.ep[w] = d.nu.ep[w][i];
      r.en[w] = d.nu.en[w][i];
    }
  }
}

// Column element i with a 32-bit byte offset: lets the compiler use the
// SGPR-base + 32-bit VGPR-offset form of global loads/stores (no 64-bit
// address arithmetic per column).  Node counts are < 2^26, so offsets fit.
template <typename T>
__device__ __forceinline__ const T &col(const T *base, int32_t i) {
  return *reinterpret_cast<const T *>(reinterpret_cast<const char *>(base) + (uint32_t)i * (uint32_t)sizeof(T));
}
template <typename T>
__device__ __forceinline__ T &col(T *base, int32_t i) {
  return *reinterpret_cast<T *>(reinterpret_cast<char *>(base) + (uint32_t)i * (uint32_t)sizeof(T));
}

// Load node i's columns the evaluation needs (coalesced across lanes).
__device__ __forceinline__ void load_node(NV &v, const DevNodes &d, int32_t i, const Need &n, const DevCfg &c) {
  v.flags = col(d.flags, i);
  v.sa = (n.sa && d.sallow) ? col(d.sallow, i) : 0xFFFFFFFFu;
  if (n.pods) {
    v.a_pods = col(d.alloc_pods, i);
    v.npods = col(d.npods, i);
  }
  if (n.a_cpu) v.a[KOORDHIP_RES_CPU] = col(d.alloc[KOORDHIP_RES_CPU], i);
  if (n.a_mem) v.a[KOORDHIP_RES_MEM] = col(d.alloc[KOORDHIP_RES_MEM], i);
  if (n.r_cpu) v.r[KOORDHIP_RES_CPU] = col(d.requested[KOORDHIP_RES_CPU], i);
  if (n.r_mem) v.r[KOORDHIP_RES_MEM] = col(d.requested[KOORDHIP_RES_MEM], i);
  if (n.eph) {
    v.a[KOORDHIP_RES_EPH] = col(d.alloc[KOORDHIP_RES_EPH], i);
    v.r[KOORDHIP_RES_EPH] = col(d.requested[KOORDHIP_RES_EPH], i);
  }
  if (n.bcpu) {
    v.a[KOORDHIP_RES_BCPU] = col(d.alloc[KOORDHIP_RES_BCPU], i);
    v.r[KOORDHIP_RES_BCPU] = col(d.requested[KOORDHIP_RES_BCPU], i);
  }
  if (n.bmem) {
    v.a[KOORDHIP_RES_BMEM] = col(d.alloc[KOORDHIP_RES_BMEM], i);
    v.r[KOORDHIP_RES_BMEM] = col(d.requested[KOORDHIP_RES_BMEM], i);
  }
  if (n.nz_cpu) v.nz_cpu = col(d.nz_cpu, i);
  if (n.nz_mem) v.nz_mem = col(d.nz_mem, i);
  if (n.la) {
    if (c.la_alias) {
      v.la_a_cpu = v.a[KOORDHIP_RES_CPU];
      v.la_a_mem = v.a[KOORDHIP_RES_MEM];
    } else {
      v.la_a_cpu = col(d.la_alloc_cpu, i);
      v.la_a_mem = col(d.la_alloc_mem, i);
    }
    if (n.la_prod) {
      v.la_up_cpu = col(d.la_used_prod_cpu, i);
      v.la_up_mem = col(d.la_used_prod_mem, i);
    }
    if (n.la_nonprod) {
      v.la_u_cpu = col(d.la_used_cpu, i);
      v.la_u_mem = col(d.la_used_mem, i);
    }
  }
}

// The per-(pod,node) functions below branch only on wave-uniform values (pod
// record, plugin config); per-node conditions are computed for every lane and
// combined with selects, so a wave runs one straight-line sequence instead of
// exec-masked short-circuit paths.

// num / ws for the weighted averages (num <= 100 * sum of weights <= 50000,
// ws <= 500): an f32 reciprocal estimate (relative error ~2^-23, so the
// absolute error is < 0.01) truncated, then one exact int32 fix-up each way.
__device__ __forceinline__ int32_t div_weights(int32_t num, int32_t ws) {
  int32_t q = (int32_t)((float)num * __builtin_amdgcn_rcpf((float)ws));
  const int32_t r = num - q * ws;
  q -= (r < 0);
  q += (r >= ws);
  return q;
}
// ... with a wave-uniform power-of-two weight sum: a shift
__device__ __forceinline__ int32_t div_weights_uniform(int32_t num, int32_t ws) {
  if ((ws & (ws - 1)) == 0) return num >> __builtin_ctz((uint32_t)ws);
  return div_weights(num, ws);
}

// leastRequestedScore, load_aware.go:388-397 / least_allocated.go:49-58:
// (cap - req) * 100 / cap in int64, 0 if cap == 0 or req > cap.
// f = (cap - req) * 100 < 2^52 is exact, the reciprocal estimate of f / cap
// (<= 100) is within 1 of the quotient, and the remainder f - q * cap (one
// fma, exact: an integer < 2^53) fixes it up.
__device__ __forceinline__ int32_t lrs(double req, double cap) {
  const bool zero = (cap == 0.0) | (req > cap);
  const double f = (cap - req) * 100.0;
  int32_t q = (int32_t)(f * __builtin_amdgcn_rcp(cap));
  const double r = __builtin_fma(-(double)q, cap, f);
  q -= (r < 0.0);
  q += (r >= cap);
  return zero ? 0 : q;
}

// mostRequestedScore, nodenumaresource/most_allocated.go:51-62: min(req, cap)
// * 100 / cap in int64 (cap == 0 -> 0), with the same exact quotient fix-up.
__device__ __forceinline__ int32_t mrs(double req, double cap) {
  const double f = (req > cap ? cap : req) * 100.0;
  int32_t q = (int32_t)(f * __builtin_amdgcn_rcp(cap));
  const double r = __builtin_fma(-(double)q, cap, f);
  q -= (r < 0.0);
  q += (r >= cap);
  return cap == 0.0 ? 0 : q;
}

// Fit LeastAllocated score (upstream resource_allocation.go + least_allocated.go;
// koord copy nodenumaresource/scoring.go:191-246): resources with Allocatable 0
// are left out of both sums; scalar resources only when the pod requests them.
__device__ __forceinline__ int32_t fit_score(const DevPod &p, const NV &v, const DevCfg &c) {
  int32_t num = 0, ws = 0;
  auto term = [&](double req, double cap, int32_t w) {
    const bool on = cap != 0.0;
    num += on ? lrs(req, cap) * w : 0;
    ws += on ? w : 0;
  };
  if (c.fit_w[KOORDHIP_RES_CPU]) term(v.nz_cpu + p.nz_cpu_m, v.a[KOORDHIP_RES_CPU], c.fit_w[KOORDHIP_RES_CPU]);
  if (c.fit_w[KOORDHIP_RES_MEM]) term(v.nz_mem + p.nz_mem, v.a[KOORDHIP_RES_MEM], c.fit_w[KOORDHIP_RES_MEM]);
  if (c.fit_w[KOORDHIP_RES_EPH])
    term(v.r[KOORDHIP_RES_EPH] + p.req[KOORDHIP_RES_EPH], v.a[KOORDHIP_RES_EPH], c.fit_w[KOORDHIP_RES_EPH]);
#pragma unroll
  for (int r = KOORDHIP_RES_BCPU; r <= KOORDHIP_RES_BMEM; r++)
    if (c.fit_w[r] && p.req[r] != 0.0) term(v.r[r] + p.req[r], v.a[r], c.fit_w[r]);
  return ws == 0 ? 0 : div_weights(num, ws);
}

// fitsRequest (upstream fit.go; mirror reservation/plugin.go:445-494).  A zero
// request on cpu/memory/ephemeral reduces to "Requested > Allocatable", kept
// as the NF_OVER_* bits so such pods need not read those columns.
__device__ __forceinline__ bool fit_filter(const DevPod &p, const NV &v) {
  bool ok = v.npods < v.a_pods;  // npods + 1 > allowedPods fails
  if (!(p.flags & KOORDHIP_POD_HAS_REQ)) return ok;
  if (p.req[KOORDHIP_RES_CPU] != 0.0)
    ok &= !(p.req[KOORDHIP_RES_CPU] > v.a[KOORDHIP_RES_CPU] - v.r[KOORDHIP_RES_CPU]);
  else
    ok &= !(v.flags & NF_OVER_CPU);
  if (p.req[KOORDHIP_RES_MEM] != 0.0)
    ok &= !(p.req[KOORDHIP_RES_MEM] > v.a[KOORDHIP_RES_MEM] - v.r[KOORDHIP_RES_MEM]);
  else
    ok &= !(v.flags & NF_OVER_MEM);
  if (p.req[KOORDHIP_RES_EPH] != 0.0)
    ok &= !(p.req[KOORDHIP_RES_EPH] > v.a[KOORDHIP_RES_EPH] - v.r[KOORDHIP_RES_EPH]);
  else
    ok &= !(v.flags & NF_OVER_EPH);
  if (p.flags & KOORDHIP_POD_REQ_BCPU)
    ok &= !(p.req[KOORDHIP_RES_BCPU] > v.a[KOORDHIP_RES_BCPU] - v.r[KOORDHIP_RES_BCPU]);
  if (p.flags & KOORDHIP_POD_REQ_BMEM)
    ok &= !(p.req[KOORDHIP_RES_BMEM] > v.a[KOORDHIP_RES_BMEM] - v.r[KOORDHIP_RES_BMEM]);
  return ok;
}

// LoadAware Filter (load_aware.go:123-171): static mask + DaemonSet bypass.
__device__ __forceinline__ bool la_filter(const DevPod &p, const NV &v) {
  if (p.flags & KOORDHIP_POD_DAEMONSET) return true;
  return (v.flags & ((p.flags & KOORDHIP_POD_PROD) ? NF_LA_OK_PROD : NF_LA_OK_NONPROD)) != 0;
}

// LoadAware Score (load_aware.go:269-335, scorer :378-386): every configured
// weight counts in the denominator.
__device__ __forceinline__ int32_t la_score(const DevPod &p, const NV &v, const DevCfg &c) {
  const bool prod = c.according && (p.flags & KOORDHIP_POD_PROD);
  const double ucpu = p.est_cpu + (prod ? v.la_up_cpu : v.la_u_cpu);
  const double umem = p.est_mem + (prod ? v.la_up_mem : v.la_u_mem);
  const int32_t num = lrs(ucpu, v.la_a_cpu) * c.la_w_cpu + lrs(umem, v.la_a_mem) * c.la_w_mem;
  const int32_t s = div_weights_uniform(num, c.la_w_cpu + c.la_w_mem);
  return (v.flags & NF_LA_SCORE_ZERO) ? 0 : s;
}

// extension.Amplify (node_resource_amplification.go:191-196) on an exact f64 integer
__device__ __forceinline__ double amplify(double v, double ratio) { return ratio <= 1.0 ? v : ceil(v * ratio); }

// filterAmplifiedCPUs, plugin.go:326-363: the allocated cpuset CPUs count
// amplified in Requested; a cpuset pod's request is amplified too.
__device__ __forceinline__ bool amp_filter_ok(const DevPod &p, const NV &v, const NumaRow &r) {
  const double cpu = p.req[KOORDHIP_RES_CPU];
  if (cpu == 0.0 || r.amp <= 1.0) return true;
  const double req = is_cpuset(p) ? amplify(cpu, r.amp) : cpu;
  const double allocm = r.cls >= 0 ? (double)r.cnt * 1000.0 : 0.0;  // GetAvailableCPUs
  double requested = v.r[KOORDHIP_RES_CPU];
  if (requested >= allocm && allocm > 0.0) requested = requested - allocm + amplify(allocm, r.amp);
  return !(req > v.a[KOORDHIP_RES_CPU] - requested);
}

// NodeNUMAResource Score (scoring.go:55-168).
// filtered: the NodeNUMAResource Filter passed on this (pod, node) -- under a
// required bind policy that already proved Allocate feasible (plugin.go:307-316)
// P: the reservation-preferred CPUs of the pod on this node (resv_pref_cpus;
// NULL or zero: none)
template <bool Z>
__device__ __forceinline__ int32_t numa_score(const DevPod &p, const NV &v, const NumaRow &r,
                                              const DevNumaClass *classes, const DevCfg &c, bool filtered = false,
                                              const uint64_t *P = nullptr) {
  if (p.flags & (KOORDHIP_POD_NUMA_SKIP | KOORDHIP_POD_NUMA_ERROR)) return 0;
  if (r.cls < 0) return 0;  // no CPU topology: getResourceOptions / Allocate error -> 0
  const bool most = c.numa_most != 0;  // leastResourceScorer / mostResourceScorer (scoring.go:35-53)
  auto lr = [most](double a, double b) { return most ? mrs(a, b) : lrs(a, b); };
  auto dw = [](int32_t a, int32_t b) { return div_weights(a, b); };
  const bool cs = (p.flags & KOORDHIP_POD_CPUSET) != 0;
  const int tp = Z ? topo_policy(r.nflags) : 0;
  if (!cs && tp == 0) {  // scoreWithAmplifiedCPUs (:95-120)
    double rq = v.r[KOORDHIP_RES_CPU];
    if (c.amp && p.req[KOORDHIP_RES_CPU] != 0.0 && r.amp > 1.0) {
      const double allocm = (double)r.cnt * 1000.0;
      rq = rq - allocm + amplify(allocm, r.amp);
    }
    return numa_la(rq + p.req[KOORDHIP_RES_CPU], v.a[KOORDHIP_RES_CPU], v.r[KOORDHIP_RES_MEM] + p.req[KOORDHIP_RES_MEM],
                   v.a[KOORDHIP_RES_MEM], c.numa_w_cpu, c.numa_w_mem, lr, dw);
  }
  const DevNumaClass &C = classes[r.cls];
  double ac = v.a[KOORDHIP_RES_CPU], am = v.a[KOORDHIP_RES_MEM];
  double rc = v.r[KOORDHIP_RES_CPU], rm = v.r[KOORDHIP_RES_MEM];
  uint32_t mask = 0;
  const bool hp = cs && P && any4(P);  // a nominated reservation's CPUs (the pod is a cpuset pod)
  int taken_p = 0;                     // how many of them the pod takes
  if (Z && tp != 0) {  // the affinity stored by Filter's admit, then Allocate with it (:80-89)
    double av[2][ZMAX];
    zone_avail_all(r, C.nnuma, av);
    if (!zone_hint(C.nnuma, av, p, tp, &mask)) return 0;
    if (mask) {
      // Score's getResourceOptions counts P as reusable zone resources (plugin.go:465-479)
      double ru[ZMAX];
#pragma unroll
      for (int k = 0; k < ZMAX; k++) ru[k] = 0.0;
      if (hp) {
        zone_reusable(C, P, ru);
        zone_avail_reus(r, C.nnuma, ru, av);
      }
      double z[2][ZMAX];
      if (!zone_alloc(C.nnuma, av, p, mask, z)) return 0;
      if (cs) {
        uint64_t m[NW];
        if (KOORDHIP_NUMA_REQUIRED(p.numa_policy) == KOORDHIP_CPUBIND_NONE) {
          if (!zone_cpus_ok(C, r, p, z, hp ? P : nullptr, &taken_p)) return 0;
        } else {
          if (!zone_allocate(C, r, p, z, m, hp ? P : nullptr)) return 0;
          if (hp) taken_p = popc_and(m, P);
        }
      }
      // calculateAllocatableAndRequested over the pod's zones (:134-152), the
      // allocated amounts less the reusable ones
      ac = am = rc = rm = 0.0;
#pragma unroll
      for (int k = 0; k < ZMAX; k++)
        if (zone_used(z, k)) {
          ac += r.za[k];
          am += r.za[ZMAX + k];
          rc += zone_cpu_allocated(r, k, ru);
          rm += r.zu[1][k];
        }
    }
  }
  double qc = p.req[KOORDHIP_RES_CPU];
  if (hp) {
    // Allocate with the preferred CPUs (free | P; P is allocated, so disjoint
    // from the free CPUs); calculateAllocatableAndRequested then counts the
    // allocated CPUs less P's CPUs the pod did not take (:161-166): without a
    // hint the pod takes min(need, |P|) of them
    const int need = p.numa_cpus, np = popc4(P);
    if (!mask) {
      if (popc4(r.fr) + np < need) return 0;
      if (KOORDHIP_NUMA_REQUIRED(p.numa_policy) != KOORDHIP_CPUBIND_NONE &&
          !numa_allocate_pref(C, r, p, P[0], P[1], P[2], P[3]))
        return 0;
      taken_p = need < np ? need : np;
    }
    rc = amplify((double)(r.cnt - (np - taken_p)) * 1000.0, r.amp);
    qc = amplify(qc, r.amp);
  } else if (cs) {
    const bool proven = filtered && tp == 0 && KOORDHIP_NUMA_REQUIRED(p.numa_policy) != KOORDHIP_CPUBIND_NONE;
    if (!mask && !proven && !numa_alloc_ok(C, r, p)) return 0;
    // requested cpu := the allocated cpuset size, amplified (:161-166); the
    // pod's own request amplified too (getResourceOptions, plugin.go:481-485)
    rc = amplify((double)r.cnt * 1000.0, r.amp);
    qc = amplify(qc, r.amp);
  }
  return numa_la(rc + qc, ac, rm + p.req[KOORDHIP_RES_MEM], am, c.numa_w_cpu, c.numa_w_mem, lr, dw);
}

// NodeResourcesBalancedAllocation Score (upstream k8s v1.24.15
// balanced_allocation.go balancedResourceScorer over resource_allocation.go's
// calculateResourceAllocatableRequest with useRequested: Requested + the
// pod's request, cpu and memory with weight 1, resources with Allocatable 0
// left out): fraction = min(1, req / alloc) in f64, std = |f_cpu - f_mem| / 2
// for two fractions (0 for fewer), score = int64((1 - std) * 100).
__device__ __forceinline__ int32_t bal_score(const DevPod &p, const NV &v) {
  const double ac = v.a[KOORDHIP_RES_CPU], am = v.a[KOORDHIP_RES_MEM];
  double fc = (v.r[KOORDHIP_RES_CPU] + p.req[KOORDHIP_RES_CPU]) / ac;
  double fm = (v.r[KOORDHIP_RES_MEM] + p.req[KOORDHIP_RES_MEM]) / am;
  fc = fc > 1.0 ? 1.0 : fc;
  fm = fm > 1.0 ? 1.0 : fm;
  const double std = (ac != 0.0 && am != 0.0) ? fabs((fc - fm) / 2.0) : 0.0;
  return (int32_t)((1.0 - std) * 100.0);
}

// Total weighted score, or -1 when any enabled Filter fails.
__device__ __forceinline__ int32_t eval_total(const DevPod &p, const NV &v, const DevCfg &c) {
  bool ok = true;
  if (c.filt & KOORDHIP_PLUGIN_NODE_STATIC) ok &= ((v.sa >> p.sclass) & 1u) != 0;
  if (c.filt & KOORDHIP_PLUGIN_FIT) ok &= fit_filter(p, v);
  if (c.filt & KOORDHIP_PLUGIN_LOADAWARE) ok &= la_filter(p, v);
  int32_t t = 0;
  if (c.score & KOORDHIP_PLUGIN_FIT) t += c.w_fit * fit_score(p, v, c);
  if (c.score & KOORDHIP_PLUGIN_LOADAWARE) t += c.w_la * la_score(p, v, c);
  if (c.score & KOORDHIP_PLUGIN_BALANCED) t += c.w_bal * bal_score(p, v);
  return ok ? t : -1;
}

// ... with NodeNUMAResource
template <bool Z>
__device__ __forceinline__ int32_t eval_total_numa(const DevPod &p, const NV &v, const NumaRow &r,
                                                   const DevNumaClass *classes, const DevCfg &c,
                                                   const uint64_t *P = nullptr) {
  int32_t t = eval_total(p, v, c);
  if (t < 0) return t;
  const bool nf = (c.filt & KOORDHIP_PLUGIN_NUMA) != 0;
  if (nf && (p.flags & KOORDHIP_POD_NUMA_ERROR)) return -1;
  if (nf && c.amp && !amp_filter_ok(p, v, r)) return -1;
  if (nf && !numa_filter<Z>(p, r, classes)) return -1;
  if (c.score & KOORDHIP_PLUGIN_NUMA) t += c.w_numa * numa_score<Z>(p, v, r, classes, c, nf, P);
  return t;
}

}  // namespace kh

#include "resv.hpp"

namespace kh {

// ... with the Reservation plugin (NM == 3): the cycle's restore of the
// node's reservation first (every plugin sees the restored NodeInfo), then
// filterWithReservations and the ranking total of resv.hpp.
// RC: some reservation holds CPUs (the NM 5 build).  Z (the sequential cycle's
// topology-policy snapshots; RC with S > 1): the zone row of node zi is read
// into a copy of the row after the reserved CPUs (which share its bytes) are
// taken, and the NodeNUMAResource Filter / Score run with the zone code.
template <int S, bool RC = false, bool Z = false>
__device__ __forceinline__ int32_t eval_total_resv(const DevPod &p, const NV &v, const NumaRowRS<S> &r,
                                                   const DevNumaClass *classes, const DevCfg &c,
                                                   const DevNodes *zd = nullptr, int32_t zi = 0,
                                                   ResvXS rx = no_rx()) {
  NV w = v;
  uint32_t mm;
  const int nmatch = resv_restore(w, r, p, mm, rx);
  int32_t t;
  if constexpr (Z) {
    static_assert(RC && S > 1, "the zone build is the several-slot reserved-CPU build");
    uint64_t P[NW];
    resv_pref_cpus(r, p, (c.score & KOORDHIP_PLUGIN_RESERVATION) ? mm : 0u, P, rx);
    NumaRow q = r;
    if (topo_policy(q.nflags) != 0) load_zones(q, *zd, zi);
    t = eval_total_numa<true>(p, w, q, classes, c, P);
  } else if constexpr (RC && S > 1) {
    // the NodeNUMAResource Score reads the reserved CPUs of the reservation
    // PreScore nominated on the node (scoring.go:86-166, plugin.go:503-524)
    uint64_t P[NW];
    resv_pref_cpus(r, p, (c.score & KOORDHIP_PLUGIN_RESERVATION) ? mm : 0u, P, rx);
    t = eval_total_numa<false>(p, w, r, classes, c, P);
  } else {
    t = eval_total_numa<false>(p, w, r, classes, c);
  }
  if (t < 0) return t;
  if (nmatch == 0)  // a required reservation affinity needs a matched reservation on the node (plugin.go:378-381)
    return ((c.filt & KOORDHIP_PLUGIN_RESERVATION) && (p.flags & KOORDHIP_POD_RESV_AFFINITY)) ? -1 : t;
  if ((c.filt & KOORDHIP_PLUGIN_RESERVATION) && !resv_filter(p, w, r, mm, nmatch, rx)) return -1;
  if (c.score & KOORDHIP_PLUGIN_RESERVATION) {
    const int rk = resv_node_rank(r, mm);
    if (rk >= 0) return 101 * c.resv_b1 + (KOORDHIP_RESV_MAX_ORDERS - 1 - rk);
    const int q = resv_nominate(p, r, mm, rx);
    if (q >= 0) t += resv_score(p, r.rs[q], q == rx.h, rx) * c.resv_b1;
  }
  return t;
}

// Ranking key: larger is better; equal totals -> lower node index wins
// (replaces selectHost's reservoir-random tie-break).  0 = infeasible.
__device__ __forceinline__ uint64_t make_key(int32_t total, int32_t node) {
  return total < 0 ? 0ull : (((uint64_t)(uint32_t)(total + 1)) << 32) | (uint64_t)(0xFFFFFFFFu - (uint32_t)node);
}
__device__ __forceinline__ int32_t key_node(uint64_t k) { return (int32_t)(0xFFFFFFFFu - (uint32_t)k); }
__device__ __forceinline__ int32_t key_score(uint64_t k) { return (int32_t)(k >> 32) - 1; }

// Reserve delta (podAssignCache.assign + NodeInfo.AddPod), sign = +1 / -1.
__device__ __forceinline__ void apply_delta(NV &v, const DevPod &p, int sign) {
  const double sg = (double)sign;
#pragma unroll
  for (int r = 0; r < KOORDHIP_NRES; r++) v.r[r] = __builtin_fma(sg, p.req[r], v.r[r]);
  v.nz_cpu = __builtin_fma(sg, p.nz_cpu_m, v.nz_cpu);
  v.nz_mem = __builtin_fma(sg, p.nz_mem, v.nz_mem);
  v.npods += sign;
  v.la_u_cpu = __builtin_fma(sg, p.est_cpu, v.la_u_cpu);
  v.la_u_mem = __builtin_fma(sg, p.est_mem, v.la_u_mem);
  if (p.flags & KOORDHIP_POD_PROD) {
    v.la_up_cpu = __builtin_fma(sg, p.est_cpu, v.la_up_cpu);
    v.la_up_mem = __builtin_fma(sg, p.est_mem, v.la_up_mem);
  }
  uint32_t f = v.flags & ~(NF_OVER_CPU | NF_OVER_MEM | NF_OVER_EPH);
  if (v.r[KOORDHIP_RES_CPU] > v.a[KOORDHIP_RES_CPU]) f |= NF_OVER_CPU;
  if (v.r[KOORDHIP_RES_MEM] > v.a[KOORDHIP_RES_MEM]) f |= NF_OVER_MEM;
  if (v.r[KOORDHIP_RES_EPH] > v.a[KOORDHIP_RES_EPH]) f |= NF_OVER_EPH;
  v.flags = f;
}

// Full row load / store (resolve and commit paths).
__device__ __forceinline__ void load_row(NV &v, const DevNodes &d, int32_t i) {
#pragma unroll
  for (int r = 0; r < KOORDHIP_NRES; r++) {
    v.a[r] = d.alloc[r][i];
    v.r[r] = d.requested[r][i];
  }
  v.a_pods = d.alloc_pods[i];
  v.npods = d.npods[i];
  v.nz_cpu = d.nz_cpu[i];
  v.nz_mem = d.nz_mem[i];
  v.la_a_cpu = d.la_alloc_cpu[i];
  v.la_a_mem = d.la_alloc_mem[i];
  v.la_u_cpu = d.la_used_cpu[i];
  v.la_u_mem = d.la_used_mem[i];
  v.la_up_cpu = d.la_used_prod_cpu[i];
  v.la_up_mem = d.la_used_prod_mem[i];
  v.flags = d.flags[i];
  v.sa = d.sallow ? d.sallow[i] : 0xFFFFFFFFu;
}

template <bool Z = true>
__device__ __forceinline__ void load_numa_row(NumaRow &r, const DevNodes &d, int32_t i) {
  r.cls = d.nu.node_cls[i];
  r.nflags = d.nu.nflags[i];
  r.cnt = d.nu.cnt[i];
#pragma unroll
  for (int w = 0; w < NW; w++) {
    r.fr[w] = d.nu.fr[w][i];
    r.ep[w] = d.nu.ep[w][i];
    r.en[w] = d.nu.en[w][i];
  }
  if (Z && d.nu.za && topo_policy(r.nflags) != 0) load_zones(r, d, i);
  r.amp = d.nu.amp ? d.nu.amp[i] : 1.0;
}

template <bool Z = true>
__device__ __forceinline__ void store_numa_row(const NumaRow &r, const DevNodes &d, int32_t i) {
  d.nu.cnt[i] = r.cnt;
#pragma unroll
  for (int w = 0; w < NW; w++) {
    d.nu.fr[w][i] = r.fr[w];
    d.nu.ep[w][i] = r.ep[w];
    d.nu.en[w][i] = r.en[w];
  }
  if (Z && d.nu.za && topo_policy(r.nflags) != 0) {
    double *zu = d.nu.zu + (size_t)i * 2 * ZMAX;
#pragma unroll
    for (int q = 0; q < ZMAX; q++) {
      zu[q] = r.zu[0][q];
      zu[ZMAX + q] = r.zu[1][q];
    }
  }
}

// NodeNUMAResource Reserve / Release on a row (resourceManager.Update / Release,
// node_allocation.go:76-131).
// P (Reserve only): reservation-preferred CPUs the pod may have taken -- they
// were allocated already (RefCount 1 -> 2: the allocated count does not grow),
// and addPodAllocation overwrites their exclusive policy with the pod's.
__device__ __forceinline__ void numa_apply(NumaRow &r, const DevPod &p, const uint64_t *cpus, int sign,
                                           const uint64_t *P = nullptr) {
  const int ex = (int)KOORDHIP_NUMA_EXCLUSIVE(p.numa_policy);
  int n = 0;
#pragma unroll
  for (int w = 0; w < NW; w++) {
    n += __popcll(P ? (cpus[w] & ~P[w]) : cpus[w]);
    if (sign > 0) {
      r.fr[w] &= ~cpus[w];
      r.ep[w] = (r.ep[w] & ~cpus[w]) | (ex == (int)KOORDHIP_CPUEXCL_PCPU ? cpus[w] : 0ull);
      r.en[w] = (r.en[w] & ~cpus[w]) | (ex == (int)KOORDHIP_CPUEXCL_NUMA ? cpus[w] : 0ull);
    } else {
      r.fr[w] |= cpus[w];
      r.ep[w] &= ~cpus[w];
      r.en[w] &= ~cpus[w];
    }
  }
  r.cnt += sign * n;
}

__device__ __forceinline__ void store_row(const NV &v, const DevNodes &d, int32_t i) {
#pragma unroll
  for (int r = 0; r < KOORDHIP_NRES; r++) d.requested[r][i] = v.r[r];
  d.npods[i] = v.npods;
  d.nz_cpu[i] = v.nz_cpu;
  d.nz_mem[i] = v.nz_mem;
  d.la_used_cpu[i] = v.la_u_cpu;
  d.la_used_mem[i] = v.la_u_mem;
  d.la_used_prod_cpu[i] = v.la_up_cpu;
  d.la_used_prod_mem[i] = v.la_up_mem;
  d.flags[i] = (uint8_t)v.flags;
}

// The resolve's write-back of a committed row (the mutable columns), write-through.
__device__ __forceinline__ void store_row_wt(const NV &v, const DevNodes &d, int32_t i) {
#pragma unroll
  for (int r = 0; r < KOORDHIP_NRES; r++) st_wt(&d.requested[r][i], v.r[r]);
  st_wt(&d.npods[i], v.npods);
  st_wt(&d.nz_cpu[i], v.nz_cpu);
  st_wt(&d.nz_mem[i], v.nz_mem);
  st_wt(&d.la_used_cpu[i], v.la_u_cpu);
  st_wt(&d.la_used_mem[i], v.la_u_mem);
  st_wt(&d.la_used_prod_cpu[i], v.la_up_cpu);
  st_wt(&d.la_used_prod_mem[i], v.la_up_mem);
  st_wt(&d.flags[i], (uint8_t)v.flags);
}

template <bool Z = true>
__device__ __forceinline__ void store_numa_row_wt(const NumaRow &r, const DevNodes &d, int32_t i) {
  st_wt(&d.nu.cnt[i], r.cnt);
#pragma unroll
  for (int w = 0; w < NW; w++) {
    st_wt(&d.nu.fr[w][i], r.fr[w]);
    st_wt(&d.nu.ep[w][i], r.ep[w]);
    st_wt(&d.nu.en[w][i], r.en[w]);
  }
  if (Z && d.nu.za && topo_policy(r.nflags) != 0) {
    double *zu = d.nu.zu + (size_t)i * 2 * ZMAX;
#pragma unroll
    for (int q = 0; q < ZMAX; q++) {
      st_wt(&zu[q], r.zu[0][q]);
      st_wt(&zu[ZMAX + q], r.zu[1][q]);
    }
  }
}

// NodeNUMAResource Reserve on a row for a pod with numa_active(): the cpuset
// (Allocate, resource_manager.go:142-164) and, on a topology-policy node, the
// hinted zones' amounts (resourceManager.Update, node_allocation.go:76-103).
// false = Allocate fails (nothing applied).
// WAVE: called by every lane of one wave with the same inputs (the resolve's
// Reserve): the accumulator's CPU-id ordered takes run lane-parallel.
// pref: the reservation-preferred CPUs (resv_pref_cpus), NULL or zero: none.
template <bool Z, bool WAVE = false>
__device__ __attribute__((noinline)) bool numa_reserve(const DevNumaClass *classes, NumaRow &row, const DevPod &pod,
                                                       uint64_t *cpus_out, const uint64_t *pref = nullptr) {
  // registers for the whole replay (the references point at the caller's stack)
  NumaRow r = row;
  const DevPod p = pod;
  uint64_t cpus[NW] = {0, 0, 0, 0};
  uint64_t P[NW] = {0, 0, 0, 0};
  if (pref)
    for (int w = 0; w < NW; w++) P[w] = pref[w];
  for (int w = 0; w < NW; w++) cpus_out[w] = 0;
  const bool cs = (p.flags & KOORDHIP_POD_CPUSET) != 0;
  const int tp = Z ? topo_policy(r.nflags) : 0;
  if (!cs && tp == 0) return true;
  if (r.cls < 0) return false;
  const DevNumaClass &C = classes[r.cls];
  if (!Z || tp == 0) {
    if (cs && any4(P)) {
      if (!numa_allocate_pref_in<WAVE>(C, r, p, P, cpus)) return false;
    } else if (!numa_allocate_in<WAVE>(C, r, p, cpus)) {
      return false;
    }
    numa_apply(r, p, cpus, +1, P);
  } else {
    // the hint is Filter's (no reservation nominated yet); the allocation
    // counts the nominated reservation's CPUs P as reusable zone resources and
    // takes them first (getResourceOptions, plugin.go:455-501)
    uint32_t mask;
    double av[2][ZMAX];
    zone_avail_all(r, C.nnuma, av);
    if (!zone_hint(C.nnuma, av, p, tp, &mask)) return false;
    const bool hp = cs && any4(P);
    if (hp) {
      double ru[ZMAX];
      zone_reusable(C, P, ru);
      zone_avail_reus(r, C.nnuma, ru, av);
    }
    double z[2][ZMAX];
    if (mask && !zone_alloc(C.nnuma, av, p, mask, z)) return false;
    if (cs) {
      if (mask) {
        if (!zone_allocate_in(C, r, p, z, cpus, hp ? P : nullptr)) return false;
      } else if (hp) {
        if (!numa_allocate_pref_in<WAVE>(C, r, p, P, cpus)) return false;
      } else if (!numa_allocate_in<WAVE>(C, r, p, cpus)) {
        return false;
      }
      numa_apply(r, p, cpus, +1, P);
    }
    if (mask) {
#pragma unroll
      for (int k = 0; k < ZMAX; k++) {
        r.zu[0][k] += z[0][k];
        r.zu[1][k] += z[1][k];
      }
    }
  }
  row = r;
  for (int w = 0; w < NW; w++) cpus_out[w] = cpus[w];
  return true;
}

}  // namespace kh
