// numa.hpp -- NodeNUMAResource on CDNA4 (maxRefCount 1, no
// reservation-preferred CPUs, cpus_per_core 1 or 2; NUMA topology policies
// None / BestEffort / Restricted / SingleNUMANode over <= 8 NUMA zones).
//
// Node state is a handful of 4 x 64-bit masks over core-major CPU positions
// (pos = core_rank * cpc + t), so a core is an aligned group of cpc bits:
// "any CPU of the core" / "every CPU of the core" are one shift + OR / AND
// and NUMA-node / socket membership is an AND with a per-class mask.
//
// Filter/Score need only whether resourceManager.Allocate would succeed
// (scoring.go:86-91 uses the allocated size of the NODE, not of the choice),
// which has a closed form per bind policy (derived from the accumulator's
// control flow, cpu_accumulator.go:87-232; checked against the oracle's
// literal accumulator in tests):
//   preferred only      : |free| >= need                           (:257-259)
//   required FullPCPUs  : cpc * #fully-free cores >= need          (:105-177 take whole cores first)
//   required Spread     : the first NUMA node / socket the accumulator
//                         would pick decides; see numa_spread_ok.
// Reserve needs the exact CPUs: acc_take_cpus replays the accumulator on the
// masks (wave-uniform: every lane computes the same result).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/koordhip.h"
#include "pod.hpp"

namespace kh {

// The running best of the node / socket selection loops (whose trip counts
// come from the per-node topology class, i.e. divergent in the scan kernel) is
// pinned: with ROCm 7.2's optimizer these selections came out wrong
// (tests/test_gpu_numa.py: e.g. "allocate in the smallest idle socket") unless
// the functions were built optnone, which made the scan 5x and the cpuset
// Reserve 30x slower.  Pinning just these variables is enough: after every
// iteration an empty asm takes the value in a VGPR and hands it back "changed":
// the optimizer can neither fold the running best into a select chain nor
// move it across iterations, and the value stays in a register (a volatile
// stack slot cost a scratch round trip per access: ~30k cycles per Reserve).
#define KH_PIN(x) asm volatile("" : "+v"(x))

// The selections themselves are a max over one integer key per candidate:
// the strategy-ordered primary and secondary counts (MostAllocated:
// ascending, LeastAllocated: descending; <= 256 each), then the lower index
// (ties keep the first candidate, like the reference's strict comparisons).
// A plain integer max-reduction is what the optimizer handles robustly.
__device__ __forceinline__ int sel_key(int most, int primary, int secondary, int idx) {
  const int p = most ? 511 - primary : primary;
  const int q = most ? 511 - secondary : secondary;
  return (1 << 30) | (p << 20) | (q << 10) | (1023 - idx);
}
__device__ __forceinline__ int sel_index(int key) { return key ? 1023 - (key & 1023) : -1; }

constexpr int NW = KOORDHIP_NUMA_WORDS;
constexpr int NMAX = KOORDHIP_NUMA_MAX_NODES;
constexpr int ZMAX = KOORDHIP_NUMA_MAX_ZONES;

struct DevNumaClass {
  int32_t ncpu, cpc, cpn, cps, nnuma, nsock;
  uint8_t sock_of_node[NMAX];
  uint64_t nm[NMAX][NW];  // CPUs of NUMA node k
  uint64_t sm[NMAX][NW];  // CPUs of socket s
  uint8_t pos_by_id[KOORDHIP_NUMA_MAX_CPUS];  // positions in ascending CPU id
};

static_assert(sizeof(DevNumaClass) % 16 == 0, "classes are staged in LDS as 16-B words");
static_assert(offsetof(DevNumaClass, pos_by_id) % 16 == 0, "pos_by_id is read 16 entries per load");

struct NumaRow {
  int32_t cls;     // -1: no CPU topology
  uint32_t nflags; // KOORDHIP_NODE_* (0 unless loaded)
  int32_t cnt;     // allocated CPUs
  int32_t pad;
  uint64_t fr[NW], ep[NW], en[NW];
  // NUMA zones of a node with a topology policy (zone k = NUMA node rank k):
  // the NRT allocatable is static and stays in HBM (za: the node's [2][ZMAX]
  // row there, read only by the zone code); NodeAllocation.allocatedResources
  // is mutable and travels with the row, [cpu milli, memory][zone]
  const double *za;
  union {
    double zu[2][ZMAX];
    // Reservation builds (no topology-policy nodes, so no zones): the reserved
    // CPUs left in each reservation slot of the node (RestoreReservation,
    // nodenumaresource/reservation.go:76-113), see resv.hpp
    uint64_t rcm[KOORDHIP_RESV_SLOTS][NW];
  };
  double amp;  // CPU amplification ratio (1 unless loaded)
};
static_assert(sizeof(uint64_t[KOORDHIP_RESV_SLOTS][NW]) == sizeof(double[2][ZMAX]), "rcm shares the zone row's bytes");

struct DevNuma {
  const DevNumaClass *cls;
  const int32_t *node_cls;
  const uint8_t *nflags;
  uint64_t *fr[NW], *ep[NW], *en[NW];
  int32_t *cnt;
  const double *za;  // [n][2][ZMAX], NULL when no node has a topology policy
  double *zu;        // [n][2][ZMAX]
  const double *amp; // CPU amplification ratio per node, NULL when none is > 1
  int32_t ncls;      // topology classes at cls
};

// Reservation columns on device (f64 hold the int64 values exactly), see resv.hpp.
struct DevResv {
  const uint32_t *flags;  // NULL: no reservation columns
  const int32_t *rank;
  const double *ra[2];    // Allocatable cpu milli, memory
  const double *rz[2];    // the reserve pod's non-zero cpu / memory request
  double *rd[2];          // Allocated
  int32_t *rn;            // len(AssignedPods)
  int32_t slots;          // reservation slots per node: the columns hold slots x stride values, slot-major
  int32_t stride;         // = the node count
  uint64_t *rc[KOORDHIP_NUMA_WORDS];  // reserved CPUs left per slot (RestoreReservation); NULL: none hold CPUs
};

struct ZoneRow {  // one node's [2][ZMAX] zone row (update_nodes scatter element)
  double v[2 * ZMAX];
};
static_assert(sizeof(ZoneRow) == 128, "zone rows are 8 zones x 2 resources");

__device__ __forceinline__ int topo_policy(uint32_t nflags) {
  return (int)KOORDHIP_NODE_NUMA_POLICY(nflags);
}

// Kernels stage up to this many topology classes in LDS (800 B each): the
// accumulator's loops and the closed-form Filter read them with dependent,
// data-driven indexes, at LDS instead of L2 latency.
constexpr int NUMA_LDS_CLASSES = 8;

__device__ __forceinline__ int popc4(const uint64_t *m) {
  return __popcll(m[0]) + __popcll(m[1]) + __popcll(m[2]) + __popcll(m[3]);
}

// lead bit of every core with any / every CPU set in m
__device__ __forceinline__ uint64_t fold_or(uint64_t m, int cpc) {
  return cpc == 1 ? m : ((m | (m >> 1)) & 0x5555555555555555ull);
}
__device__ __forceinline__ uint64_t fold_and(uint64_t m, int cpc) {
  return cpc == 1 ? m : ((m & (m >> 1)) & 0x5555555555555555ull);
}
__device__ __forceinline__ uint64_t expand(uint64_t lead, int cpc) { return cpc == 1 ? lead : (lead | (lead << 1)); }

__device__ __forceinline__ int popc_and(const uint64_t *a, const uint64_t *b) {
  return __popcll(a[0] & b[0]) + __popcll(a[1] & b[1]) + __popcll(a[2] & b[2]) + __popcll(a[3] & b[3]);
}

// strategy direction of a free-score comparison: MostAllocated -> ascending
__device__ __forceinline__ bool free_before(int most, int x, int y) { return (most ? y - x : x - y) > 0; }

__device__ __forceinline__ int node_policy(uint32_t nflags, int preferred) {
  const uint32_t p = nflags & KOORDHIP_NODE_CPUBIND_MASK;  // getPreferredCPUBindPolicy, plugin.go:546-566
  return p == 1 ? (int)KOORDHIP_CPUBIND_FULL_PCPUS : (p == 2 ? (int)KOORDHIP_CPUBIND_SPREAD_BY_PCPUS : preferred);
}

// CPUs excluded by the pod's exclusive policy (isCPUExclusivePCPULevel /
// isCPUExclusiveNUMANodeLevel, cpu_accumulator.go:318-330): whole cores holding a
// PCPULevel-allocated CPU, or whole NUMA nodes holding a NUMANodeLevel one.
__device__ __forceinline__ void excluded_set(const DevNumaClass &C, const NumaRow &r, int excl, bool pcpu_only,
                                             uint64_t *X) {
  for (int w = 0; w < NW; w++) X[w] = 0;
  if (excl == (int)KOORDHIP_CPUEXCL_PCPU) {
    for (int w = 0; w < NW; w++) X[w] = expand(fold_or(r.ep[w], C.cpc), C.cpc);
  } else if (excl == (int)KOORDHIP_CPUEXCL_NUMA && !pcpu_only) {
    for (int k = 0; k < C.nnuma; k++)
      if (popc_and(r.en, C.nm[k]))
        for (int w = 0; w < NW; w++) X[w] |= C.nm[k][w];
  }
}

// distinct cores among m & g
__device__ __forceinline__ int cores_in(const uint64_t *m, const uint64_t *g, int cpc) {
  int c = 0;
  for (int w = 0; w < NW; w++) c += __popcll(fold_or(m[w] & g[w], cpc));
  return c;
}

// Required SpreadByPCPUs with cpc == 2: whether takeCPUs' choice is one CPU
// per core.  Stages follow cpu_accumulator.go:184-229; a stage that finds a
// group big enough returns immediately, with distinct cores iff the group has
// that many distinct cores (spreadCPUs takes one CPU per core first).
// (masks by value: the caller's row never has to go through scratch memory)
__device__ __attribute__((noinline)) bool numa_spread_ok(const DevNumaClass &C, uint64_t f0, uint64_t f1, uint64_t f2,
                                                         uint64_t f3, uint64_t p0, uint64_t p1, uint64_t p2, uint64_t p3,
                                                         uint64_t n0, uint64_t n1, uint64_t n2, uint64_t n3, int need,
                                                         int excl, bool most) {
  NumaRow r;
  r.fr[0] = f0, r.fr[1] = f1, r.fr[2] = f2, r.fr[3] = f3;
  r.ep[0] = p0, r.ep[1] = p1, r.ep[2] = p2, r.ep[3] = p3;
  r.en[0] = n0, r.en[1] = n1, r.en[2] = n2, r.en[3] = n3;
  const int cpc = C.cpc;
  uint64_t X[NW], Xp[NW], F[NW];
  excluded_set(C, r, excl, false, X);
  excluded_set(C, r, excl, true, Xp);
  if (need <= C.cpn) {
    // pass filterExclusive=true: extracted lists (distinct cores) -> any big enough node succeeds
    for (int w = 0; w < NW; w++) F[w] = r.fr[w] & ~X[w];
    for (int k = 0; k < C.nnuma; k++)
      if (cores_in(F, C.nm[k], cpc) >= need) return true;
    // pass false: the first node in (free, socket free, id) order with >= need CPUs decides
    int bkey = 0;
    for (int k = 0; k < C.nnuma; k++) {
      const int f = popc_and(r.fr, C.nm[k]);
      if (f < need) continue;
      const int sf = popc_and(r.fr, C.sm[C.sock_of_node[k]]);
      bkey = max(bkey, sel_key(most, f, sf, k));
    }
    const int best = sel_index(bkey);
    if (best >= 0) return cores_in(r.fr, C.nm[best], cpc) >= need;
  }
  if (need <= C.cps) {
    for (int w = 0; w < NW; w++) F[w] = r.fr[w] & ~Xp[w];  // socket pass true filters PCPULevel only (:612)
    for (int s = 0; s < C.nsock; s++)
      if (cores_in(F, C.sm[s], cpc) >= need) return true;
    int bkey = 0;
    for (int s = 0; s < C.nsock; s++) {
      const int f = popc_and(r.fr, C.sm[s]);
      if (f < need) continue;
      bkey = max(bkey, sel_key(most, f, 0, s));
    }
    const int best = sel_index(bkey);
    if (best >= 0) return cores_in(r.fr, C.sm[best], cpc) >= need;
  }
  // freeCPUs(true) spread, then freeCPUs(false) over what is left (:218-229)
  uint64_t allm[NW], FX[NW];
  for (int w = 0; w < NW; w++) {
    allm[w] = ~0ull;
    F[w] = r.fr[w] & ~X[w];
    FX[w] = r.fr[w] & X[w];
  }
  const int cT = popc4(F), dT = cores_in(F, allm, cpc);
  if (need <= dT) return true;
  if (cT >= need || cT > dT) return false;
  return need - cT <= cores_in(FX, allm, cpc);
}

// resourceManager.Allocate succeeds? (empty hint, no preferred CPUs)
__device__ __forceinline__ bool numa_alloc_ok(const DevNumaClass &C, const NumaRow &r, const DevPod &p) {
  const int need = p.numa_cpus;
  if (popc4(r.fr) < need) return false;  // allocateCPUSet :257-259 (filterAvailableCPUsByRequiredCPUBindPolicy is a no-op)
  const int req = (int)KOORDHIP_NUMA_REQUIRED(p.numa_policy);
  if (req == (int)KOORDHIP_CPUBIND_NONE) return true;  // takeCPUs never fails once need <= |available|
  const int pol = node_policy(r.nflags, (int)KOORDHIP_NUMA_PREFERRED(p.numa_policy));
  if (pol == (int)KOORDHIP_CPUBIND_FULL_PCPUS) {
    int full = 0;
    for (int w = 0; w < NW; w++) full += __popcll(fold_and(r.fr[w], C.cpc));
    return full * C.cpc >= need;
  }
  if (C.cpc == 1) return true;
  return numa_spread_ok(C, r.fr[0], r.fr[1], r.fr[2], r.fr[3], r.ep[0], r.ep[1], r.ep[2], r.ep[3], r.en[0], r.en[1],
                        r.en[2], r.en[3], need, (int)KOORDHIP_NUMA_EXCLUSIVE(p.numa_policy),
                        (r.nflags & KOORDHIP_NODE_NUMA_MOST_ALLOCATED) != 0);
}

__device__ __forceinline__ bool numa_policy_ok(const DevNumaClass &C, const NumaRow &r, const DevPod &p);

// Filter, plugin.go:266-324; true = passes.  Z = false: no node has a
// topology policy (the zone code is compiled out).
template <bool Z>
__device__ __forceinline__ bool numa_filter(const DevPod &p, const NumaRow &r, const DevNumaClass *classes) {
  if (p.flags & KOORDHIP_POD_NUMA_ERROR) return false;
  const int tp = Z ? topo_policy(r.nflags) : 0;
  const bool cs = (p.flags & KOORDHIP_POD_CPUSET) != 0;
  if ((p.flags & KOORDHIP_POD_NUMA_SKIP) || (!cs && tp == 0)) return true;  // skipTheNode, util.go:59-61
  if (r.cls < 0) return false;  // no CPU topology (a policy node: getResourceOptions fails in Allocate)
  const DevNumaClass &C = classes[r.cls];
  if constexpr (Z) {
    if (!cs) return numa_policy_ok(C, r, p);
  }
  const int req = (int)KOORDHIP_NUMA_REQUIRED(p.numa_policy);
  const bool full_only = (r.nflags & KOORDHIP_NODE_CPUBIND_MASK) == 1u;
  if (full_only || req == (int)KOORDHIP_CPUBIND_FULL_PCPUS) {
    if (p.numa_cpus % C.cpc != 0) return false;
    if (full_only && (req != (int)KOORDHIP_CPUBIND_FULL_PCPUS ||
                      (int)KOORDHIP_NUMA_PREFERRED(p.numa_policy) != (int)KOORDHIP_CPUBIND_FULL_PCPUS))
      return false;
  }
  if constexpr (Z) {
    if (tp != 0) return numa_policy_ok(C, r, p);
  }
  if (req != (int)KOORDHIP_CPUBIND_NONE) return numa_alloc_ok(C, r, p);
  return true;
}

// leastResourceScorer over {cpu, memory}, alloc 0 left out (scoring.go:191-230)
template <typename Lrs, typename Div>
__device__ __forceinline__ int32_t numa_la(double rc, double ac, double rm, double am, int32_t wc, int32_t wm,
                                           Lrs lrs_fn, Div div_fn) {
  int32_t num = 0, ws = 0;
  if (wc && ac != 0.0) {
    num += lrs_fn(rc, ac) * wc;
    ws += wc;
  }
  if (wm && am != 0.0) {
    num += lrs_fn(rm, am) * wm;
    ws += wm;
  }
  return ws ? div_fn(num, ws) : 0;
}

// ---------------------------------------------------------------------------
// Exact accumulator replay for Reserve (cpu_accumulator.go:87-232, mask form).
//
// The replay's functions stay noinline (one copy, called from the 1-wave
// resolve and from k_commit); their node / socket selections keep the running
// best pinned by KH_PIN (see the top of this file): ROCm 7.2 otherwise
// picks a different NUMA node / socket than the reference's order for some
// states, -O2 and -O3 alike.  tests/test_gpu_numa.py pins every choice bit for
// bit (reference KATs, randomized states, streams).

struct Acc {
  uint64_t A[NW];   // allocatable
  uint64_t R[NW];   // result
  uint64_t XC[NW];  // exclusiveInCores (lead bits)
  uint32_t XN;      // exclusiveInNUMANodes
  int need, excl;
  int most;  // 1: MostAllocated (ascending free), 0: LeastAllocated
};

// Bit p of a 4-word mask held in registers: the word is chosen by selects,
// never by a dynamic index (which would move the whole array to scratch).
__device__ __forceinline__ bool tbit(const uint64_t *m, int p) {
  const int w = p >> 6;
  const uint64_t x = w == 0 ? m[0] : (w == 1 ? m[1] : (w == 2 ? m[2] : m[3]));
  return (x >> (p & 63)) & 1ull;
}
__device__ __forceinline__ void sbit(uint64_t *m, int p) {
  const uint64_t b = 1ull << (p & 63);
#pragma unroll
  for (int w = 0; w < NW; w++) m[w] |= (w == (p >> 6)) ? b : 0ull;
}
__device__ __forceinline__ void cbit(uint64_t *m, int p) {
  const uint64_t b = 1ull << (p & 63);
#pragma unroll
  for (int w = 0; w < NW; w++) m[w] &= (w == (p >> 6)) ? ~b : ~0ull;
}
// ... of a mask in memory (the class tables): one load
__device__ __forceinline__ bool tbit_mem(const uint64_t *m, int p) { return (m[p >> 6] >> (p & 63)) & 1ull; }

__device__ __forceinline__ void acc_take1(const DevNumaClass &C, Acc &a, int p) {
  sbit(a.R, p);
  cbit(a.A, p);
  if (a.excl == (int)KOORDHIP_CPUEXCL_PCPU) sbit(a.XC, p - (p % C.cpc));
  if (a.excl == (int)KOORDHIP_CPUEXCL_NUMA)
    for (int k = 0; k < C.nnuma; k++)
      if (tbit_mem(C.nm[k], p)) a.XN |= 1u << k;
  a.need--;
}

// take every position of T at once: the result, the available set, the
// exclusivity state and `need` are order-free functions of the taken set,
// so this equals acc_take1 over T's positions in any order
__device__ __forceinline__ void acc_take_mask(const DevNumaClass &C, Acc &a, const uint64_t *T) {
  int n = 0;
  for (int w = 0; w < NW; w++) {
    a.R[w] |= T[w];
    a.A[w] &= ~T[w];
    n += __popcll(T[w]);
  }
  if (a.excl == (int)KOORDHIP_CPUEXCL_PCPU)
    for (int w = 0; w < NW; w++) a.XC[w] |= fold_or(T[w], C.cpc);
  if (a.excl == (int)KOORDHIP_CPUEXCL_NUMA)
    for (int k = 0; k < C.nnuma; k++)
      if (popc_and(T, C.nm[k])) a.XN |= 1u << k;
  a.need -= n;
}

// the lowest k set bits of x (binary search on prefix popcounts)
__device__ __forceinline__ uint64_t low_bits(uint64_t x, int k) {
  if (k <= 0) return 0ull;
  if (k >= __popcll(x)) return x;
  int lo = 0;  // popc(x & mask(lo)) < k, mask(t) = bits [0, t)
  for (int st = 32; st; st >>= 1) {
    const int t = lo + st;
    if (__popcll(x & (t >= 64 ? ~0ull : ((1ull << t) - 1ull))) < k) lo = t;
  }
  const int t = lo + 1;
  return x & (t >= 64 ? ~0ull : ((1ull << t) - 1ull));
}

// take the lowest n positions of m
__device__ __forceinline__ void acc_take_low(const DevNumaClass &C, Acc &a, const uint64_t *m, int n) {
  uint64_t T[NW];
  for (int w = 0; w < NW; w++) {
    T[w] = low_bits(m[w], n);
    n -= __popcll(T[w]);
  }
  acc_take_mask(C, a, T);
}

// ---- WAVE = true: the replay runs in every lane of one wave with the same
// inputs (the resolve's Reserve); the CPU-id ordered takes then split the ids
// over the lanes and combine with ballots instead of walking them one by one.
__device__ __forceinline__ uint64_t acc_wave_or(uint64_t v) {
  uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
  for (int m = 1; m < 64; m <<= 1) {
    lo |= (uint32_t)__shfl_xor((int)lo, m, 64);
    hi |= (uint32_t)__shfl_xor((int)hi, m, 64);
  }
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t word_of(const uint64_t *S, int w) {
  return w == 0 ? S[0] : (w == 1 ? S[1] : (w == 2 ? S[2] : S[3]));
}
// T |= the n positions of S with the smallest CPU ids (every lane, same inputs)
__device__ __forceinline__ void acc_first_by_id(const DevNumaClass &C, const uint64_t *S, int n, uint64_t *T) {
  if (n <= 0) return;
  const int lane = __lane_id();
  uint64_t t[NW] = {0, 0, 0, 0};
  int taken = 0;
  for (int base = 0; base < C.ncpu && taken < n; base += 64) {
    const int i = base + lane;
    const int p = i < C.ncpu ? (int)C.pos_by_id[i] : 0;
    const bool in = i < C.ncpu && ((word_of(S, p >> 6) >> (p & 63)) & 1ull);
    const uint64_t b = __ballot(in);
    const int rank = taken + __popcll(b & ((1ull << lane) - 1ull));
    if (in && rank < n) {
      const uint64_t bit = 1ull << (p & 63);
      const int w = p >> 6;
      t[0] |= w == 0 ? bit : 0ull;
      t[1] |= w == 1 ? bit : 0ull;
      t[2] |= w == 2 ? bit : 0ull;
      t[3] |= w == 3 ? bit : 0ull;
    }
    taken += __popcll(b);
  }
  for (int w = 0; w < NW; w++) T[w] |= acc_wave_or(t[w]);
}

// the accumulator's exclusion mask for filterExclusive passes
__device__ __forceinline__ void acc_excluded(const DevNumaClass &C, const Acc &a, bool pcpu_only, uint64_t *X) {
  for (int w = 0; w < NW; w++) X[w] = 0;
  if (a.excl == (int)KOORDHIP_CPUEXCL_PCPU) {
    for (int w = 0; w < NW; w++) X[w] = expand(a.XC[w], C.cpc);
  } else if (a.excl == (int)KOORDHIP_CPUEXCL_NUMA && !pcpu_only) {
    for (int k = 0; k < C.nnuma; k++)
      if (a.XN & (1u << k))
        for (int w = 0; w < NW; w++) X[w] |= C.nm[k][w];
  }
}

// One lane: T |= the n positions of S with the smallest CPU ids.  pos_by_id
// is read 16 entries per load (the loads are independent of the takes).
__device__ __forceinline__ void lane_first_by_id(const DevNumaClass &C, const uint64_t *S, int n, uint64_t *T) {
  for (int i = 0; i < C.ncpu && n > 0; i += 16) {
    const uint4 q = *reinterpret_cast<const uint4 *>(C.pos_by_id + i);
    const uint32_t wd[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int j = 0; j < 16; j++) {
      const int p = (int)((wd[j >> 2] >> ((j & 3) * 8)) & 255u);
      if (i + j < C.ncpu && n > 0 && tbit(S, p)) {
        sbit(T, p);
        n--;
      }
    }
  }
}

// spread order of the CPUs of m listed in ascending CPU id (freeCPUsInNode /
// freeCPUsInSocket + spreadCPUs): round t takes each core's t-th CPU by id,
// rounds in id order; lists of <= cpc CPUs are kept in id order.  Takes n.
// WAVE: the order is (round, id) with round 1 = the second CPU of a core whose
// first is in m too -- positions ascend by id inside a core (build_numa_class
// checks it), so that is the odd position of a core with both bits in m.
// The same (round, id) order serves lists of <= cpc CPUs, which the
// reference keeps in id order: inside a core positions ascend by id.
template <bool WAVE = false>
__device__ __forceinline__ void acc_take_spread_by_id(const DevNumaClass &C, Acc &a, const uint64_t *m, int n) {
  if (n <= 0) return;
  uint64_t S0[NW], S1[NW], T[NW];
  for (int w = 0; w < NW; w++) {
    S1[w] = C.cpc == 2 ? (m[w] & (m[w] << 1) & 0xAAAAAAAAAAAAAAAAull) : 0ull;
    S0[w] = m[w] & ~S1[w];
    T[w] = 0ull;
  }
  const int n0 = popc4(S0);
  if constexpr (WAVE) {
    acc_first_by_id(C, S0, min(n, n0), T);
    if (n > n0) acc_first_by_id(C, S1, n - n0, T);
  } else {
    lane_first_by_id(C, S0, min(n, n0), T);
    if (n > n0) lane_first_by_id(C, S1, n - n0, T);
  }
  acc_take_mask(C, a, T);
}

// freeCPUs(filterExclusive) + spreadCPUs + one-by-one take (:218-229).
__device__ __forceinline__ void acc_fallback_pass(const DevNumaClass &C, Acc &a, bool fe) {
  uint64_t X[NW], F[NW];
  if (fe) acc_excluded(C, a, false, X);
  else
    for (int w = 0; w < NW; w++) X[w] = 0;
  for (int w = 0; w < NW; w++) F[w] = a.A[w] & ~X[w];
  int nfree[NMAX], sfree[NMAX], colo[NMAX];
  for (int k = 0; k < NMAX; k++) nfree[k] = sfree[k] = colo[k] = 0;
  for (int k = 0; k < C.nnuma; k++) nfree[k] = popc_and(F, C.nm[k]);
  for (int s = 0; s < C.nsock; s++) {
    sfree[s] = popc_and(F, C.sm[s]);
    colo[s] = popc_and(a.R, C.sm[s]);
  }
  // core groups (node k, free CPUs in core cf): every sort key except the core id
  // is constant inside a group; order groups, merge equal keys, list cores by id.
  int gk[2 * NMAX], gc[2 * NMAX], ng = 0;
  for (int k = 0; k < C.nnuma; k++)
    for (int cf = 1; cf <= C.cpc; cf++) {
      gk[ng] = k;
      gc[ng] = cf;
      ng++;
    }
  auto before = [&](int x, int y) -> int {  // 1: x before y, -1: y before x, 0: equal key
    const int sx = C.sock_of_node[gk[x]], sy = C.sock_of_node[gk[y]];
    if (colo[sx] != colo[sy]) return colo[sx] > colo[sy] ? 1 : -1;
    if (sfree[sx] != sfree[sy]) return free_before(a.most, sfree[sx], sfree[sy]) ? 1 : -1;
    if (nfree[gk[x]] != nfree[gk[y]]) return free_before(a.most, nfree[gk[x]], nfree[gk[y]]) ? 1 : -1;
    if (gc[x] != gc[y]) return gc[x] < gc[y] ? 1 : -1;
    if (sx != sy) return sx < sy ? 1 : -1;
    return 0;
  };
  for (int i = 1; i < ng; i++)
    for (int j = i; j > 0 && before(j, j - 1) > 0; j--) {
      const int tk = gk[j], tc = gc[j];
      gk[j] = gk[j - 1];
      gc[j] = gc[j - 1];
      gk[j - 1] = tk;
      gc[j - 1] = tc;
    }
  // the list: merged groups in order, cores ascending, CPUs ascending by id (= t order)
  // collected as positions; then spread (round t = t-th CPU of each listed core)
  int16_t lst[KOORDHIP_NUMA_MAX_CPUS];
  int nl = 0;
  for (int g0 = 0; g0 < ng;) {
    int g1 = g0 + 1;
    while (g1 < ng && before(g0, g1) == 0) g1++;
    uint64_t lead[NW] = {0, 0, 0, 0};
    for (int g = g0; g < g1; g++)
      for (int w = 0; w < NW; w++) {
        const uint64_t nmF = F[w] & C.nm[gk[g]][w];
        const uint64_t any = fold_or(nmF, C.cpc), all = fold_and(nmF, C.cpc);
        lead[w] |= (gc[g] == C.cpc) ? all : (any & ~all);  // cpc <= 2: 1 CPU or both
      }
    for (int w = 0; w < NW; w++) {
      uint64_t x = lead[w];
      while (x) {
        const int b = __builtin_ctzll(x);
        x &= x - 1;
        for (int t = 0; t < C.cpc; t++)
          if (tbit(F, w * 64 + b + t)) lst[nl++] = (int16_t)(w * 64 + b + t);
      }
    }
    g0 = g1;
  }
  if (nl > C.cpc) {
    // spreadCPUs: stable rounds over the listed order
    uint64_t done[NW] = {0, 0, 0, 0};
    for (int round = 0; round < C.cpc && a.need > 0; round++) {
      uint64_t seen[NW] = {0, 0, 0, 0};
      for (int i = 0; i < nl && a.need > 0; i++) {
        const int p = lst[i];
        if (tbit(done, p)) continue;
        const int lead = p - (p % C.cpc);
        if (tbit(seen, lead)) continue;
        sbit(seen, lead);
        sbit(done, p);
        acc_take1(C, a, p);
      }
    }
  } else {
    for (int i = 0; i < nl && a.need > 0; i++) acc_take1(C, a, lst[i]);
  }
}

// The len-only socket sorts (cpu_accumulator.go:142-144, 161-163) with go 1.18's
// sort.Slice for <= 12 elements (go.mod:3; zsortfunc.go quickSort_func): one
// shell pass with gap 6, then an insertion sort.  The gap pass is not stable:
// 7-8 tied sockets come out in Go's order, not in a stable sort's.
__device__ __forceinline__ void go118_sort_by_count(int *ord, int *cnt, int n, bool desc) {
  auto less = [&](int x, int y) { return desc ? cnt[x] > cnt[y] : cnt[x] < cnt[y]; };
  auto swp = [&](int x, int y) {
    const int to = ord[x], tc = cnt[x];
    ord[x] = ord[y];
    cnt[x] = cnt[y];
    ord[y] = to;
    cnt[y] = tc;
  };
  for (int i = 6; i < n; i++)
    if (less(i, i - 6)) swp(i, i - 6);
  for (int i = 1; i < n; i++)
    for (int j = i; j > 0 && less(j, j - 1); j--) swp(j, j - 1);
}

// takeCPUs; returns true with a.R filled.
template <bool WAVE = false>
__device__ __forceinline__ bool acc_take_cpus(const DevNumaClass &C, Acc &a, int policy) {
  if (a.need < 1) return true;
  if (a.need > popc4(a.A)) return false;
  const int cpc = C.cpc;
  const bool full = policy == (int)KOORDHIP_CPUBIND_FULL_PCPUS;
  uint64_t FA[NW], T[NW], X[NW];
  if (full || cpc == 1) {
    if (a.need <= C.cpn) {  // :111-121
      for (int fe = 1; fe >= 0; fe--) {
        if (fe) acc_excluded(C, a, false, X);
        for (int w = 0; w < NW; w++) {
          uint64_t allowed = a.A[w];
          if (fe && a.excl == (int)KOORDHIP_CPUEXCL_NUMA) allowed &= ~X[w];  // NUMANodeLevel only (:377)
          FA[w] = expand(fold_and(allowed, cpc), cpc);
          X[w] = fe ? X[w] : 0;
        }
        int bkey = 0;
        for (int k = 0; k < C.nnuma; k++) {
          const int cnt = popc_and(FA, C.nm[k]);
          if (cnt < a.need) continue;
          int sf = 0;  // socketFreeScores: allowed CPUs of the node's socket
          for (int w = 0; w < NW; w++) {
            uint64_t allowed = a.A[w];
            if (fe && a.excl == (int)KOORDHIP_CPUEXCL_NUMA) allowed &= ~X[w];
            sf += __popcll(allowed & C.sm[C.sock_of_node[k]][w]);
          }
          bkey = max(bkey, sel_key(a.most, cnt, sf, k));
        }
        const int best = sel_index(bkey);
        if (best >= 0) {
          for (int w = 0; w < NW; w++) T[w] = FA[w] & C.nm[best][w];
          acc_take_low(C, a, T, a.need);
          return true;
        }
      }
    }
    for (int w = 0; w < NW; w++) FA[w] = expand(fold_and(a.A[w], cpc), cpc);
    if (a.need <= C.cps) {  // :126-134
      int bkey = 0;
      for (int s = 0; s < C.nsock; s++) {
        const int cnt = popc_and(FA, C.sm[s]);
        if (cnt < a.need) continue;
        bkey = max(bkey, sel_key(a.most, cnt, 0, s));
      }
      const int best = sel_index(bkey);
      if (best >= 0) {
        for (int w = 0; w < NW; w++) T[w] = FA[w] & C.sm[best][w];
        acc_take_low(C, a, T, a.need);
        return true;
      }
    }
    // :141-155: sockets (in strategy order, then stably by count desc)
    int ord[NMAX], cnt[NMAX], no = 0;
    for (int s = 0; s < C.nsock; s++) {
      const int c = popc_and(FA, C.sm[s]);
      if (c == 0) continue;
      int j = no++;
      // strategy order: (count per strategy, id)
      while (j > 0 && free_before(a.most, c, cnt[j - 1])) {
        ord[j] = ord[j - 1];
        cnt[j] = cnt[j - 1];
        j--;
      }
      ord[j] = s;
      cnt[j] = c;
    }
    go118_sort_by_count(ord, cnt, no, true);  // count desc (go 1.18 sort.Slice)
    int uo[NMAX], uc[NMAX], nu = 0;
    for (int i = 0; i < no; i++) {
      if (a.need < cnt[i]) {
        uo[nu] = ord[i];
        uc[nu] = cnt[i];
        nu++;
      } else {
        for (int w = 0; w < NW; w++) T[w] = FA[w] & C.sm[ord[i]][w];
        acc_take_low(C, a, T, cnt[i]);
        if (a.need < 1) return true;
      }
    }
    if (a.need >= cpc) {  // :159-176: deferred sockets by count asc, core by core
      go118_sort_by_count(uo, uc, nu, false);  // count asc (go 1.18 sort.Slice)
      for (int i = 0; i < nu; i++) {
        for (int w = 0; w < NW; w++) T[w] = FA[w] & C.sm[uo[i]][w];
        bool stop = false;
#pragma unroll
        for (int w = 0; w < NW; w++) {  // (unrolled: T stays in registers)
          uint64_t x = stop ? 0ull : T[w];
          while (x) {
            const int b = __builtin_ctzll(x);
            uint64_t core = (cpc == 1) ? (1ull << b) : (3ull << b);
            x &= ~core;
            for (int t = 0; t < cpc; t++) acc_take1(C, a, w * 64 + b + t);
            if (a.need < 1) return true;
            if (a.need < cpc) {
              stop = true;
              break;
            }
          }
        }
      }
    }
  }
  if (!full) {
    if (a.need <= C.cpn) {  // :187-199
      for (int fe = 1; fe >= 0; fe--) {
        if (fe) acc_excluded(C, a, false, X);
        uint64_t Fl[NW];
        for (int w = 0; w < NW; w++) Fl[w] = a.A[w] & ~(fe ? X[w] : 0ull);
        int bkey = 0;
        for (int k = 0; k < C.nnuma; k++) {
          const int nf = popc_and(Fl, C.nm[k]);
          if (nf == 0) continue;
          const int len = fe ? cores_in(Fl, C.nm[k], cpc) : nf;
          if (len < a.need) continue;
          const int sf = popc_and(Fl, C.sm[C.sock_of_node[k]]);
          bkey = max(bkey, sel_key(a.most, nf, sf, k));
        }
        const int best = sel_index(bkey);
        if (best >= 0) {
          for (int w = 0; w < NW; w++) T[w] = Fl[w] & C.nm[best][w];
          if (fe) {  // extractCPU: each core's lowest-id allowed CPU
            uint64_t E[NW];
            for (int w = 0; w < NW; w++) {
              const uint64_t any = fold_or(T[w], cpc);
              E[w] = cpc == 1 ? T[w] : ((T[w] & 0x5555555555555555ull) | ((any & ~T[w]) << 1));
            }
            acc_take_spread_by_id<WAVE>(C, a, E, a.need);
          } else {
            acc_take_spread_by_id<WAVE>(C, a, T, a.need);
          }
          return true;
        }
      }
    }
    if (a.need <= C.cps) {  // :203-214
      for (int fe = 1; fe >= 0; fe--) {
        if (fe) acc_excluded(C, a, true, X);
        uint64_t Fl[NW];
        for (int w = 0; w < NW; w++) Fl[w] = a.A[w] & ~(fe ? X[w] : 0ull);
        int bkey = 0;
        for (int s = 0; s < C.nsock; s++) {
          const int nf = popc_and(Fl, C.sm[s]);
          if (nf == 0) continue;
          const int len = fe ? cores_in(Fl, C.sm[s], cpc) : nf;
          if (len < a.need) continue;
          bkey = max(bkey, sel_key(a.most, len, 0, s));
        }
        const int best = sel_index(bkey);
        if (best >= 0) {
          for (int w = 0; w < NW; w++) T[w] = Fl[w] & C.sm[best][w];
          if (fe) {
            uint64_t E[NW];
            for (int w = 0; w < NW; w++) {
              const uint64_t any = fold_or(T[w], cpc);
              E[w] = cpc == 1 ? T[w] : ((T[w] & 0x5555555555555555ull) | ((any & ~T[w]) << 1));
            }
            acc_take_spread_by_id<WAVE>(C, a, E, a.need);
          } else {
            acc_take_spread_by_id<WAVE>(C, a, T, a.need);
          }
          return true;
        }
      }
    }
  }
  acc_fallback_pass(C, a, true);
  if (a.need < 1) return true;
  acc_fallback_pass(C, a, false);
  return a.need < 1;
}

// takeCPUs over the available set A (cpu_accumulator.go:87-232) into out[]
template <bool WAVE = false>
__device__ __forceinline__ bool acc_run(const DevNumaClass &C, const NumaRow &r, const DevPod &p,
                                                  const uint64_t *A, int need, uint64_t *out) {
  Acc a;
  for (int w = 0; w < NW; w++) {
    a.A[w] = A[w];
    a.R[w] = 0;
    a.XC[w] = fold_or(r.ep[w], C.cpc);
  }
  a.XN = 0;
  for (int k = 0; k < C.nnuma; k++)
    if (popc_and(r.en, C.nm[k])) a.XN |= 1u << k;
  a.need = need;
  a.excl = (int)KOORDHIP_NUMA_EXCLUSIVE(p.numa_policy);
  a.most = (r.nflags & KOORDHIP_NODE_NUMA_MOST_ALLOCATED) ? 1 : 0;
  const int pol = node_policy(r.nflags, (int)KOORDHIP_NUMA_PREFERRED(p.numa_policy));
  const bool ok = acc_take_cpus<WAVE>(C, a, pol);
  for (int w = 0; w < NW; w++) out[w] = a.R[w];
  return ok;
}

// satisfiedRequiredCPUBindPolicy (resource_manager.go:442-463) on the result
__device__ __forceinline__ bool required_ok(const DevNumaClass &C, const NumaRow &r, const DevPod &p,
                                            const uint64_t *R) {
  if (KOORDHIP_NUMA_REQUIRED(p.numa_policy) == KOORDHIP_CPUBIND_NONE) return true;
  const int pol = node_policy(r.nflags, (int)KOORDHIP_NUMA_PREFERRED(p.numa_policy));
  int n = popc4(R), cores = 0;
  for (int w = 0; w < NW; w++) cores += __popcll(fold_or(R[w], C.cpc));
  if (pol == (int)KOORDHIP_CPUBIND_FULL_PCPUS && cores * C.cpc != n) return false;
  if (pol == (int)KOORDHIP_CPUBIND_SPREAD_BY_PCPUS && cores != n) return false;
  return true;
}

// Allocate for Reserve: exact CPUs into cpus[]; false = Allocate fails.
template <bool WAVE = false>
__device__ __forceinline__ bool numa_allocate_in(const DevNumaClass &C, const NumaRow &r, const DevPod &p, uint64_t *cpus) {
  for (int w = 0; w < NW; w++) cpus[w] = 0;
  const int need = p.numa_cpus;
  if (popc4(r.fr) < need) return false;
  uint64_t R[NW];
  if (!acc_run<WAVE>(C, r, p, r.fr, need, R)) return false;
  if (!required_ok(C, r, p, R)) return false;
  for (int w = 0; w < NW; w++) cpus[w] = R[w];
  return true;
}

// Allocate with reservation-preferred CPUs P (getResourceOptions' preferredCPUs,
// plugin.go:503-524; no hint): the available set is free | P -- P's RefCount
// drops to 0 in getAvailableCPUs, so its exclusive policy leaves allocateInfo
// too (node_allocation.go:133-153) -- and takePreferredCPUs
// (cpu_accumulator.go:29-85) takes min(need, |P|) CPUs from P, then the rest
// from the available CPUs outside P, each by its own accumulator over the
// same allocateInfo; the required bind policy holds for the union
// (resource_manager.go:244-326).
template <bool WAVE = false>
__device__ __forceinline__ bool numa_allocate_pref_in(const DevNumaClass &C, const NumaRow &r, const DevPod &p,
                                                      const uint64_t *P, uint64_t *cpus) {
  for (int w = 0; w < NW; w++) cpus[w] = 0;
  const int need = p.numa_cpus;
  uint64_t A[NW];
  for (int w = 0; w < NW; w++) A[w] = r.fr[w] | P[w];
  if (popc4(A) < need) return false;
  NumaRow q = r;
  for (int w = 0; w < NW; w++) {
    q.ep[w] &= ~P[w];
    q.en[w] &= ~P[w];
    A[w] &= ~P[w];
  }
  const int np = popc4(P);
  const int n1 = need < np ? need : np;
  uint64_t R1[NW] = {0, 0, 0, 0}, R2[NW] = {0, 0, 0, 0};
  if (n1 > 0 && !acc_run<WAVE>(C, q, p, P, n1, R1)) return false;
  if (need > n1 && !acc_run<WAVE>(C, q, p, A, need - n1, R2)) return false;
  for (int w = 0; w < NW; w++) R1[w] |= R2[w];
  if (!required_ok(C, r, p, R1)) return false;
  for (int w = 0; w < NW; w++) cpus[w] = R1[w];
  return true;
}

__device__ __forceinline__ bool any4(const uint64_t *m) { return (m[0] | m[1] | m[2] | m[3]) != 0ull; }

// Score-time Allocate with reservation-preferred CPUs (outlined: only cpuset
// pods on nodes whose nominated reservation holds CPUs get here)
__device__ __attribute__((noinline)) bool numa_allocate_pref(const DevNumaClass &C, const NumaRow &r, const DevPod &p,
                                                             uint64_t P0, uint64_t P1, uint64_t P2, uint64_t P3) {
  const NumaRow rl = r;
  const DevPod pl = p;
  const uint64_t P[NW] = {P0, P1, P2, P3};
  uint64_t o[NW];
  return numa_allocate_pref_in(C, rl, pl, P, o);
}

// The outlined entry points copy their by-reference inputs into registers
// first: the accumulator then never touches the caller's stack copy.
__device__ __attribute__((noinline)) bool numa_allocate(const DevNumaClass &C, const NumaRow &r, const DevPod &p, uint64_t *cpus) {
  const NumaRow rl = r;
  const DevPod pl = p;
  uint64_t o[NW];
  const bool ok = numa_allocate_in(C, rl, pl, o);
  for (int w = 0; w < NW; w++) cpus[w] = o[w];
  return ok;
}

// ---------------------------------------------------------------------------
// NUMA topology policies (frameworkext/topologymanager, topology_hint.go,
// resource_manager.go:142-242,384-428).  The plugin is the only hint
// provider; its hints for cpu and memory (the requested ones) are the same
// list S of zone masks whose summed availability covers the request,
// preferred = minimal size.  Merging one hint per list (policy.go:52-208) then
// has a closed form: with one list the narrowest minimal mask, with two the
// narrowest non-empty AND of two minimal masks; no list or an empty S is a
// provider without preference ({default affinity, preferred}).

// getAvailableNUMANodeResources: allocatable - allocated, non-negative, of
// every zone (one pass over the row's HBM allocatable)
__device__ __forceinline__ void zone_avail_all(const NumaRow &r, int M, double av[2][ZMAX]) {
#pragma unroll
  for (int k = 0; k < ZMAX; k++)
#pragma unroll
    for (int q = 0; q < 2; q++) {
      const double a = k < M ? r.za[q * ZMAX + k] - r.zu[q][k] : 0.0;
      av[q][k] = a > 0.0 ? a : 0.0;
    }
}

// ... with getResourceOptions' reusableResources (plugin.go:469-479,
// node_allocation.go:155-177): zone k's allocated cpu less ru[k] (the
// nominated reservation's reserved CPUs in zone k x 1000), non-negative
__device__ __forceinline__ double zone_cpu_allocated(const NumaRow &r, int k, const double ru[ZMAX]) {
  const double u = r.zu[0][k] - ru[k];
  return u > 0.0 ? u : 0.0;
}
__device__ __forceinline__ void zone_avail_reus(const NumaRow &r, int M, const double ru[ZMAX], double av[2][ZMAX]) {
#pragma unroll
  for (int k = 0; k < ZMAX; k++) {
    const double ac = k < M ? r.za[k] - zone_cpu_allocated(r, k, ru) : 0.0;
    const double am = k < M ? r.za[ZMAX + k] - r.zu[1][k] : 0.0;
    av[0][k] = ac > 0.0 ? ac : 0.0;
    av[1][k] = am > 0.0 ? am : 0.0;
  }
}
// ru[k]: the reservation-preferred CPUs P in zone k x 1000 (no amplification on policy nodes)
__device__ __forceinline__ void zone_reusable(const DevNumaClass &C, const uint64_t *P, double ru[ZMAX]) {
#pragma unroll
  for (int k = 0; k < ZMAX; k++) ru[k] = k < C.nnuma ? (double)popc_and(P, C.nm[k]) * 1000.0 : 0.0;
}

// bitmask.IsNarrowerThan order as one integer (masks < 256)
__device__ __forceinline__ int narrow_key(uint32_t m) { return __popc(m) * 256 + (int)m; }

// Merge + canAdmitPodResult for policy tp; *mask = the hint (0 = nil affinity).
// S (256 bits): the zone masks whose summed availability covers the request,
// enumerated in Gray-code order so each mask's sums are one add / subtract
// away from the previous mask's (exact: integers below 2^53).
__device__ __forceinline__ bool zone_hint(int M, const double av[2][ZMAX], const DevPod &p, int tp, uint32_t *mask) {
  const double qc = p.req[KOORDHIP_RES_CPU], qm = p.req[KOORDHIP_RES_MEM];
  const bool rc = qc != 0.0, rm = qm != 0.0;
  const uint32_t all = (1u << M) - 1u;
  uint32_t S[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int minsize = M;
  double sc = 0.0, sm = 0.0;
  for (uint32_t i = 1; i <= all; i++) {  // generateResourceHints :384-428
    const uint32_t m = i ^ (i >> 1), b = __builtin_ctz(i);
    const double dc = av[0][0], dm = av[1][0];  // (placeholders: the switch below picks zone b)
    double zc = dc, zm = dm;
#pragma unroll
    for (int k = 1; k < ZMAX; k++)
      if ((int)b == k) {
        zc = av[0][k];
        zm = av[1][k];
      }
    if ((m >> b) & 1u) {
      sc += zc;
      sm += zm;
    } else {
      sc -= zc;
      sm -= zm;
    }
    if ((!rc || qc <= sc) && (!rm || qm <= sm)) {
#pragma unroll
      for (int w = 0; w < 8; w++)
        if ((int)(m >> 5) == w) S[w] |= 1u << (m & 31);
      minsize = min(minsize, __popc(m));
    }
  }
  auto inS = [&](uint32_t m) -> bool {
    uint32_t x = 0;
#pragma unroll
    for (int w = 0; w < 8; w++)
      if ((int)(m >> 5) == w) x = S[w];
    return (x >> (m & 31)) & 1u;
  };
  bool any = false;
#pragma unroll
  for (int w = 0; w < 8; w++) any |= S[w] != 0u;
  if ((!rc && !rm) || !any) {  // no hints: {default, preferred}
    *mask = tp == (int)KOORDHIP_NUMA_TOPO_SINGLE_NUMA_NODE ? 0u : all;
    return true;
  }
  if (tp == (int)KOORDHIP_NUMA_TOPO_SINGLE_NUMA_NODE) {  // policy_single_numa_node.go:37-78
    if (minsize != 1) return false;                        // nothing survives the filter: {default, false}
    uint32_t best = 0;
    for (int k = M - 1; k >= 0; k--)
      if (inS(1u << k)) best = 1u << k;
    *mask = best == all ? 0u : best;
    return true;
  }
  // preferred merged hints: AND of one minimal mask per requested resource
  // (both lists are S); the narrowest non-empty one wins (policy.go:124-169)
  uint32_t best = all;
  int bk = 1 << 30;
  for (uint32_t a = 1; a <= all; a++) {
    if (__popc(a) != minsize || !inS(a)) continue;
    if (narrow_key(a) < bk) {  // a & a
      bk = narrow_key(a);
      best = a;
    }
    if (!(rc && rm)) continue;
    for (uint32_t b = a + 1; b <= all; b++) {
      if (__popc(b) != minsize || !(a & b) || narrow_key(a & b) >= bk || !inS(b)) continue;
      bk = narrow_key(a & b);
      best = a & b;
    }
  }
  *mask = best;
  return true;  // preferred: BestEffort and Restricted admit
}

// allocateResourcesByHint (:166-242): the hinted zones in ascending id take
// min(available, still requested) of cpu and memory
__device__ __forceinline__ bool zone_alloc(int M, const double av[2][ZMAX], const DevPod &p, uint32_t mask,
                                           double z[2][ZMAX]) {
  double rem[2] = {p.req[KOORDHIP_RES_CPU], p.req[KOORDHIP_RES_MEM]};
#pragma unroll
  for (int k = 0; k < ZMAX; k++) {
    z[0][k] = 0.0;
    z[1][k] = 0.0;
    if (k < M && ((mask >> k) & 1u)) {
#pragma unroll
      for (int q = 0; q < 2; q++) {
        const double a = av[q][k] < rem[q] ? av[q][k] : rem[q];
        z[q][k] = a;
        rem[q] -= a;
      }
    }
  }
  return rem[0] == 0.0 && rem[1] == 0.0;
}

__device__ __forceinline__ bool zone_used(const double z[2][ZMAX], int k) { return z[0][k] != 0.0 || z[1][k] != 0.0; }

// allocateCPUSet with allocated NUMA nodes (:264-295): zone k takes
// min(|its available CPUs|, floor(cpu_k / 1000)) CPUs; the sum must be exact.
// Preferred-only: takeCPUs never fails below |available| (closed form).
// P: reservation-preferred CPUs (allocated, so disjoint from the free ones;
// GetAvailableCPUs makes them available), NULL: none.  *taken_p: how many of
// P the zones' takePreferredCPUs take (min(n_k, |P in zone k|) each).
__device__ __forceinline__ bool zone_cpus_ok(const DevNumaClass &C, const NumaRow &r, const DevPod &p,
                                             const double z[2][ZMAX], const uint64_t *P = nullptr,
                                             int *taken_p = nullptr) {
  uint64_t A[NW];
  for (int w = 0; w < NW; w++) A[w] = r.fr[w] | (P ? P[w] : 0ull);
  if (popc4(A) < p.numa_cpus) return false;
  int got = 0, tp = 0;
  for (int k = 0; k < C.nnuma && k < ZMAX; k++)
    if (zone_used(z, k)) {
      const int n = min(popc_and(A, C.nm[k]), (int)((long long)z[0][k] / 1000));
      got += n;
      if (P) tp += min(n, popc_and(P, C.nm[k]));
    }
  if (taken_p) *taken_p = tp;
  return got == p.numa_cpus;
}

// ... exact CPUs (Reserve, and Filter / Score under a required policy).
// P (NULL: none): each zone's takePreferredCPUs (cpu_accumulator.go:29-85)
// takes from P's CPUs in the zone first, then from the zone's others, both
// over the allocateInfo P has left (numa_allocate_pref_in)
__device__ __forceinline__ bool zone_allocate_in(const DevNumaClass &C, const NumaRow &r, const DevPod &p,
                                                 const double z[2][ZMAX], uint64_t *cpus,
                                                 const uint64_t *P = nullptr) {
  for (int w = 0; w < NW; w++) cpus[w] = 0;
  NumaRow q = r;
  uint64_t PP[NW];
  for (int w = 0; w < NW; w++) {
    PP[w] = P ? P[w] : 0ull;
    q.fr[w] |= PP[w];
    q.ep[w] &= ~PP[w];
    q.en[w] &= ~PP[w];
  }
  if (popc4(q.fr) < p.numa_cpus) return false;
  int got = 0;
  for (int k = 0; k < C.nnuma && k < ZMAX; k++) {
    if (!zone_used(z, k)) continue;
    uint64_t A[NW], B[NW], o[NW];
    for (int w = 0; w < NW; w++) {
      A[w] = q.fr[w] & C.nm[k][w] & ~PP[w];
      B[w] = PP[w] & C.nm[k][w];
    }
    const int n = min(popc4(A) + popc4(B), (int)((long long)z[0][k] / 1000));
    if (n <= 0) continue;
    const int n1 = min(n, popc4(B));
    if (n1 > 0) {
      if (!acc_run(C, q, p, B, n1, o)) return false;
      for (int w = 0; w < NW; w++) cpus[w] |= o[w];
      got += popc4(o);
    }
    if (n > n1) {
      if (!acc_run(C, q, p, A, n - n1, o)) return false;
      for (int w = 0; w < NW; w++) cpus[w] |= o[w];
      got += popc4(o);
    }
  }
  if (got != p.numa_cpus) return false;
  return required_ok(C, r, p, cpus);
}

__device__ __attribute__((noinline)) bool zone_allocate(const DevNumaClass &C, const NumaRow &r, const DevPod &p,
                                                        const double z[2][ZMAX], uint64_t *cpus,
                                                        const uint64_t *P = nullptr) {
  const NumaRow rl = r;
  const DevPod pl = p;
  double zl[2][ZMAX];
  for (int q = 0; q < 2; q++)
    for (int k = 0; k < ZMAX; k++) zl[q][k] = z[q][k];
  uint64_t o[NW], pl4[NW];
  for (int w = 0; w < NW; w++) pl4[w] = P ? P[w] : 0ull;
  const bool ok = zone_allocate_in(C, rl, pl, zl, o, P ? pl4 : nullptr);
  for (int w = 0; w < NW; w++) cpus[w] = o[w];
  return ok;
}

// Filter's FilterByNUMANode -> Admit -> Allocate on a policy node (topology_hint.go:30-86)
__device__ __forceinline__ bool numa_policy_ok(const DevNumaClass &C, const NumaRow &r, const DevPod &p) {
  uint32_t mask;
  double av[2][ZMAX];
  zone_avail_all(r, C.nnuma, av);
  if (!zone_hint(C.nnuma, av, p, topo_policy(r.nflags), &mask)) return false;
  double z[2][ZMAX];
  if (mask && !zone_alloc(C.nnuma, av, p, mask, z)) return false;
  if (!(p.flags & KOORDHIP_POD_CPUSET)) return true;
  if (!mask) return numa_alloc_ok(C, r, p);
  if (KOORDHIP_NUMA_REQUIRED(p.numa_policy) == KOORDHIP_CPUBIND_NONE) return zone_cpus_ok(C, r, p, z);
  uint64_t m[NW];
  return zone_allocate(C, r, p, z, m);
}

}  // namespace kh
