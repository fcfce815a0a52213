/*
 * numa_oracle.c -- TEST INFRASTRUCTURE (see koord_oracle.h).  Plain-C
 * restatement of NodeNUMAResource:
 *   - the cpuAccumulator (pkg/scheduler/plugins/nodenumaresource/cpu_accumulator.go),
 *     kept in the reference's own shape: per-call grouping of the allocatable
 *     CPUs into per-core / per-NUMA-node / per-socket lists, the same sort
 *     keys, the same passes;
 *   - Allocate / allocateCPUSet / satisfiedRequiredCPUBindPolicy
 *     (resource_manager.go:142-164,244-326,442-463);
 *   - Filter / Score / Reserve (plugin.go:266-324,365-405, scoring.go:55-168);
 *   - NUMA topology policies: the topology manager's hint merge and admit
 *     (frameworkext/topologymanager/manager.go:58-111, policy*.go), the
 *     plugin's hints (topology_hint.go:30-86, resource_manager.go:384-428)
 *     and allocateResourcesByHint (:166-242).
 * Go's sort.Slice is not stable.  Every comparator but two ends in an id
 * tie-break, so any correct sort gives Go's order; those are insertion sorts
 * here.  The two len-only socket sorts (cpu_accumulator.go:142-144, 161-163)
 * reproduce go 1.18's sort.Slice for <= 12 elements exactly (a gap-6 shell
 * pass, then insertion sort: sort_groups_len), which differs from a stable
 * sort when 7-8 sockets tie.
 * Pinned by the known-answer tables of cpu_accumulator_test.go (tests/golden/).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "koord_oracle.h"

#define MAXC KOORDHIP_NUMA_MAX_CPUS
#define MAXG 16

typedef struct acc {
  const koordhip_numa_class *t;
  int ncpu, cpc, cpn, cps; /* CPUsPerCore / PerNode / PerSocket (cpu_topology.go:82-103) */
  uint8_t allocatable[MAXC];
  int need;
  int excl_policy; /* pod's preferredCPUExclusivePolicy */
  int exclusive;
  uint8_t excl_core[MAXC];               /* exclusiveInCores, by core rank */
  uint8_t excl_node[KOORDHIP_NUMA_MAX_NODES]; /* exclusiveInNUMANodes */
  int most_allocated;
  uint8_t result[MAXC];
  int nresult;
} acc;

typedef struct list {
  int n;
  int16_t v[MAXC];
} list;

typedef struct groups {
  int n;
  int id[MAXG];
  list l[MAXG];
} groups;

static int core_of(const acc *a, int p) { return p / a->cpc; }
static int node_of(const acc *a, int p) { return a->t->node_of[p]; }
static int sock_of(const acc *a, int p) { return a->t->socket_of[p]; }
static int cpuid(const acc *a, int p) { return a->t->cpu_id[p]; }

static int bit(const uint64_t *m, int p) { return (int)((m[p >> 6] >> (p & 63)) & 1u); }

/* newCPUAccumulator, cpu_accumulator.go:247-288 (maxRefCount = 1). */
static void acc_init(acc *a, const koordhip_numa_class *t, const uint64_t *avail, const uint64_t *excl_pcpu,
                     const uint64_t *excl_numa, int need, int excl_policy, int most_allocated) {
  memset(a, 0, sizeof(*a));
  a->t = t;
  a->ncpu = t->num_cpus;
  a->cpc = t->num_cores ? t->num_cpus / t->num_cores : 0;
  a->cpn = t->num_nodes ? t->num_cpus / t->num_nodes : 0;
  a->cps = t->num_sockets ? t->num_cpus / t->num_sockets : 0;
  for (int p = 0; p < a->ncpu; p++) {
    a->allocatable[p] = (uint8_t)bit(avail, p);
    if (excl_pcpu && bit(excl_pcpu, p)) a->excl_core[p / a->cpc] = 1; /* :258-261 */
    if (excl_numa && bit(excl_numa, p)) a->excl_node[t->node_of[p]] = 1;
  }
  a->need = need;
  a->excl_policy = excl_policy;
  a->exclusive = excl_policy == KOORDHIP_CPUEXCL_PCPU || excl_policy == KOORDHIP_CPUEXCL_NUMA; /* :265-266 */
  a->most_allocated = most_allocated;
}

/* take, :290-304 */
static void acc_take(acc *a, const int16_t *cpus, int n) {
  for (int i = 0; i < n; i++) {
    int p = cpus[i];
    if (!a->result[p]) a->nresult++;
    a->result[p] = 1;
    a->allocatable[p] = 0;
    if (a->exclusive) {
      if (a->excl_policy == KOORDHIP_CPUEXCL_PCPU) a->excl_core[core_of(a, p)] = 1;
      else a->excl_node[node_of(a, p)] = 1;
    }
  }
  a->need -= n;
}
static int acc_needs(const acc *a, int n) { return a->need >= n; }
static int acc_satisfied(const acc *a) { return a->need < 1; }
static int acc_navail(const acc *a) {
  int c = 0;
  for (int p = 0; p < a->ncpu; p++) c += a->allocatable[p];
  return c;
}
static int acc_failed(const acc *a) { return a->need > acc_navail(a); }

static int excl_pcpu_level(const acc *a, int p) {
  return a->excl_policy == KOORDHIP_CPUEXCL_PCPU && a->excl_core[core_of(a, p)]; /* :318-323 */
}
static int excl_numa_level(const acc *a, int p) {
  return a->excl_policy == KOORDHIP_CPUEXCL_NUMA && a->excl_node[node_of(a, p)]; /* :325-330 */
}

/* sort.Ints on positions by CPU id (insertion sort) */
static void sort_by_cpuid(const acc *a, int16_t *v, int n) {
  for (int i = 1; i < n; i++) {
    int16_t x = v[i];
    int j = i - 1;
    while (j >= 0 && cpuid(a, v[j]) > cpuid(a, x)) {
      v[j + 1] = v[j];
      j--;
    }
    v[j + 1] = x;
  }
}

/* extractCPU, :332-343: first CPU of each core, in list order */
static void extract_cpu(const acc *a, list *l) {
  uint8_t seen[MAXC];
  memset(seen, 0, sizeof(seen));
  int m = 0;
  for (int i = 0; i < l->n; i++) {
    int c = core_of(a, l->v[i]);
    if (!seen[c]) {
      seen[c] = 1;
      l->v[m++] = l->v[i];
    }
  }
  l->n = m;
}

/* spreadCPUs, :798-822 */
static void spread_cpus(const acc *a, list *l) {
  if (l->n <= a->cpc) return;
  list prep = *l, keep;
  l->n = 0;
  while (prep.n > 0) {
    uint8_t seen[MAXC];
    memset(seen, 0, sizeof(seen));
    keep.n = 0;
    for (int i = 0; i < prep.n; i++) {
      int c = core_of(a, prep.v[i]);
      if (seen[c]) {
        keep.v[keep.n++] = prep.v[i];
        continue;
      }
      l->v[l->n++] = prep.v[i];
      seen[c] = 1;
    }
    prep = keep;
  }
}

/* strategy comparison of free scores: MostAllocated -> ascending (:434-438) */
static int free_before(const acc *a, int x, int y) { return a->most_allocated ? x < y : x > y; }

/* Per-core allowed CPUs (ascending CPU id) for a predicate. */
typedef int (*allow_fn)(const acc *a, int p);

/* freeCoresInNode (by_socket = 0, :371-461) / freeCoresInSocket (by_socket = 1, :464-527) */
static void free_cores(const acc *a, int by_socket, int filter_full, int filter_excl, groups *out) {
  int core_cnt[MAXC];
  int socket_free[KOORDHIP_NUMA_MAX_NODES];
  memset(core_cnt, 0, sizeof(core_cnt));
  memset(socket_free, 0, sizeof(socket_free));
  for (int p = 0; p < a->ncpu; p++) {
    if (!a->allocatable[p]) continue;
    if (!by_socket && filter_excl && excl_numa_level(a, p)) continue;
    core_cnt[core_of(a, p)]++;
    socket_free[sock_of(a, p)]++;
  }
  const int ncores = a->ncpu / a->cpc;
  /* group -> cores (ascending core id == sortCores order: all counts equal
   * when filter_full; otherwise count desc then core id, :345-368) */
  out->n = 0;
  int gid_of[KOORDHIP_NUMA_MAX_NODES];
  for (int g = 0; g < KOORDHIP_NUMA_MAX_NODES; g++) gid_of[g] = -1;
  int core_list[KOORDHIP_NUMA_MAX_NODES][MAXC];
  int ncl[KOORDHIP_NUMA_MAX_NODES];
  memset(ncl, 0, sizeof(ncl));
  for (int c = 0; c < ncores; c++) {
    if (!core_cnt[c]) continue;
    if (filter_full && core_cnt[c] != a->cpc) continue;
    int first = c * a->cpc; /* any CPU of the core carries its node / socket */
    int g = by_socket ? sock_of(a, first) : node_of(a, first);
    core_list[g][ncl[g]++] = c;
  }
  for (int g = 0; g < KOORDHIP_NUMA_MAX_NODES; g++) {
    if (!ncl[g]) continue;
    /* sortCores: cpus count desc, core id asc (insertion) */
    for (int i = 1; i < ncl[g]; i++) {
      int x = core_list[g][i], j = i - 1;
      while (j >= 0 && (core_cnt[core_list[g][j]] < core_cnt[x] ||
                        (core_cnt[core_list[g][j]] == core_cnt[x] && core_list[g][j] > x))) {
        core_list[g][j + 1] = core_list[g][j];
        j--;
      }
      core_list[g][j + 1] = x;
    }
    list *l = &out->l[out->n];
    l->n = 0;
    for (int i = 0; i < ncl[g]; i++) {
      int c = core_list[g][i];
      int16_t tmp[8];
      int nt = 0;
      for (int t = 0; t < a->cpc; t++) {
        int p = c * a->cpc + t;
        if (a->allocatable[p] && !(!by_socket && filter_excl && excl_numa_level(a, p))) tmp[nt++] = (int16_t)p;
      }
      sort_by_cpuid(a, tmp, nt);
      for (int t = 0; t < nt; t++) l->v[l->n++] = tmp[t];
    }
    out->id[out->n] = g;
    gid_of[g] = out->n;
    out->n++;
  }
  /* order groups */
  for (int i = 1; i < out->n; i++) {
    int j = i;
    while (j > 0) {
      int x = j, y = j - 1; /* is x before y? */
      int lx = out->l[x].n, ly = out->l[y].n, before;
      if (lx != ly) {
        before = free_before(a, lx, ly);
      } else if (!by_socket) {
        int sx = socket_free[sock_of(a, out->l[x].v[0])], sy = socket_free[sock_of(a, out->l[y].v[0])];
        before = sx != sy ? free_before(a, sx, sy) : out->id[x] < out->id[y];
      } else {
        before = out->id[x] < out->id[y];
      }
      if (!before) break;
      int tid = out->id[x];
      out->id[x] = out->id[y];
      out->id[y] = tid;
      list tl = out->l[x];
      out->l[x] = out->l[y];
      out->l[y] = tl;
      j--;
    }
  }
  (void)gid_of;
}

/* freeCPUsInNode (by_socket = 0, :530-605) / freeCPUsInSocket (by_socket = 1, :608-656) */
static void free_cpus_in(const acc *a, int by_socket, int filter_excl, groups *out) {
  int gfree[KOORDHIP_NUMA_MAX_NODES], socket_free[KOORDHIP_NUMA_MAX_NODES];
  memset(gfree, 0, sizeof(gfree));
  memset(socket_free, 0, sizeof(socket_free));
  list lists[KOORDHIP_NUMA_MAX_NODES];
  for (int g = 0; g < KOORDHIP_NUMA_MAX_NODES; g++) lists[g].n = 0;
  for (int p = 0; p < a->ncpu; p++) {
    if (!a->allocatable[p]) continue;
    if (filter_excl) {
      if (excl_pcpu_level(a, p)) continue;
      if (!by_socket && excl_numa_level(a, p)) continue;
    }
    int g = by_socket ? sock_of(a, p) : node_of(a, p);
    lists[g].v[lists[g].n++] = (int16_t)p;
    gfree[g]++;
    socket_free[sock_of(a, p)]++;
  }
  out->n = 0;
  for (int g = 0; g < KOORDHIP_NUMA_MAX_NODES; g++) {
    if (!lists[g].n) continue;
    sort_by_cpuid(a, lists[g].v, lists[g].n);
    if (filter_excl) extract_cpu(a, &lists[g]);
    out->id[out->n] = g;
    out->l[out->n] = lists[g];
    out->n++;
  }
  for (int i = 1; i < out->n; i++) {
    int j = i;
    while (j > 0) {
      int x = j, y = j - 1, before;
      if (!by_socket) {
        int gx = out->id[x], gy = out->id[y];
        int sx = socket_free[sock_of(a, out->l[x].v[0])], sy = socket_free[sock_of(a, out->l[y].v[0])];
        if (gfree[gx] != gfree[gy]) before = free_before(a, gfree[gx], gfree[gy]);
        else if (sx != sy) before = free_before(a, sx, sy);
        else before = gx < gy;
      } else {
        int lx = out->l[x].n, ly = out->l[y].n; /* len after extractCPU, :637-646 */
        before = lx != ly ? free_before(a, lx, ly) : out->id[x] < out->id[y];
      }
      if (!before) break;
      int tid = out->id[x];
      out->id[x] = out->id[y];
      out->id[y] = tid;
      list tl = out->l[x];
      out->l[x] = out->l[y];
      out->l[y] = tl;
      j--;
    }
  }
}

/* freeCPUs, :666-774 */
static void free_cpus(const acc *a, int filter_excl, list *out) {
  const int ncores = a->ncpu / a->cpc;
  int core_cnt[MAXC], node_free[KOORDHIP_NUMA_MAX_NODES], socket_free[KOORDHIP_NUMA_MAX_NODES],
      colo[KOORDHIP_NUMA_MAX_NODES];
  memset(core_cnt, 0, sizeof(core_cnt));
  memset(node_free, 0, sizeof(node_free));
  memset(socket_free, 0, sizeof(socket_free));
  memset(colo, 0, sizeof(colo));
  uint8_t allowed[MAXC];
  for (int p = 0; p < a->ncpu; p++) {
    allowed[p] = a->allocatable[p] && !(filter_excl && (excl_pcpu_level(a, p) || excl_numa_level(a, p)));
    if (!allowed[p]) continue;
    core_cnt[core_of(a, p)]++;
    node_free[node_of(a, p)]++;
    socket_free[sock_of(a, p)]++;
  }
  /* socketColoScores: CPUs of the result on each socket (:690-694) */
  for (int p = 0; p < a->ncpu; p++)
    if (a->result[p]) colo[sock_of(a, p)]++;
  int cores[MAXC], nc = 0;
  for (int c = 0; c < ncores; c++)
    if (core_cnt[c]) cores[nc++] = c;
  for (int i = 1; i < nc; i++) {
    int j = i;
    while (j > 0) {
      int x = cores[j], y = cores[j - 1], before;
      int fx = x * a->cpc, fy = y * a->cpc;
      int sx = sock_of(a, fx), sy = sock_of(a, fy);
      int nx = node_of(a, fx), ny = node_of(a, fy);
      if (colo[sx] != colo[sy]) before = colo[sx] > colo[sy];
      else if (socket_free[sx] != socket_free[sy]) before = free_before(a, socket_free[sx], socket_free[sy]);
      else if (node_free[nx] != node_free[ny]) before = free_before(a, node_free[nx], node_free[ny]);
      else if (core_cnt[x] != core_cnt[y]) before = core_cnt[x] < core_cnt[y];
      else if (sx != sy) before = sx < sy;
      else before = x < y;
      if (!before) break;
      cores[j] = y;
      cores[j - 1] = x;
      j--;
    }
  }
  out->n = 0;
  for (int i = 0; i < nc; i++) {
    int16_t tmp[8];
    int nt = 0;
    for (int t = 0; t < a->cpc; t++) {
      int p = cores[i] * a->cpc + t;
      if (allowed[p]) tmp[nt++] = (int16_t)p;
    }
    sort_by_cpuid(a, tmp, nt);
    for (int t = 0; t < nt; t++) out->v[out->n++] = tmp[t];
  }
}

/* sort.Slice of groups by list length (desc = 1 / asc = 0), :142-144 / :161-163.
 * The reference builds with go 1.18 (go.mod:3), whose sort.Slice on n <= 12
 * elements (zsortfunc.go quickSort_func) runs ONE shell pass with gap 6 --
 * swap(i, i-6) when less(i, i-6), for i = 6 .. n-1 -- and then an insertion
 * sort.  The gap pass is not stable: with 7-8 sockets of tied length it can
 * reorder them, so it is reproduced here (and in numa.hpp) literally. */
static void swap_groups(groups *g, int x, int y) {
  list tl = g->l[x];
  g->l[x] = g->l[y];
  g->l[y] = tl;
  int ti = g->id[x];
  g->id[x] = g->id[y];
  g->id[y] = ti;
}
static int len_less(const groups *g, int x, int y, int desc) {
  return desc ? g->l[x].n > g->l[y].n : g->l[x].n < g->l[y].n;
}
static void sort_groups_len(groups *g, int desc) {
  if (g->n > 12) abort(); /* quickSort_func proper: never reached (<= 8 sockets) */
  for (int i = 6; i < g->n; i++)
    if (len_less(g, i, i - 6, desc)) swap_groups(g, i, i - 6);
  for (int i = 1; i < g->n; i++)
    for (int j = i; j > 0 && len_less(g, j, j - 1, desc); j--) swap_groups(g, j, j - 1);
}

/* takeCPUs, cpu_accumulator.go:87-232.  Returns 1 and fills a->result on success. */
static int take_cpus(acc *a, int bind_policy) {
  if (acc_satisfied(a)) return 1; /* :98-100 */
  if (acc_failed(a)) return 0;    /* :101-103 */
  groups g;
  const int full = bind_policy == KOORDHIP_CPUBIND_FULL_PCPUS;
  if (full || a->cpc == 1) {
    if (a->need <= a->cpn) { /* :111-121 */
      for (int fe = 1; fe >= 0; fe--) {
        free_cores(a, 0, 1, fe, &g);
        for (int i = 0; i < g.n; i++)
          if (g.l[i].n >= a->need) {
            acc_take(a, g.l[i].v, a->need);
            return 1;
          }
      }
    }
    if (a->need <= a->cps) { /* :126-134 */
      free_cores(a, 1, 1, 0, &g);
      for (int i = 0; i < g.n; i++)
        if (g.l[i].n >= a->need) {
          acc_take(a, g.l[i].v, a->need);
          return 1;
        }
    }
    free_cores(a, 1, 1, 0, &g); /* :141-155 */
    sort_groups_len(&g, 1);
    groups uns;
    uns.n = 0;
    for (int i = 0; i < g.n; i++) {
      if (!acc_needs(a, g.l[i].n)) {
        uns.l[uns.n] = g.l[i];
        uns.id[uns.n] = g.id[i];
        uns.n++;
      } else {
        acc_take(a, g.l[i].v, g.l[i].n);
        if (acc_satisfied(a)) return 1;
      }
    }
    if (acc_needs(a, a->cpc)) { /* :159-176 */
      sort_groups_len(&uns, 0);
      for (int i = 0; i < uns.n; i++) {
        for (int k = 0; k < uns.l[i].n; k += a->cpc) {
          acc_take(a, uns.l[i].v + k, a->cpc);
          if (acc_satisfied(a)) return 1;
          if (!acc_needs(a, a->cpc)) break;
        }
      }
    }
  }
  if (!full) {
    if (a->need <= a->cpn) { /* :187-199 */
      for (int fe = 1; fe >= 0; fe--) {
        free_cpus_in(a, 0, fe, &g);
        for (int i = 0; i < g.n; i++)
          if (g.l[i].n >= a->need) {
            spread_cpus(a, &g.l[i]);
            acc_take(a, g.l[i].v, a->need);
            return 1;
          }
      }
    }
    if (a->need <= a->cps) { /* :203-214 */
      for (int fe = 1; fe >= 0; fe--) {
        free_cpus_in(a, 1, fe, &g);
        for (int i = 0; i < g.n; i++)
          if (g.l[i].n >= a->need) {
            spread_cpus(a, &g.l[i]);
            acc_take(a, g.l[i].v, a->need);
            return 1;
          }
      }
    }
  }
  for (int fe = 1; fe >= 0; fe--) { /* :218-229 */
    list l;
    free_cpus(a, fe, &l);
    spread_cpus(a, &l);
    for (int i = 0; i < l.n; i++) {
      if (acc_needs(a, 1)) acc_take(a, &l.v[i], 1);
      if (acc_satisfied(a)) return 1;
    }
  }
  return 0;
}

/* ------------------------------------------------------------------------ */

int orc_take_cpus(const koordhip_numa_class *t, const uint64_t *avail, const uint64_t *excl_pcpu,
                  const uint64_t *excl_numa, int need, int bind_policy, int excl_policy, int most_allocated,
                  uint64_t *out) {
  acc a;
  acc_init(&a, t, avail, excl_pcpu, excl_numa, need, excl_policy, most_allocated);
  int ok = take_cpus(&a, bind_policy);
  for (int w = 0; w < KOORDHIP_NUMA_WORDS; w++) out[w] = 0;
  if (!ok) return 0;
  for (int p = 0; p < a.ncpu; p++)
    if (a.result[p]) out[p >> 6] |= 1ull << (p & 63);
  return 1;
}

/* the spread order of freeCPUs(false) on a fresh accumulator (TestCPUSpreadByPCPUs) */
int orc_spread_order(const koordhip_numa_class *t, const uint64_t *avail, int most_allocated, int32_t *cpu_ids) {
  acc a;
  acc_init(&a, t, avail, NULL, NULL, 0, KOORDHIP_CPUEXCL_NONE, most_allocated);
  list l;
  free_cpus(&a, 0, &l);
  spread_cpus(&a, &l);
  for (int i = 0; i < l.n; i++) cpu_ids[i] = cpuid(&a, l.v[i]);
  return l.n;
}

static int popc(const uint64_t *m) {
  int c = 0;
  for (int w = 0; w < KOORDHIP_NUMA_WORDS; w++) c += __builtin_popcountll(m[w]);
  return c;
}

/* getPreferredCPUBindPolicy, plugin.go:546-566 */
static int effective_bind_policy(uint8_t node_flags, int preferred) {
  switch (node_flags & KOORDHIP_NODE_CPUBIND_MASK) {
    case 1: return KOORDHIP_CPUBIND_FULL_PCPUS;       /* FullPCPUsOnly */
    case 2: return KOORDHIP_CPUBIND_SPREAD_BY_PCPUS;  /* SpreadByPCPUs */
    default: return preferred;
  }
}

/* ------------------------------------------------------------------------ */
/* NUMA topology policies                                                    */
/* ------------------------------------------------------------------------ */

static int popc64(uint64_t x) { return __builtin_popcountll(x); }

static int node_policy(const orc_state *st, int32_t i) {
  return st->soa->numa_flags ? (int)KOORDHIP_NODE_NUMA_POLICY(st->soa->numa_flags[i]) : 0;
}

/* bitmask.IsNarrowerThan (pkg/util/bitmask/bitmask.go:142-157): fewer bits,
 * or as many and numerically smaller. */
static int narrower(uint64_t a, uint64_t b) {
  const int ca = popc64(a), cb = popc64(b);
  return ca == cb ? a < b : ca < cb;
}

typedef struct tm_list {
  int n;
  orc_tm_hint h[ORC_TM_MAX_HINTS];
} tm_list;

#define TM_MAXL 16

/* mergeFilteredHints (policy.go:119-151): every permutation of one hint per
 * list (iterateAllProviderTopologyHints :170-208), AND-ed into the default
 * affinity (mergePermutation :52-72); preferred beats non-preferred, then the
 * narrowest wins.  A list with no hint yields no permutation. */
static orc_tm_hint merge_filtered(uint64_t deflt, const tm_list *L, int nl) {
  orc_tm_hint best = {deflt, 0, 0};
  int idx[TM_MAXL] = {0};
  for (int i = 0; i < nl; i++)
    if (L[i].n == 0) return best;
  for (;;) {
    uint64_t m = deflt;
    int pref = 1;
    for (int i = 0; i < nl; i++) {
      const orc_tm_hint *h = &L[i].h[idx[i]];
      m &= h->nil ? deflt : h->mask;
      if (!h->preferred) pref = 0;
    }
    if (popc64(m) != 0) {
      if (pref && !best.preferred) {
        best.mask = m;
        best.preferred = 1;
      } else if (!(!pref && best.preferred) && narrower(m, best.mask)) {
        best.mask = m;
        best.preferred = pref;
      }
    }
    int k = nl - 1;
    while (k >= 0 && ++idx[k] == L[k].n) idx[k--] = 0;
    if (k < 0) break;
  }
  return best;
}

int orc_tm_merge(int policy, uint64_t numa_nodes, const orc_tm_entry *e, int32_t ne, orc_tm_hint *out) {
  static __thread tm_list L[TM_MAXL];
  int nl = 0;
  /* filterProvidersHints (policy.go:93-117) */
  for (int32_t q = 0; q < ne && nl < TM_MAXL; q++, nl++) {
    L[nl].n = 1;
    L[nl].h[0].mask = 0;
    L[nl].h[0].nil = 1;
    switch (e[q].kind) {
      case ORC_TM_PROVIDER_EMPTY:
      case ORC_TM_RES_NIL: L[nl].h[0].preferred = 1; break;
      case ORC_TM_RES_EMPTY: L[nl].h[0].preferred = 0; break;
      default:
        L[nl].n = e[q].n;
        for (int j = 0; j < e[q].n; j++) L[nl].h[j] = e[q].h[j];
    }
  }
  orc_tm_hint best;
  int admit = 1;
  switch (policy) {
    case KOORDHIP_NUMA_TOPO_SINGLE_NUMA_NODE: /* policy_single_numa_node.go:37-78 */
      for (int i = 0; i < nl; i++) {
        int m = 0;
        for (int j = 0; j < L[i].n; j++) {
          const orc_tm_hint h = L[i].h[j];
          if (h.preferred && (h.nil || popc64(h.mask) == 1)) L[i].h[m++] = h;
        }
        L[i].n = m;
      }
      best = merge_filtered(numa_nodes, L, nl);
      if (!best.nil && best.mask == numa_nodes) {
        best.nil = 1;
        best.mask = 0;
      }
      admit = best.preferred;
      break;
    case KOORDHIP_NUMA_TOPO_RESTRICTED: /* policy_restricted.go:34-47 */
      best = merge_filtered(numa_nodes, L, nl);
      admit = best.preferred;
      break;
    case KOORDHIP_NUMA_TOPO_BEST_EFFORT: /* policy_best_effort.go:35-48 */
      best = merge_filtered(numa_nodes, L, nl);
      break;
    default: /* policy_none.go:37-42 */
      best.mask = 0;
      best.nil = 1;
      best.preferred = 0;
  }
  *out = best;
  return admit;
}

static int64_t zone_at(const int64_t *z, int32_t i, int r, int k) {
  return z[((size_t)i * 2 + (size_t)r) * KOORDHIP_NUMA_MAX_NODES + (size_t)k];
}

/* NodeAllocation.getAvailableNUMANodeResources (node_allocation.go:155-177)
 * with getResourceOptions' reusableResources (plugin.go:465-479): zone k's
 * allocated cpu less reus[k] (the nominated reservation's reserved CPUs in the
 * zone x 1000; no amplification on policy nodes), non-negative; then
 * allocatable - allocated, non-negative.  reus = NULL: none. */
static int64_t zone_allocated(const orc_state *st, int32_t i, int r, int k, const int64_t *reus) {
  int64_t u = zone_at(st->numa_zone_used, i, r, k);
  if (r == 0 && reus) u -= reus[k];
  return u > 0 ? u : 0;
}
static int64_t zone_avail(const orc_state *st, int32_t i, int r, int k, const int64_t *reus) {
  const int64_t a = zone_at(st->soa->numa_zone_alloc, i, r, k) - zone_allocated(st, i, r, k, reus);
  return a > 0 ? a : 0;
}

static int zones_of(const orc_state *st, int32_t i) {
  const koordhip_node_soa *s = st->soa;
  if (!s->numa_class || s->numa_class[i] < 0 || !s->numa_zone_alloc) return 0;
  return s->numa_classes[s->numa_class[i]].num_nodes;
}

/* GetPodTopologyHints + generateResourceHints (topology_hint.go:41-62,
 * resource_manager.go:384-428) for the pod's cpu / memory requests (a request
 * of 0 counts as absent: the marshaller drops explicit zero requests), then
 * the node policy's Merge. */
static int node_merge(const orc_state *st, const koordhip_pod *pod, int32_t i, int M, int policy, orc_tm_hint *best) {
  static __thread orc_tm_entry e[2];
  const int64_t req[2] = {pod->req[KOORDHIP_RES_CPU], pod->req[KOORDHIP_RES_MEM]};
  int minsize = M, nh = 0;
  uint64_t hm[ORC_TM_MAX_HINTS];
  /* IterateBitMasks order (bitmask.go:200-222): by size, then lexicographic */
  for (int size = 1; size <= M; size++)
    for (uint64_t m = 1; m < (1ull << M); m++) {
      if (popc64(m) != size) continue;
      int sat = 1;
      for (int r = 0; r < 2; r++) {
        if (req[r] == 0) continue;
        int64_t sum = 0;
        for (int k = 0; k < M; k++)
          if ((m >> k) & 1) sum += zone_avail(st, i, r, k, NULL);
        if (req[r] > sum) sat = 0;
      }
      if (!sat) continue;
      if (size < minsize) minsize = size;
      hm[nh++] = m;
    }
  int ne = 0;
  for (int r = 0; r < 2 && nh > 0; r++) {
    if (req[r] == 0) continue;
    e[ne].kind = ORC_TM_RES_HINTS;
    e[ne].n = nh;
    for (int j = 0; j < nh; j++) {
      e[ne].h[j].mask = hm[j];
      e[ne].h[j].nil = 0;
      e[ne].h[j].preferred = popc64(hm[j]) == minsize;
    }
    ne++;
  }
  if (ne == 0) { /* no hint map entries: the provider has no preference */
    e[0].kind = ORC_TM_PROVIDER_EMPTY;
    ne = 1;
  }
  return orc_tm_merge(policy, (1ull << M) - 1, e, ne, best);
}

/* allocateResourcesByHint (resource_manager.go:166-227): the hinted zones in
 * ascending id take min(available, still requested) of cpu and memory; the
 * availability counts the reusable reservation CPUs (reus, NULL: none). */
static int alloc_by_hint(const orc_state *st, const koordhip_pod *pod, int32_t i, int M, uint64_t mask, int64_t *zones,
                         const int64_t *reus) {
  int64_t rem[2] = {pod->req[KOORDHIP_RES_CPU], pod->req[KOORDHIP_RES_MEM]};
  for (int q = 0; q < 2 * KOORDHIP_NUMA_MAX_NODES; q++) zones[q] = 0;
  for (int k = 0; k < M; k++) {
    if (!((mask >> k) & 1)) continue;
    for (int r = 0; r < 2; r++) {
      const int64_t av = zone_avail(st, i, r, k, reus);
      const int64_t a = av < rem[r] ? av : rem[r];
      zones[r * KOORDHIP_NUMA_MAX_NODES + k] = a;
      rem[r] -= a;
    }
  }
  return rem[0] == 0 && rem[1] == 0; /* :230-241 Insufficient NUMA <resource> */
}

int orc_numa_hint_alloc(const orc_state *st, const koordhip_pod *pod, int32_t i, uint64_t *mask, int32_t *nil,
                        int32_t *admit, int64_t *zones) {
  for (int q = 0; q < 2 * KOORDHIP_NUMA_MAX_NODES; q++) zones[q] = 0;
  *mask = 0;
  *nil = 1;
  *admit = 0;
  const int M = zones_of(st, i);
  const int policy = node_policy(st, i);
  if (M == 0) return 0; /* FilterByNUMANode: missing NUMA resources (topology_hint.go:34-37) */
  orc_tm_hint best;
  *admit = node_merge(st, pod, i, M, policy, &best);
  *mask = best.mask;
  *nil = best.nil;
  if (!*admit) return 0;
  if (best.nil) return 1;
  return alloc_by_hint(st, pod, i, M, best.mask, zones, NULL);
}

/* takePreferredCPUs (cpu_accumulator.go:29-85): the preferred CPUs among the
 * available ones first (at most need of them), then the rest from the
 * available CPUs outside the preferred set; both accumulators see the same
 * allocateInfo (ep / en). */
static int take_preferred(const koordhip_numa_class *t, const uint64_t *avail_in, const uint64_t *pref,
                          const uint64_t *ep, const uint64_t *en, int need, int policy, int excl, int most,
                          uint64_t *out) {
  uint64_t avail[KOORDHIP_NUMA_WORDS], pr[KOORDHIP_NUMA_WORDS], got[KOORDHIP_NUMA_WORDS];
  for (int w = 0; w < KOORDHIP_NUMA_WORDS; w++) {
    out[w] = 0;
    avail[w] = avail_in[w];
    pr[w] = avail[w] & (pref ? pref[w] : 0); /* preferredCPUs = availableCPUs.Intersection(preferredCPUs) :41 */
  }
  if (popc(pr) > 0) {
    const int needed = need > popc(pr) ? popc(pr) : need; /* :43-46 */
    if (!orc_take_cpus(t, pr, ep, en, needed, policy, excl, most, got)) return 0;
    for (int w = 0; w < KOORDHIP_NUMA_WORDS; w++) {
      out[w] = got[w];
      avail[w] &= ~pr[w]; /* availableCPUs.Difference(preferredCPUs) :61 */
    }
    need -= popc(got);
  }
  if (need > 0) { /* :64-82 */
    if (!orc_take_cpus(t, avail, ep, en, need, policy, excl, most, got)) return 0;
    for (int w = 0; w < KOORDHIP_NUMA_WORDS; w++) out[w] |= got[w];
  }
  return 1;
}

/* allocateCPUSet (resource_manager.go:244-326): zones = NULL for a nil hint,
 * else the pod's per-zone allocation from allocateResourcesByHint -- every
 * zone holding a non-zero amount takes floor(cpu / 1000) CPUs from its own
 * available CPUs (:264-295).  pref: the reservation-preferred CPUs (NULL =
 * none): GetAvailableCPUs(preferredCPUs) drops their RefCount 1 -> 0, so they
 * join the available CPUs and leave allocateInfo (node_allocation.go:133-153);
 * both branches take them first through takePreferredCPUs (:277-287 per zone,
 * :298-310 without a hint). */
static int alloc_cpuset(const orc_state *st, const koordhip_pod *pod, int32_t i, const int64_t *zones, uint64_t *out,
                        const uint64_t *pref) {
  const koordhip_node_soa *s = st->soa;
  for (int w = 0; w < KOORDHIP_NUMA_WORDS; w++) out[w] = 0;
  int cls = s->numa_class[i];
  if (cls < 0) return 0; /* GetAvailableCPUs: ErrNotFoundCPUTopology */
  const koordhip_numa_class *t = &s->numa_classes[cls];
  uint64_t avail[KOORDHIP_NUMA_WORDS], ep[KOORDHIP_NUMA_WORDS], en[KOORDHIP_NUMA_WORDS];
  for (int w = 0; w < KOORDHIP_NUMA_WORDS; w++) {
    const uint64_t p = pref ? pref[w] : 0;
    avail[w] = st->numa_free[w][i] | p;
    ep[w] = st->numa_excl_pcpu[w][i] & ~p;
    en[w] = st->numa_excl_numa[w][i] & ~p;
  }
  const int need = pod->numa_cpus;
  const int required = KOORDHIP_NUMA_REQUIRED(pod->numa_policy) != KOORDHIP_CPUBIND_NONE;
  const int policy = effective_bind_policy(s->numa_flags[i], (int)KOORDHIP_NUMA_PREFERRED(pod->numa_policy));
  const int excl = (int)KOORDHIP_NUMA_EXCLUSIVE(pod->numa_policy);
  const int most = (s->numa_flags[i] & KOORDHIP_NODE_NUMA_MOST_ALLOCATED) != 0;
  /* filterAvailableCPUsByRequiredCPUBindPolicy (:430-440) returns a set equal
   * to availableCPUs on both branches: no-op. */
  if (popc(avail) < need) return 0; /* :257-259 */
  if (zones) {
    int got = 0;
    for (int k = 0; k < t->num_nodes && k < KOORDHIP_NUMA_MAX_NODES; k++) {
      if (zones[k] == 0 && zones[KOORDHIP_NUMA_MAX_NODES + k] == 0) continue; /* not in NUMANodeResources */
      uint64_t zav[KOORDHIP_NUMA_WORDS] = {0, 0, 0, 0}, zo[KOORDHIP_NUMA_WORDS];
      for (int p = 0; p < t->num_cpus; p++)
        if (t->node_of[p] == k && bit(avail, p)) zav[p >> 6] |= 1ull << (p & 63);
      int n = popc(zav);
      const int64_t want = zones[k] / 1000;
      if (want < n) n = (int)want;
      if (n > 0) {
        if (!take_preferred(t, zav, pref, ep, en, n, policy, excl, most, zo)) return 0;
        for (int w = 0; w < KOORDHIP_NUMA_WORDS; w++) out[w] |= zo[w];
        got += popc(zo);
      }
    }
    if (got != need) return 0; /* :290-293 */
  } else if (!take_preferred(t, avail, pref, ep, en, need, policy, excl, most, out)) {
    return 0;
  }
  if (required) { /* satisfiedRequiredCPUBindPolicy :442-463 */
    const int cpc = t->num_cpus / t->num_cores;
    int cores = 0, n = popc(out);
    for (int c = 0; c < t->num_cpus / cpc; c++) {
      int any = 0;
      for (int q = 0; q < cpc; q++) any |= bit(out, c * cpc + q);
      cores += any;
    }
    if (policy == KOORDHIP_CPUBIND_FULL_PCPUS && cores * cpc != n) return 0;
    if (policy == KOORDHIP_CPUBIND_SPREAD_BY_PCPUS && cores != n) return 0;
  }
  return 1;
}

/* resourceManager.Allocate for a cpuset pod with an empty hint and no
 * reservation (resource_manager.go:142-164). */
int orc_numa_allocate(const orc_state *st, const koordhip_pod *pod, int32_t i, uint64_t *out) {
  return alloc_cpuset(st, pod, i, NULL, out, NULL);
}


/* reusableResources (plugin.go:469-479): per zone, the reservation-preferred
 * CPUs in it x 1000 (no amplification: policy nodes have none); NULL when pref
 * holds no CPU. */
static const int64_t *reusable_of(const orc_state *st, int32_t i, const uint64_t *pref, int64_t *reus) {
  const koordhip_node_soa *s = st->soa;
  if (!pref || !(pref[0] | pref[1] | pref[2] | pref[3])) return NULL;
  const koordhip_numa_class *t = &s->numa_classes[s->numa_class[i]];
  for (int k = 0; k < KOORDHIP_NUMA_MAX_NODES; k++) reus[k] = 0;
  for (int p = 0; p < t->num_cpus; p++)
    if (bit(pref, p) && t->node_of[p] < KOORDHIP_NUMA_MAX_NODES) reus[t->node_of[p]] += 1000;
  return reus;
}

/* The whole Allocate of Filter's topology-manager admit / Score / Reserve on a
 * node with a topology policy (manager.go:58-79 -> plugin Allocate,
 * topology_hint.go:66-86): the merged hint's zones, then the cpuset inside
 * them.  The hint is Filter's (the store's affinity, computed before PreScore
 * nominates a reservation: no reusable resources); Score and Reserve then
 * allocate with the nominated reservation's reserved CPUs (pref, NULL: none) as
 * reusable zone resources and preferred CPUs (getResourceOptions,
 * plugin.go:455-501). */
static int policy_allocate(const orc_state *st, const koordhip_pod *pod, int32_t i, int64_t *zones, uint64_t *cpus,
                           int *has_zones, const uint64_t *pref, int64_t *reus_out) {
  uint64_t mask;
  int32_t nil, admit;
  int64_t reus[KOORDHIP_NUMA_MAX_NODES];
  for (int w = 0; w < KOORDHIP_NUMA_WORDS; w++) cpus[w] = 0;
  if (reus_out)
    for (int k = 0; k < KOORDHIP_NUMA_MAX_NODES; k++) reus_out[k] = 0;
  if (!orc_numa_hint_alloc(st, pod, i, &mask, &nil, &admit, zones)) return 0;
  *has_zones = !nil;
  const int64_t *ru = reusable_of(st, i, pref, reus);
  if (ru && reus_out)
    for (int k = 0; k < KOORDHIP_NUMA_MAX_NODES; k++) reus_out[k] = ru[k];
  if (!nil && ru && !alloc_by_hint(st, pod, i, zones_of(st, i), mask, zones, ru)) return 0;
  if (pod->flags & KOORDHIP_POD_CPUSET) return alloc_cpuset(st, pod, i, nil ? NULL : zones, cpus, pref);
  return 1;
}

/* The node's CPU amplification ratio (<= 1: none). */
static double amp_ratio(const orc_state *st, int32_t i) {
  return st->soa->numa_amp_cpu ? st->soa->numa_amp_cpu[i] : 1.0;
}

/* extension.Amplify, apis/extension/node_resource_amplification.go:191-196 */
int64_t orc_amplify(int64_t origin, double ratio) {
  if (ratio <= 1.0) return origin;
  return (int64_t)ceil((double)origin * ratio);
}

/* filterAmplifiedCPUs, plugin.go:326-363: the node's allocated cpuset CPUs
 * count amplified in Requested; a cpuset pod's request is amplified too. */
static int amp_filter_ok(const orc_state *st, const koordhip_pod *pod, int32_t i) {
  const int64_t cpu = pod->req[KOORDHIP_RES_CPU];
  const double ratio = amp_ratio(st, i);
  if (cpu == 0 || ratio <= 1.0) return 1;
  const int cpuset = (pod->flags & KOORDHIP_POD_CPUSET) && !(pod->flags & KOORDHIP_POD_NUMA_SKIP);
  const int64_t req = cpuset ? orc_amplify(cpu, ratio) : cpu;
  const koordhip_node_soa *s = st->soa;
  const int has_topo = s->numa_class && s->numa_class[i] >= 0;
  const int64_t allocm = has_topo ? (int64_t)st->numa_alloc_cnt[i] * 1000 : 0; /* GetAvailableCPUs */
  int64_t requested = st->requested[KOORDHIP_RES_CPU][i];
  if (requested >= allocm && allocm > 0) requested = requested - allocm + orc_amplify(allocm, ratio);
  return !(req > s->alloc[KOORDHIP_RES_CPU][i] - requested);
}

/* Filter, plugin.go:266-324.  A CPU amplification ratio > 1 is supported on
 * nodes without a NUMA topology policy (the host rejects the combination). */
int orc_numa_filter(const koordhip_config *cfg, const orc_state *st, const koordhip_pod *pod, int32_t i) {
  (void)cfg;
  const koordhip_node_soa *s = st->soa;
  const int tp = node_policy(st, i);
  const int cpuset = (pod->flags & KOORDHIP_POD_CPUSET) != 0;
  if (pod->flags & KOORDHIP_POD_NUMA_ERROR) return 0;   /* PreFilter error */
  if (!amp_filter_ok(st, pod, i)) return 0;           /* :272-274 */
  if ((pod->flags & KOORDHIP_POD_NUMA_SKIP) || (!cpuset && tp == KOORDHIP_NUMA_TOPO_NONE))
    return 1;                                          /* skipTheNode, util.go:59-61 */
  if (cpuset) {
    if (!s->numa_class || s->numa_class[i] < 0) return 0; /* :285-294 */
    const koordhip_numa_class *t = &s->numa_classes[s->numa_class[i]];
    const int req = (int)KOORDHIP_NUMA_REQUIRED(pod->numa_policy);
    const int pref = (int)KOORDHIP_NUMA_PREFERRED(pod->numa_policy);
    const int node_full_only = (s->numa_flags[i] & KOORDHIP_NODE_CPUBIND_MASK) == 1;
    if (node_full_only || req == KOORDHIP_CPUBIND_FULL_PCPUS) { /* :295-305 */
      const int cpc = t->num_cpus / t->num_cores;
      if (pod->numa_cpus % cpc != 0) return 0;
      if (node_full_only && (req != KOORDHIP_CPUBIND_FULL_PCPUS || pref != KOORDHIP_CPUBIND_FULL_PCPUS)) return 0;
    }
    if (req != KOORDHIP_CPUBIND_NONE && tp == KOORDHIP_NUMA_TOPO_NONE) { /* :307-316 */
      uint64_t out[KOORDHIP_NUMA_WORDS];
      if (!orc_numa_allocate(st, pod, i, out)) return 0;
    }
  }
  if (tp != KOORDHIP_NUMA_TOPO_NONE) { /* FilterByNUMANode, :319-321 */
    int64_t zones[2 * KOORDHIP_NUMA_MAX_NODES];
    uint64_t cpus[KOORDHIP_NUMA_WORDS];
    int hz;
    return policy_allocate(st, pod, i, zones, cpus, &hz, NULL, NULL);
  }
  return 1;
}

/* mostRequestedScore, nodenumaresource/most_allocated.go:51-62. */
static int64_t most_requested(int64_t requested, int64_t capacity) {
  if (capacity == 0) return 0;
  if (requested > capacity) requested = capacity;
  return (requested * 100) / capacity;
}

/* leastResourceScorer / mostResourceScorer over {cpu, memory}
 * (nodenumaresource/scoring.go:35-53,191-230, least_allocated.go:30-58,
 * most_allocated.go:30-44): resources with allocatable 0 are left out. */
static int64_t numa_least_allocated(const koordhip_config *cfg, int64_t req_cpu, int64_t alloc_cpu, int64_t req_mem,
                                    int64_t alloc_mem) {
  int64_t (*rs)(int64_t, int64_t) = cfg->numa_most_allocated ? most_requested : orc_least_requested;
  int64_t num = 0, wsum = 0;
  if (cfg->numa_weight_cpu && alloc_cpu != 0) {
    num += rs(req_cpu, alloc_cpu) * cfg->numa_weight_cpu;
    wsum += cfg->numa_weight_cpu;
  }
  if (cfg->numa_weight_mem && alloc_mem != 0) {
    num += rs(req_mem, alloc_mem) * cfg->numa_weight_mem;
    wsum += cfg->numa_weight_mem;
  }
  return wsum ? num / wsum : 0;
}

/* resourceManager.Allocate with a given hint (resource_manager.go:142-164, the
 * entry resource_manager_test.go drives): mask = NUMANodeAffinity (0 = no
 * hint), zones = allocateResourcesByHint's amounts, cpus = allocateCPUSet's
 * (cpuset pods).  1 = ok. */
int orc_numa_allocate_hint(const orc_state *st, const koordhip_pod *pod, int32_t i, uint64_t mask, int64_t *zones,
                           uint64_t *cpus) {
  for (int q = 0; q < 2 * KOORDHIP_NUMA_MAX_NODES; q++) zones[q] = 0;
  for (int w = 0; w < KOORDHIP_NUMA_WORDS; w++) cpus[w] = 0;
  if (mask) {
    const int M = zones_of(st, i);
    if (M == 0 || !alloc_by_hint(st, pod, i, M, mask, zones, NULL)) return 0; /* :167-169, :209-219 */
  }
  if (!(pod->flags & KOORDHIP_POD_CPUSET)) return 1;
  return alloc_cpuset(st, pod, i, mask ? zones : NULL, cpus, NULL);
}

/* Score, scoring.go:55-120,122-168. */
int64_t orc_numa_score(const koordhip_config *cfg, const orc_state *st, const koordhip_pod *pod, int32_t i) {
  const koordhip_node_soa *s = st->soa;
  if (pod->flags & (KOORDHIP_POD_NUMA_SKIP | KOORDHIP_POD_NUMA_ERROR)) return 0; /* :70-72 */
  const int has_topo = s->numa_class && s->numa_class[i] >= 0;
  const int cpuset = (pod->flags & KOORDHIP_POD_CPUSET) != 0;
  const int tp = node_policy(st, i);
  int64_t acpu = s->alloc[KOORDHIP_RES_CPU][i], amem = s->alloc[KOORDHIP_RES_MEM][i];
  int64_t rcpu = st->requested[KOORDHIP_RES_CPU][i], rmem = st->requested[KOORDHIP_RES_MEM][i];
  /* no topology: getResourceOptions fails (:82-85, :97-100) */
  if (!has_topo) return 0;
  const double ratio = amp_ratio(st, i);
  if (!cpuset && tp == KOORDHIP_NUMA_TOPO_NONE) { /* scoreWithAmplifiedCPUs :95-120 */
    if (pod->req[KOORDHIP_RES_CPU] != 0 && ratio > 1.0) {
      const int64_t allocm = (int64_t)st->numa_alloc_cnt[i] * 1000;
      rcpu = rcpu - allocm + orc_amplify(allocm, ratio);
    }
    return numa_least_allocated(cfg, rcpu + pod->req[KOORDHIP_RES_CPU], acpu, rmem + pod->req[KOORDHIP_RES_MEM], amem);
  }
  int64_t zones[2 * KOORDHIP_NUMA_MAX_NODES];
  uint64_t cpus[KOORDHIP_NUMA_WORDS], pref[KOORDHIP_NUMA_WORDS];
  int hz = 0;
  int64_t reus[KOORDHIP_NUMA_MAX_NODES];
  orc_resv_pref(cfg, st, pod, i, pref); /* getResourceOptions' preferredCPUs (plugin.go:465-495) */
  if (tp != KOORDHIP_NUMA_TOPO_NONE) {
    if (!policy_allocate(st, pod, i, zones, cpus, &hz, pref, reus)) return 0; /* :86-89 */
  } else if (!alloc_cpuset(st, pod, i, NULL, cpus, pref)) {
    return 0;
  }
  if (hz) { /* calculateAllocatableAndRequested over the pod's zones :134-152 (allocated less the reusable CPUs) */
    acpu = amem = rcpu = rmem = 0;
    for (int k = 0; k < KOORDHIP_NUMA_MAX_NODES; k++) {
      if (zones[k] == 0 && zones[KOORDHIP_NUMA_MAX_NODES + k] == 0) continue;
      acpu += zone_at(s->numa_zone_alloc, i, 0, k);
      amem += zone_at(s->numa_zone_alloc, i, 1, k);
      rcpu += zone_allocated(st, i, 0, k, reus);
      rmem += zone_allocated(st, i, 1, k, NULL);
    }
  }
  /* requested cpu := allocated cpuset size, amplified (:161-166); the cpuset
   * pod's request is amplified too (getResourceOptions, plugin.go:481-485) */
  int64_t qcpu = pod->req[KOORDHIP_RES_CPU];
  if (cpuset) {
    /* getAvailableCPUs(preferredCPUs - the pod's CPUs): the preferred CPUs the
     * pod leaves drop out of the allocated set (RefCount 1 -> 0) */
    int64_t left = 0;
    for (int w = 0; w < KOORDHIP_NUMA_WORDS; w++) left += __builtin_popcountll(pref[w] & ~cpus[w]);
    rcpu = orc_amplify(((int64_t)st->numa_alloc_cnt[i] - left) * 1000, ratio);
    qcpu = orc_amplify(qcpu, ratio);
  }
  return numa_least_allocated(cfg, rcpu + qcpu, acpu, rmem + pod->req[KOORDHIP_RES_MEM], amem);
}

int orc_numa_reserve_active(const orc_state *st, const koordhip_pod *pod, int32_t i) {
  if (pod->flags & KOORDHIP_POD_NUMA_SKIP) return 0;
  return (pod->flags & KOORDHIP_POD_CPUSET) || node_policy(st, i) != KOORDHIP_NUMA_TOPO_NONE;
}

/* Reserve (plugin.go:365-405) + resourceManager.Update (resource_manager.go:328-339,
 * node_allocation.go:76-103): the cpuset and the zone amounts; returns 0 when
 * Allocate fails. */
int orc_numa_reserve(orc_state *st, const koordhip_pod *pod, int32_t i, uint64_t *cpus_out, const uint64_t *pref) {
  uint64_t out[KOORDHIP_NUMA_WORDS] = {0, 0, 0, 0};
  int64_t zones[2 * KOORDHIP_NUMA_MAX_NODES] = {0};
  int hz = 0;
  if (node_policy(st, i) != KOORDHIP_NUMA_TOPO_NONE) {
    if (!policy_allocate(st, pod, i, zones, out, &hz, pref, NULL)) return 0;
  } else if (!alloc_cpuset(st, pod, i, NULL, out, pref)) {
    return 0;
  }
  /* addPodAllocation (node_allocation.go:76-103): every CPU's ExclusivePolicy
   * becomes the pod's, RefCount + 1 -- a preferred CPU was allocated already
   * (the reservation's), so the allocated count grows by the others only */
  const int ex = (int)KOORDHIP_NUMA_EXCLUSIVE(pod->numa_policy);
  int grow = 0;
  for (int w = 0; w < KOORDHIP_NUMA_WORDS; w++) {
    const uint64_t was_alloc = ~st->numa_free[w][i] & (pref ? pref[w] : 0);
    grow += __builtin_popcountll(out[w] & ~was_alloc);
    st->numa_free[w][i] &= ~out[w];
    st->numa_excl_pcpu[w][i] = (st->numa_excl_pcpu[w][i] & ~out[w]) | (ex == KOORDHIP_CPUEXCL_PCPU ? out[w] : 0);
    st->numa_excl_numa[w][i] = (st->numa_excl_numa[w][i] & ~out[w]) | (ex == KOORDHIP_CPUEXCL_NUMA ? out[w] : 0);
    if (cpus_out) cpus_out[w] = out[w];
  }
  st->numa_alloc_cnt[i] += grow;
  if (hz)
    for (int q = 0; q < 2 * KOORDHIP_NUMA_MAX_NODES; q++) st->numa_zone_used[(size_t)i * 2 * KOORDHIP_NUMA_MAX_NODES + q] += zones[q];
  return 1;
}

/* Unreserve -> resourceManager.Release (node_allocation.go:105-131). */
void orc_numa_release(orc_state *st, int32_t i, const uint64_t *cpus) {
  for (int w = 0; w < KOORDHIP_NUMA_WORDS; w++) {
    st->numa_free[w][i] |= cpus[w];
    st->numa_excl_pcpu[w][i] &= ~cpus[w];
    st->numa_excl_numa[w][i] &= ~cpus[w];
  }
  st->numa_alloc_cnt[i] -= popc(cpus);
}
