/*
 * koord_oracle.c -- TEST INFRASTRUCTURE (see koord_oracle.h).  A plain-C
 * restatement of the reference algorithm, one function per reference rule,
 * each citing the koordinator file:line it follows.  It is the checker for the
 * HIP path and the timed `cpu_baseline` of bench.py; it is never linked into
 * the product.
 *
 * Build: see oracle/Makefile (gcc -O2 -ffp-contract=off, no fast-math, so the
 * f64 usage arithmetic matches Go's IEEE float64 exactly).
 */
#define _GNU_SOURCE
#include "koord_oracle.h"

#include <math.h>
#include <pthread.h>
#include <sched.h>
#include <stdatomic.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------ */
/* Scalar rules                                                              */
/* ------------------------------------------------------------------------ */

/* load_aware.go:214 and :248:
 *   usage := int64(math.Round(float64(used.MilliValue()) / float64(total.MilliValue()) * 100))
 * math.Round is half-away-from-zero == C round(). */
int64_t orc_usage_percent(int64_t used_milli, int64_t total_milli) {
  double u = (double)used_milli / (double)total_milli;
  u = u * 100.0;
  return (int64_t)round(u);
}

/* load_aware.go:388-397 leastRequestedScore; identical rule in (upstream)
 * noderesources/least_allocated.go and nodenumaresource/least_allocated.go:49-58. */
int64_t orc_least_requested(int64_t requested, int64_t capacity) {
  if (capacity == 0) return 0;
  if (requested > capacity) return 0;
  return ((capacity - requested) * 100) / capacity; /* framework.MaxNodeScore = 100 */
}

/* ------------------------------------------------------------------------ */
/* LoadAware Filter (static per snapshot)                                    */
/* ------------------------------------------------------------------------ */

/* filterNodeUsage, load_aware.go:173-224: per resource, skip threshold 0
 * (:186-188), skip zero total (:194-197), skip absent usage source (:209-211),
 * fail when usage >= threshold (:215). */
static int la_usage_ok(const koordhip_node_soa *s, int32_t i) {
  if (!(s->la_flags[i] & KOORDHIP_LA_FILTER_USAGE)) return 1; /* :174-176 / :209-211 */
  for (int r = 0; r < 2; r++) {
    int64_t thr = s->laf_thr[r][i];
    if (thr == 0) continue;
    int64_t total = s->laf_total_m[r][i];
    if (total == 0) continue;
    if (orc_usage_percent(s->laf_used_m[r][i], total) >= thr) return 0;
  }
  return 1;
}

/* filterProdUsage, load_aware.go:226-254. */
static int la_prod_ok(const koordhip_node_soa *s, int32_t i) {
  if (!(s->la_flags[i] & KOORDHIP_LA_HAS_PODS_METRIC)) return 1; /* :227-229 */
  for (int r = 0; r < 2; r++) {
    int64_t thr = s->laf_prod_thr[r][i];
    if (thr == 0) continue;
    int64_t total = s->laf_total_m[r][i];
    if (total == 0) continue;
    if (orc_usage_percent(s->laf_prod_used_m[r][i], total) >= thr) return 0;
  }
  return 1;
}

/* Filter, load_aware.go:123-171, resolved per node for {non-prod, prod} pods
 * (the DaemonSet bypass :129-131 is per pod, applied in orc_la_filter). */
void orc_la_flags(const koordhip_node_soa *s, int32_t n, uint8_t *out) {
  for (int32_t i = 0; i < n; i++) {
    uint8_t f = s->la_flags[i];
    uint8_t o = 0;
    if (!(f & KOORDHIP_LA_HAS_METRIC) || (f & KOORDHIP_LA_FILTER_SKIP)) {
      o |= ORC_LA_OK_NONPROD | ORC_LA_OK_PROD; /* :138-140, :144-147 */
    } else {
      int np = la_usage_ok(s, i);              /* :155-168 */
      int p = (f & KOORDHIP_LA_PROD_MODE) ? la_prod_ok(s, i) : np; /* :150-154 */
      if (np) o |= ORC_LA_OK_NONPROD;
      if (p) o |= ORC_LA_OK_PROD;
    }
    /* Score returns 0 for a missing or expired NodeMetric, load_aware.go:278-289 */
    if (!(f & KOORDHIP_LA_HAS_METRIC) || (f & KOORDHIP_LA_SCORE_EXPIRED)) o |= ORC_LA_SCORE_ZERO;
    out[i] = o;
  }
}

/* ------------------------------------------------------------------------ */
/* State                                                                     */
/* ------------------------------------------------------------------------ */

static int64_t *dup64(const int64_t *src, int32_t n) {
  int64_t *d = (int64_t *)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
  if (!d) return NULL;
  if (src) memcpy(d, src, sizeof(int64_t) * (size_t)n);
  else memset(d, 0, sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
  return d;
}

int orc_state_init(orc_state *st, const koordhip_node_soa *soa, int32_t n) {
  memset(st, 0, sizeof(*st));
  st->n = n;
  st->soa = soa;
  st->flags = (uint8_t *)malloc((size_t)(n > 0 ? n : 1));
  for (int r = 0; r < KOORDHIP_NRES; r++) st->requested[r] = dup64(soa->requested[r], n);
  st->nz_cpu_m = dup64(soa->nz_cpu_m, n);
  st->nz_mem = dup64(soa->nz_mem, n);
  st->npods = (int32_t *)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
  if (soa->npods) memcpy(st->npods, soa->npods, sizeof(int32_t) * (size_t)n);
  else memset(st->npods, 0, sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
  st->la_used_cpu_m = dup64(soa->la_used_cpu_m, n);
  st->la_used_mem = dup64(soa->la_used_mem, n);
  st->la_used_prod_cpu_m = dup64(soa->la_used_prod_cpu_m, n);
  st->la_used_prod_mem = dup64(soa->la_used_prod_mem, n);
  for (int w = 0; w < KOORDHIP_NUMA_WORDS; w++) {
    st->numa_free[w] = (uint64_t *)dup64(soa->numa_class ? (const int64_t *)soa->numa_free[w] : NULL, n);
    st->numa_excl_pcpu[w] = (uint64_t *)dup64(soa->numa_class ? (const int64_t *)soa->numa_excl_pcpu[w] : NULL, n);
    st->numa_excl_numa[w] = (uint64_t *)dup64(soa->numa_class ? (const int64_t *)soa->numa_excl_numa[w] : NULL, n);
  }
  st->numa_alloc_cnt = (int32_t *)calloc((size_t)(n > 0 ? n : 1), sizeof(int32_t));
  if (soa->numa_class && soa->numa_alloc_cnt) memcpy(st->numa_alloc_cnt, soa->numa_alloc_cnt, sizeof(int32_t) * (size_t)n);
  const size_t zn = (size_t)(n > 0 ? n : 1) * 2 * KOORDHIP_NUMA_MAX_NODES;
  st->numa_zone_used = (int64_t *)calloc(zn, sizeof(int64_t));
  if (soa->numa_zone_used && st->numa_zone_used)
    memcpy(st->numa_zone_used, soa->numa_zone_used, sizeof(int64_t) * (size_t)n * 2 * KOORDHIP_NUMA_MAX_NODES);
  /* reservation state: one value per slot of every node ([slots][n]) */
  const int32_t rn = n * (soa->resv_slots > 1 ? soa->resv_slots : 1);
  for (int r = 0; r < 2; r++)
    st->resv_allocated[r] = dup64(soa->resv_flags && soa->resv_allocated[r] ? soa->resv_allocated[r] : NULL, rn);
  st->resv_assigned = (int32_t *)calloc((size_t)(rn > 0 ? rn : 1), sizeof(int32_t));
  if (soa->resv_flags && soa->resv_assigned && st->resv_assigned)
    memcpy(st->resv_assigned, soa->resv_assigned, sizeof(int32_t) * (size_t)rn);
  if (soa->resv_flags && soa->resv_cpus[0])
    for (int w = 0; w < KOORDHIP_NUMA_WORDS; w++) st->resv_cpus[w] = (uint64_t *)dup64((const int64_t *)soa->resv_cpus[w], rn);
  /* DeviceShare deviceUsed and the extended scalars' Requested (dev_oracle.c) */
  const int32_t dn = soa->dev_slots > 0 ? n * KOORDHIP_DEV_TYPES * soa->dev_slots * KOORDHIP_DEV_RES : 0;
  st->dev_used = dup64(dn ? soa->dev_used : NULL, dn);
  st->xrequested = dup64(soa->xrequested, n * KOORDHIP_NXRES);
  if (soa->pts_keys > 0 && soa->pts_cons > 0) {
    const size_t pn = (size_t)soa->pts_cons * (size_t)(n > 0 ? n : 1);
    st->pts_cnt = (int32_t *)calloc(pn, sizeof(int32_t));
    if (!st->pts_cnt) return -1;
    if (soa->pts_cnt) memcpy(st->pts_cnt, soa->pts_cnt, sizeof(int32_t) * (size_t)soa->pts_cons * (size_t)n);
  }
  if (soa->ipa_ents > 0) {
    const size_t in = (size_t)soa->ipa_ents * (size_t)(n > 0 ? n : 1);
    st->ipa_cnt = (int32_t *)calloc(in, sizeof(int32_t));
    if (!st->ipa_cnt) return -1;
    if (soa->ipa_cnt) memcpy(st->ipa_cnt, soa->ipa_cnt, sizeof(int32_t) * (size_t)soa->ipa_ents * (size_t)n);
  }
  if (soa->resv_dev && soa->resv_dev_slot && soa->dev_slots > 0) {
    st->resv_dev = dup64(soa->resv_dev, n * 2 * KOORDHIP_DEV_TYPES * soa->dev_slots * KOORDHIP_DEV_RES);
    if (!st->resv_dev) return -1;
  }
  if (soa->resv_xalloc && soa->resv_dev_slot) {
    st->resv_xallocated = dup64(soa->resv_xallocated, n * KOORDHIP_NXRES);
    if (!st->resv_xallocated) return -1;
  }
  if (!st->flags || !st->npods || !st->numa_alloc_cnt || !st->numa_zone_used || !st->resv_assigned || !st->dev_used ||
      !st->xrequested)
    return -1;
  orc_la_flags(soa, n, st->flags);
  return 0;
}

void orc_state_free(orc_state *st) {
  free(st->flags);
  for (int r = 0; r < KOORDHIP_NRES; r++) free(st->requested[r]);
  free(st->nz_cpu_m);
  free(st->nz_mem);
  free(st->npods);
  free(st->la_used_cpu_m);
  free(st->la_used_mem);
  free(st->la_used_prod_cpu_m);
  free(st->la_used_prod_mem);
  for (int w = 0; w < KOORDHIP_NUMA_WORDS; w++) {
    free(st->numa_free[w]);
    free(st->numa_excl_pcpu[w]);
    free(st->numa_excl_numa[w]);
  }
  free(st->numa_alloc_cnt);
  free(st->numa_zone_used);
  free(st->resv_allocated[0]);
  free(st->resv_allocated[1]);
  free(st->resv_assigned);
  for (int w = 0; w < KOORDHIP_NUMA_WORDS; w++) free(st->resv_cpus[w]);
  free(st->dev_used);
  free(st->xrequested);
  free(st->pts_cnt);
  free(st->ipa_cnt);
  free(st->resv_dev);
  free(st->resv_xallocated);
  memset(st, 0, sizeof(*st));
}

/* ------------------------------------------------------------------------ */
/* Per-(pod,node) plugin rules                                               */
/* ------------------------------------------------------------------------ */

/* UPSTREAM-ASSUMED: (upstream) noderesources/fit.go fitsRequest (k8s v1.24.15).
 * In-reference mirror: pkg/scheduler/plugins/reservation/plugin.go:445-494
 * (fitsNode with rInfo=nil).  1 = fits. */
int orc_fit_filter(const koordhip_config *cfg, const orc_state *st, const koordhip_pod *pod, int32_t i) {
  (void)cfg;
  const koordhip_node_soa *s = st->soa;
  if ((int64_t)st->npods[i] + 1 > (int64_t)s->alloc_pods[i]) return 0; /* Too many pods */
  if (!(pod->flags & KOORDHIP_POD_HAS_REQ)) return 1;                   /* all-zero request */
  for (int r = KOORDHIP_RES_CPU; r <= KOORDHIP_RES_EPH; r++)            /* cpu, memory, ephemeral-storage */
    if (pod->req[r] > s->alloc[r][i] - st->requested[r][i]) return 0;
  if ((pod->flags & KOORDHIP_POD_REQ_BCPU) &&
      pod->req[KOORDHIP_RES_BCPU] > s->alloc[KOORDHIP_RES_BCPU][i] - st->requested[KOORDHIP_RES_BCPU][i])
    return 0;
  if ((pod->flags & KOORDHIP_POD_REQ_BMEM) &&
      pod->req[KOORDHIP_RES_BMEM] > s->alloc[KOORDHIP_RES_BMEM][i] - st->requested[KOORDHIP_RES_BMEM][i])
    return 0;
  return 1;
}

/* UPSTREAM-ASSUMED: (upstream) noderesources/resource_allocation.go score +
 * calculateResourceAllocatableRequest + least_allocated.go leastResourceScorer.
 * Koord copy of the same rules: nodenumaresource/scoring.go:191-246 (skip a
 * scalar the pod does not request :211-215, skip alloc == 0) and
 * least_allocated.go:30-58.  cpu/memory use NonZeroRequested + the pod's
 * non-zero request; other resources use Requested + the pod request. */
int64_t orc_fit_score(const koordhip_config *cfg, const orc_state *st, const koordhip_pod *pod, int32_t i) {
  const koordhip_node_soa *s = st->soa;
  int64_t num = 0, wsum = 0;
  for (int r = 0; r < KOORDHIP_NRES; r++) {
    int64_t w = cfg->fit_weight[r];
    if (w == 0) continue; /* not in scoringStrategy.resources */
    int64_t podreq, nodereq;
    if (r == KOORDHIP_RES_CPU) {
      podreq = pod->nz_cpu_m;
      nodereq = st->nz_cpu_m[i];
    } else if (r == KOORDHIP_RES_MEM) {
      podreq = pod->nz_mem;
      nodereq = st->nz_mem[i];
    } else {
      podreq = pod->req[r];
      nodereq = st->requested[r][i];
      if (r != KOORDHIP_RES_EPH && podreq == 0) continue; /* scalar not requested -> (0,0) */
    }
    int64_t alloc = s->alloc[r][i];
    if (alloc == 0) continue; /* "Only fill the extended resource entry when it's non-zero" */
    num += orc_least_requested(nodereq + podreq, alloc) * w;
    wsum += w;
  }
  if (wsum == 0) return 0;
  return num / wsum;
}

/* load_aware.go:123-171 (static part resolved by orc_la_flags); 1 = passes. */
int orc_la_filter(const koordhip_config *cfg, const orc_state *st, const koordhip_pod *pod, int32_t i) {
  (void)cfg;
  if (pod->flags & KOORDHIP_POD_DAEMONSET) return 1; /* :129-131 */
  uint8_t bit = (pod->flags & KOORDHIP_POD_PROD) ? ORC_LA_OK_PROD : ORC_LA_OK_NONPROD;
  return (st->flags[i] & bit) ? 1 : 0;
}

/* load_aware.go:269-335 with loadAwareSchedulingScorer :378-386.  The
 * per-node usage base (nodeUsage minus estimated pods' actual usage when
 * larger :316-324, plus assigned-pod estimates :298-301) is marshalled into
 * la_used; pods committed during the stream add EstimatePod (L10). */
int64_t orc_la_score(const koordhip_config *cfg, const orc_state *st, const koordhip_pod *pod, int32_t i) {
  const koordhip_node_soa *s = st->soa;
  if (st->flags[i] & ORC_LA_SCORE_ZERO) return 0; /* :278-289 */
  int prod = (pod->flags & KOORDHIP_POD_PROD) && cfg->la_score_according_prod_usage; /* :291 */
  int64_t used_cpu = pod->est_cpu + (prod ? st->la_used_prod_cpu_m[i] : st->la_used_cpu_m[i]);
  int64_t used_mem = pod->est_mem + (prod ? st->la_used_prod_mem[i] : st->la_used_mem[i]);
  int64_t num = orc_least_requested(used_cpu, s->la_alloc_cpu_m[i]) * cfg->la_weight_cpu +
                orc_least_requested(used_mem, s->la_alloc_mem[i]) * cfg->la_weight_mem;
  int64_t wsum = cfg->la_weight_cpu + cfg->la_weight_mem; /* every weight counts, :380-384 */
  return num / wsum;
}

/* UPSTREAM-ASSUMED (k8s v1.24.15, un-vendored; parity unpinned): the static
 * node filters NodeUnschedulable (node_unschedulable.go: spec.unschedulable
 * without a toleration of node.kubernetes.io/unschedulable:NoSchedule),
 * NodeAffinity (node_affinity.go: nodeSelector + requiredDuringScheduling
 * node selector terms) and TaintToleration (taint_toleration.go: every
 * NoSchedule / NoExecute taint tolerated) depend only on the node's labels /
 * taints and the pod's spec: the host marshaller resolves them per (pod
 * static class, node) into static_allow (koordinator_amd/k8s.py
 * static_allow); this is the per-(pod, node) lookup. */
int orc_static_filter(const orc_state *st, const koordhip_pod *pod, int32_t i) {
  const uint32_t *sa = st->soa->static_allow;
  return !sa || ((sa[i] >> pod->static_class) & 1u);
}

/* UPSTREAM-ASSUMED (k8s v1.24.15 noderesources/balanced_allocation.go,
 * resource_allocation.go; un-vendored, parity unpinned):
 * NodeResourcesBalancedAllocation with its default resources cpu and memory
 * (weight 1) and useRequested = true: requested = NodeInfo.Requested + the
 * pod's request; a resource with Allocatable 0 is left out; fraction =
 * float64(requested) / float64(allocatable), capped at 1; two fractions:
 * std = |f0 - f1| / 2, fewer: 0; score = int64((1 - std) * MaxNodeScore). */
int64_t orc_bal_score(const koordhip_config *cfg, const orc_state *st, const koordhip_pod *pod, int32_t i) {
  (void)cfg;
  const koordhip_node_soa *s = st->soa;
  double f[2];
  int nf = 0;
  for (int r = KOORDHIP_RES_CPU; r <= KOORDHIP_RES_MEM; r++) {
    const int64_t alloc = s->alloc[r][i];
    if (alloc == 0) continue;
    double x = (double)(st->requested[r][i] + pod->req[r]) / (double)alloc;
    if (x > 1) x = 1;
    f[nf++] = x;
  }
  double sd = 0.0;
  if (nf == 2) sd = fabs((f[0] - f[1]) / 2);
  return (int64_t)((1 - sd) * 100.0);
}

uint32_t orc_score_plugin_bit(int p) {
  static const uint32_t bits[KOORDHIP_NPLUGINS] = {KOORDHIP_PLUGIN_FIT, KOORDHIP_PLUGIN_LOADAWARE,
                                                   KOORDHIP_PLUGIN_NUMA, KOORDHIP_PLUGIN_BALANCED};
  return p >= 0 && p < KOORDHIP_NPLUGINS ? bits[p] : 0u;
}

/* ------------------------------------------------------------------------ */
/* Combined evaluation                                                       */
/* ------------------------------------------------------------------------ */

/* The Reservation plugin's Filter: a reserve pod's own checks, else
 * filterWithReservations (a node without reservation columns fails only a
 * required reservation affinity). */
static int resv_pass(const orc_state *st, const koordhip_pod *pod, const koordhip_pod_ext *x, int32_t i) {
  if (pod->flags & KOORDHIP_POD_RESERVE) return orc_resv_reserve_pod_ok(st, pod, x, i);
  /* a reservation-operating-mode pod: the Aligned policy check first (plugin.go:332-357) */
  if ((pod->flags & KOORDHIP_POD_RESV_OPERATING) && !orc_resv_reserve_pod_ok(st, pod, NULL, i)) return 0;
  return st->soa->resv_flags ? orc_resv_filter(st, pod, i) : !(pod->flags & KOORDHIP_POD_RESV_AFFINITY);
}

static int orc_feasible(const koordhip_config *cfg, const orc_state *st, const koordhip_pod *pod,
                        const koordhip_pod_ext *x, const orc_pts *ps, const orc_ipa *ia, int32_t i) {
  if ((cfg->filter_plugins & KOORDHIP_PLUGIN_NODE_STATIC) && !orc_static_filter(st, pod, i)) return 0;
  if ((cfg->filter_plugins & KOORDHIP_PLUGIN_PTS) && !orc_pts_filter(st, x, ps, i)) return 0;
  if ((cfg->filter_plugins & KOORDHIP_PLUGIN_IPA) && !orc_ipa_filter(st, x, ia, i)) return 0;
  if ((cfg->filter_plugins & KOORDHIP_PLUGIN_FIT) && !orc_fit_filter(cfg, st, pod, i)) return 0;
  if ((cfg->filter_plugins & KOORDHIP_PLUGIN_FIT) && !orc_xfit_filter(st, x, i)) return 0;
  if ((cfg->filter_plugins & KOORDHIP_PLUGIN_DEVICESHARE) && !orc_dev_filter(st, pod, x, i)) return 0;
  if ((cfg->filter_plugins & KOORDHIP_PLUGIN_LOADAWARE) && !orc_la_filter(cfg, st, pod, i)) return 0;
  if ((cfg->filter_plugins & KOORDHIP_PLUGIN_NUMA) && !orc_numa_filter(cfg, st, pod, i)) return 0;
  if ((cfg->filter_plugins & KOORDHIP_PLUGIN_RESERVATION) && !resv_pass(st, pod, x, i)) return 0;
  return 1;
}

static int64_t orc_total(const koordhip_config *cfg, const orc_state *st, const koordhip_pod *pod, int32_t i) {
  int64_t t = 0;
  if (cfg->score_plugins & KOORDHIP_PLUGIN_FIT) t += cfg->plugin_weight[0] * orc_fit_score(cfg, st, pod, i);
  if (cfg->score_plugins & KOORDHIP_PLUGIN_LOADAWARE) t += cfg->plugin_weight[1] * orc_la_score(cfg, st, pod, i);
  if (cfg->score_plugins & KOORDHIP_PLUGIN_NUMA) t += cfg->plugin_weight[2] * orc_numa_score(cfg, st, pod, i);
  if (cfg->score_plugins & KOORDHIP_PLUGIN_BALANCED) t += cfg->plugin_weight[3] * orc_bal_score(cfg, st, pod, i);
  return t;
}

int64_t orc_bmax(const koordhip_config *cfg) {
  static const uint32_t ext[KOORDHIP_NEXT_PLUGINS] = {KOORDHIP_PLUGIN_DEVICESHARE, KOORDHIP_PLUGIN_AFFINITY_SCORE,
                                                      KOORDHIP_PLUGIN_TAINT_SCORE, KOORDHIP_PLUGIN_PTS,
                                                      KOORDHIP_PLUGIN_IPA};
  int64_t b = 0;
  for (int p = 0; p < KOORDHIP_NPLUGINS; p++)
    if (cfg->score_plugins & orc_score_plugin_bit(p)) b += 100 * cfg->plugin_weight[p];
  for (int e = 0; e < KOORDHIP_NEXT_PLUGINS; e++)
    if (cfg->score_plugins & ext[e]) b += 100 * (int64_t)cfg->ext_weight[e];
  return b;
}

/* key = (total+1) << 32 | (0xFFFFFFFF - node): larger is better, ties -> lower index. */
static inline uint64_t mkkey(int64_t total, int32_t node) {
  return ((uint64_t)(total + 1) << 32) | (uint64_t)(0xFFFFFFFFu - (uint32_t)node);
}

static int cmp_key_desc(const void *a, const void *b) {
  uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
  return x < y ? 1 : (x > y ? -1 : 0);
}

int orc_eval(const koordhip_config *cfg, const orc_state *st, const koordhip_pod *pods, int32_t n_pods,
             uint8_t *status, int32_t *scores, koordhip_topk *topk, int32_t k) {
  const int32_t n = st->n;
  uint64_t *keys = (topk && k > 0) ? (uint64_t *)malloc(sizeof(uint64_t) * (size_t)(n > 0 ? n : 1)) : NULL;
  const int rv = orc_resv_on(cfg, st);
  ((orc_state *)st)->cur_ext = NULL; /* plain records: no scalar requests */
  for (int32_t p = 0; p < n_pods; p++) {
    const koordhip_pod *pod = &pods[p];
    int32_t nk = 0;
    /* the cycle sees the Reservation restore (transformer.go:48-221); undone below */
    if (rv) orc_resv_restore((orc_state *)st, pod, +1);
    for (int32_t i = 0; i < n; i++) {
      int fit_ok = orc_fit_filter(cfg, st, pod, i);
      int la_ok = orc_la_filter(cfg, st, pod, i);
      int numa_ok = (cfg->filter_plugins & KOORDHIP_PLUGIN_NUMA) ? orc_numa_filter(cfg, st, pod, i) : 1;
      if (status) {
        uint8_t b = 0;
        if ((cfg->filter_plugins & KOORDHIP_PLUGIN_NODE_STATIC) && !orc_static_filter(st, pod, i))
          b |= KOORDHIP_ST_STATIC_FAIL;
        if ((cfg->filter_plugins & KOORDHIP_PLUGIN_FIT) && !fit_ok) b |= KOORDHIP_ST_FIT_FAIL;
        if ((cfg->filter_plugins & KOORDHIP_PLUGIN_LOADAWARE) && !la_ok) b |= KOORDHIP_ST_LA_FAIL;
        if (!numa_ok) b |= KOORDHIP_ST_NUMA_FAIL;
        if ((cfg->filter_plugins & KOORDHIP_PLUGIN_RESERVATION) && !resv_pass(st, pod, NULL, i))
          b |= KOORDHIP_ST_RESV_FAIL;
        status[(size_t)p * n + i] = b;
      }
      if (scores) {
        int32_t *row = scores + (size_t)p * KOORDHIP_NPLUGINS * n;
        row[0 * (size_t)n + i] = (cfg->score_plugins & KOORDHIP_PLUGIN_FIT) ? (int32_t)orc_fit_score(cfg, st, pod, i) : 0;
        row[1 * (size_t)n + i] =
            (cfg->score_plugins & KOORDHIP_PLUGIN_LOADAWARE) ? (int32_t)orc_la_score(cfg, st, pod, i) : 0;
        row[2 * (size_t)n + i] =
            (cfg->score_plugins & KOORDHIP_PLUGIN_NUMA) ? (int32_t)orc_numa_score(cfg, st, pod, i) : 0;
        row[3 * (size_t)n + i] =
            (cfg->score_plugins & KOORDHIP_PLUGIN_BALANCED) ? (int32_t)orc_bal_score(cfg, st, pod, i) : 0;
      }
      if (keys && orc_feasible(cfg, st, pod, NULL, NULL, NULL, i)) {
        int64_t t = orc_total(cfg, st, pod, i);
        if (rv) t = orc_resv_rank_total(cfg, st, pod, i, t);
        keys[nk++] = mkkey(t, i);
      }
    }
    if (rv) orc_resv_restore((orc_state *)st, pod, -1);
    if (keys) {
      qsort(keys, (size_t)nk, sizeof(uint64_t), cmp_key_desc);
      for (int32_t j = 0; j < k; j++) {
        koordhip_topk *o = &topk[(size_t)p * k + j];
        if (j < nk) {
          o->node = (int32_t)(0xFFFFFFFFu - (uint32_t)(keys[j] & 0xFFFFFFFFu));
          o->score = (int32_t)((keys[j] >> 32) - 1);
        } else {
          o->node = -1;
          o->score = 0;
        }
      }
    }
  }
  free(keys);
  return 0;
}

int orc_eval_ext(const koordhip_config *cfg, const orc_state *st, const koordhip_pod *pods, const koordhip_pod_ext *ext,
                 int32_t n_pods, uint16_t *status, int32_t *scores, koordhip_topk *topk, int32_t k) {
  static const uint32_t xb[KOORDHIP_NEXT_PLUGINS] = {KOORDHIP_PLUGIN_DEVICESHARE, KOORDHIP_PLUGIN_AFFINITY_SCORE,
                                                     KOORDHIP_PLUGIN_TAINT_SCORE, KOORDHIP_PLUGIN_PTS,
                                                     KOORDHIP_PLUGIN_IPA};
  const int32_t n = st->n;
  const int NP = KOORDHIP_NPLUGINS + KOORDHIP_NEXT_PLUGINS;
  const size_t nn = (size_t)(n > 0 ? n : 1);
  int32_t *feas = (int32_t *)malloc(sizeof(int32_t) * nn);
  int64_t *base = (int64_t *)malloc(sizeof(int64_t) * nn);
  int64_t *raw = (int64_t *)malloc(sizeof(int64_t) * KOORDHIP_NEXT_PLUGINS * nn);
  int64_t *ptsraw = (int64_t *)calloc(nn, sizeof(int64_t));
  int64_t *ipraw = (int64_t *)calloc(nn, sizeof(int64_t));
  uint64_t *keys = (uint64_t *)malloc(sizeof(uint64_t) * nn);
  const int rv = orc_resv_on(cfg, st);
  const int rs = rv && (cfg->score_plugins & KOORDHIP_PLUGIN_RESERVATION);
  const int pts_score = (cfg->score_plugins & KOORDHIP_PLUGIN_PTS) != 0;
  const int ipa_score = (cfg->score_plugins & KOORDHIP_PLUGIN_IPA) != 0;
  for (int32_t p = 0; p < n_pods; p++) {
    const koordhip_pod_ext *x = ext ? &ext[p] : NULL;
    const koordhip_pod pp = orc_devshare_pod(cfg, &pods[p], x);
    const koordhip_pod *pod = &pp;
    ((orc_state *)st)->cur_ext = x;
    ((orc_state *)st)->resv_restore = rv;
    orc_pts ps;
    orc_ipa ia;
    if (orc_pts_prefilter(cfg, st, x, &ps)) return -1;
    if (orc_ipa_prefilter(cfg, st, x, &ia)) return -1;
    if (rv) orc_resv_restore((orc_state *)st, pod, +1);
    int32_t nf = 0;
    for (int32_t i = 0; i < n; i++)
      if (orc_feasible(cfg, st, pod, x, &ps, &ia, i)) feas[nf++] = i;
    /* InterPodAffinity PreScore / Score: every node's raw score (its plane) */
    if (ipa_score && orc_ipa_prescore(st, x, &ia)) return -1;
    for (int32_t i = 0; i < n; i++) ipraw[i] = ipa_score ? orc_ipa_score(st, &ia, i) : 0;
    if (pts_score && orc_pts_prescore(st, x, &ps, feas, nf)) return -1;
    memset(ptsraw, 0, sizeof(int64_t) * nn);
    if (pts_score)
      for (int32_t j = 0; j < nf; j++) ptsraw[feas[j]] = orc_pts_score(st, x, &ps, feas[j]);
    for (int32_t i = 0; i < n; i++) {
      if (status) {
        uint16_t b = 0;
        if ((cfg->filter_plugins & KOORDHIP_PLUGIN_NODE_STATIC) && !orc_static_filter(st, pod, i))
          b |= KOORDHIP_ST_STATIC_FAIL;
        if ((cfg->filter_plugins & KOORDHIP_PLUGIN_FIT) && !orc_fit_filter(cfg, st, pod, i)) b |= KOORDHIP_ST_FIT_FAIL;
        if ((cfg->filter_plugins & KOORDHIP_PLUGIN_FIT) && !orc_xfit_filter(st, x, i)) b |= KOORDHIP_ST_XFIT_FAIL;
        if ((cfg->filter_plugins & KOORDHIP_PLUGIN_LOADAWARE) && !orc_la_filter(cfg, st, pod, i)) b |= KOORDHIP_ST_LA_FAIL;
        if ((cfg->filter_plugins & KOORDHIP_PLUGIN_NUMA) && !orc_numa_filter(cfg, st, pod, i)) b |= KOORDHIP_ST_NUMA_FAIL;
        if ((cfg->filter_plugins & KOORDHIP_PLUGIN_RESERVATION) && !resv_pass(st, pod, x, i))
          b |= KOORDHIP_ST_RESV_FAIL;
        if ((cfg->filter_plugins & KOORDHIP_PLUGIN_DEVICESHARE) && !orc_dev_filter(st, pod, x, i)) b |= KOORDHIP_ST_DEVICE_FAIL;
        if ((cfg->filter_plugins & KOORDHIP_PLUGIN_PTS) && !orc_pts_filter(st, x, &ps, i)) b |= KOORDHIP_ST_PTS_FAIL;
        if ((cfg->filter_plugins & KOORDHIP_PLUGIN_IPA) && !orc_ipa_filter(st, x, &ia, i)) b |= KOORDHIP_ST_IPA_FAIL;
        status[(size_t)p * n + i] = b;
      }
      if (scores) {
        int32_t *row = scores + (size_t)p * NP * n;
        const int nom = rs && orc_resv_nominated(st, pod, i);
        row[0 * (size_t)n + i] = (cfg->score_plugins & KOORDHIP_PLUGIN_FIT) ? (int32_t)orc_fit_score(cfg, st, pod, i) : 0;
        row[1 * (size_t)n + i] =
            (cfg->score_plugins & KOORDHIP_PLUGIN_LOADAWARE) ? (int32_t)orc_la_score(cfg, st, pod, i) : 0;
        row[2 * (size_t)n + i] =
            (cfg->score_plugins & KOORDHIP_PLUGIN_NUMA) ? (int32_t)orc_numa_score(cfg, st, pod, i) : 0;
        row[3 * (size_t)n + i] =
            (cfg->score_plugins & KOORDHIP_PLUGIN_BALANCED) ? (int32_t)orc_bal_score(cfg, st, pod, i) : 0;
        row[4 * (size_t)n + i] =
            (cfg->score_plugins & KOORDHIP_PLUGIN_DEVICESHARE) ? (int32_t)orc_dev_score(cfg, st, pod, x, i, nom) : 0;
        row[5 * (size_t)n + i] =
            (cfg->score_plugins & KOORDHIP_PLUGIN_AFFINITY_SCORE) ? (int32_t)orc_static_score(st, pod, i, 0) : 0;
        row[6 * (size_t)n + i] =
            (cfg->score_plugins & KOORDHIP_PLUGIN_TAINT_SCORE) ? (int32_t)orc_static_score(st, pod, i, 1) : 0;
        /* PodTopologySpread: the raw Score of a feasible node (0 elsewhere and on ignored nodes) */
        row[7 * (size_t)n + i] = (int32_t)ptsraw[i];
        /* InterPodAffinity: the raw Score of every node */
        row[8 * (size_t)n + i] = (int32_t)ipraw[i];
      }
    }
    if (topk && k > 0) {
      for (int32_t j = 0; j < nf; j++) {
        const int32_t i = feas[j];
        const int nom = rs && orc_resv_nominated(st, pod, i);
        base[j] = orc_total(cfg, st, pod, i);
        raw[j] = (cfg->score_plugins & KOORDHIP_PLUGIN_DEVICESHARE) ? orc_dev_score(cfg, st, pod, x, i, nom) : 0;
        raw[(size_t)nf + j] = (cfg->score_plugins & KOORDHIP_PLUGIN_AFFINITY_SCORE) ? orc_static_score(st, pod, i, 0) : 0;
        raw[2 * (size_t)nf + j] = (cfg->score_plugins & KOORDHIP_PLUGIN_TAINT_SCORE) ? orc_static_score(st, pod, i, 1) : 0;
        raw[3 * (size_t)nf + j] = ptsraw[i];
        raw[4 * (size_t)nf + j] = ipraw[i];
      }
      for (int e = 0; e < 3; e++)
        if (cfg->score_plugins & xb[e]) orc_default_normalize(raw + (size_t)e * nf, nf, e == 2);
      if (pts_score) orc_pts_normalize(&ps, feas, raw + 3 * (size_t)nf, nf);
      if (ipa_score) orc_ipa_normalize(raw + 4 * (size_t)nf, nf);
      for (int32_t j = 0; j < nf; j++) {
        const int32_t i = feas[j];
        int64_t t = base[j];
        for (int e = 0; e < KOORDHIP_NEXT_PLUGINS; e++)
          if (cfg->score_plugins & xb[e]) t += (int64_t)cfg->ext_weight[e] * raw[(size_t)e * nf + j];
        if (rv) t = orc_resv_rank_total(cfg, st, pod, i, t);
        keys[j] = mkkey(t, i);
      }
      qsort(keys, (size_t)nf, sizeof(uint64_t), cmp_key_desc);
      for (int32_t j = 0; j < k; j++) {
        koordhip_topk *o = &topk[(size_t)p * k + j];
        if (j < nf) {
          o->node = (int32_t)(0xFFFFFFFFu - (uint32_t)(keys[j] & 0xFFFFFFFFu));
          o->score = (int32_t)((keys[j] >> 32) - 1);
        } else {
          o->node = -1;
          o->score = 0;
        }
      }
    }
    if (rv) orc_resv_restore((orc_state *)st, pod, -1);
    orc_pts_free(&ps);
    orc_ipa_free(&ia);
  }
  free(feas);
  free(base);
  free(raw);
  free(ptsraw);
  free(ipraw);
  free(keys);
  return 0;
}

/* Reserve: podAssignCache.assign (pod_assign_cache.go:53-68) makes the pod an
 * estimated assigned pod on the node (load_aware.go:353-372: no metric ->
 * EstimatePod); (upstream) NodeInfo.AddPod adds Requested/NonZeroRequested and
 * one pod (mirror: reservation/transformer.go:280-333).  sign = -1: Unreserve.
 * NodeNUMAResource Reserve allocates a cpuset for a cpuset pod (plugin.go:365-405);
 * when it fails the framework unreserves every plugin: nothing is committed. */
static int numa_on(const koordhip_config *cfg) {
  return ((cfg->filter_plugins | cfg->score_plugins) & KOORDHIP_PLUGIN_NUMA) != 0;
}

int orc_commit(const koordhip_config *cfg, orc_state *st, const koordhip_pod *pod, int32_t i, int sign,
               uint64_t *cpus) {
  const int rv = orc_resv_on(cfg, st) && orc_resv_node_present(st, i);
  /* Unreserve of a pod one of its node's reservations could have taken: whether
   * it did (state.assumed, plugin.go:591-597) is not passed back */
  if (rv && sign < 0 && orc_resv_node_matchable(st, pod, i)) return KOORDHIP_EINVAL;
  uint64_t got[KOORDHIP_NUMA_WORDS] = {0, 0, 0, 0};
  if (numa_on(cfg) && orc_numa_reserve_active(st, pod, i)) {
    if (sign > 0) {
      /* the reserved CPUs of the reservation PreScore nominated (RestoreReservation state) */
      uint64_t pref[KOORDHIP_NUMA_WORDS];
      orc_resv_pref(cfg, st, pod, i, pref);
      if (!orc_numa_reserve(st, pod, i, got, pref)) return KOORDHIP_ERESERVE;
      if (cpus)
        for (int w = 0; w < KOORDHIP_NUMA_WORDS; w++) cpus[w] = got[w];
    } else if (st->soa->numa_flags && KOORDHIP_NODE_NUMA_POLICY(st->soa->numa_flags[i]) != KOORDHIP_NUMA_TOPO_NONE) {
      return KOORDHIP_EINVAL; /* the zone amounts of an earlier Reserve are not passed back */
    } else if (cpus) {
      orc_numa_release(st, i, cpus);
    }
  } else if (cpus && sign > 0) {
    for (int w = 0; w < KOORDHIP_NUMA_WORDS; w++) cpus[w] = 0;
  }
  if (rv && sign > 0) orc_resv_assume(st, pod, i, got); /* Reservation Reserve: assumePod (plugin.go:550-573) */
  for (int r = 0; r < KOORDHIP_NRES; r++) st->requested[r][i] += sign * pod->req[r];
  st->nz_cpu_m[i] += sign * pod->nz_cpu_m;
  st->nz_mem[i] += sign * pod->nz_mem;
  st->npods[i] += sign;
  st->la_used_cpu_m[i] += sign * pod->est_cpu;
  st->la_used_mem[i] += sign * pod->est_mem;
  if (pod->flags & KOORDHIP_POD_PROD) { /* prod-only walk, load_aware.go:349-351 */
    st->la_used_prod_cpu_m[i] += sign * pod->est_cpu;
    st->la_used_prod_mem[i] += sign * pod->est_mem;
  }
  return 0;
}

/* The Reserve of a pod with its koordhip_pod_ext: DeviceShare's allocation
 * is decided first without changing anything (the reserve plugins run in
 * profile order -- LoadAwareScheduling, NodeNUMAResource, DeviceShare --
 * and a failure unreserves every one of them, so any failure commits
 * nothing), then the plugins' Reserve, then NodeInfo.AddPod of the pod's
 * extended scalars. */
int orc_commit_ext(const koordhip_config *cfg, orc_state *st, const koordhip_pod *pod, const koordhip_pod_ext *x,
                   int32_t i, uint64_t *cpus, int nominated, uint32_t *devs) {
  uint32_t slots[KOORDHIP_DEV_TYPES] = {0, 0, 0};
  const int dev = (cfg->filter_plugins | cfg->score_plugins) & KOORDHIP_PLUGIN_DEVICESHARE;
  const koordhip_pod pp = orc_devshare_pod(cfg, pod, x);
  pod = &pp;
  st->cur_ext = x;
  st->resv_restore = orc_resv_on(cfg, st);
  /* the reservation the Reservation Reserve will assume the pod into, decided
   * on the state before any Reserve */
  const int assumed = (st->resv_restore && orc_resv_node_present(st, i)) ? orc_resv_nominate(st, pod, i) : -1;
  if (dev && orc_dev_reserve(cfg, st, pod, x, i, nominated, slots, 0)) return KOORDHIP_ERESERVE;
  const int rc = orc_commit(cfg, st, pod, i, +1, cpus);
  if (rc) return rc;
  if (dev) orc_dev_apply(st, x, i, slots, assumed);
  if (devs)
    for (int t = 0; t < KOORDHIP_DEV_TYPES; t++) devs[t] = slots[t];
  if (x)
    for (int j = 0; j < KOORDHIP_NXRES; j++)
      if ((x->xmask >> j) & 1u) st->xrequested[(size_t)j * st->n + i] += x->xreq[j];
  orc_pts_commit(st, x, i); /* NodeInfo.AddPod: one more pod for the constraints it matches */
  orc_ipa_commit(st, x, i); /* ... and for the InterPodAffinity entries that count it */
  return 0;
}

void orc_set_cpuset_out(orc_state *st, uint64_t *cpus) { st->cpuset_out = cpus; }

/* ------------------------------------------------------------------------ */
/* parallelize.Until (pkg/util/parallelize/parallelism.go:28-49)            */
/* ------------------------------------------------------------------------ */

typedef void (*piece_fn)(void *arg, int32_t lo, int32_t hi);

typedef struct pool {
  int32_t nthreads;
  pthread_t *tid;
  pthread_mutex_t mu;
  pthread_cond_t work, idle;
  int64_t gen;          /* job generation (under mu) */
  int32_t done;         /* workers finished this generation (under mu) */
  int32_t quit;
  _Atomic int32_t next; /* next piece */
  int32_t pieces, chunk;
  piece_fn fn;
  void *arg;
} pool;

/* chunkSizeFor: max(1, min(sqrt(n), n/parallelism + 1)), parallelism.go:33-44 */
static int32_t chunk_size_for(int32_t n, int32_t parallelism) {
  int32_t s = (int32_t)sqrt((double)n);
  int32_t r = n / parallelism + 1;
  if (s > r) s = r;
  else if (s < 1) s = 1;
  return s;
}

static void run_pieces(pool *p) {
  for (;;) {
    int32_t lo = atomic_fetch_add(&p->next, p->chunk);
    if (lo >= p->pieces) break;
    int32_t hi = lo + p->chunk;
    if (hi > p->pieces) hi = p->pieces;
    p->fn(p->arg, lo, hi);
  }
}

/* Workers block between jobs (a goroutine pool parks the same way); spinning
 * waiters would compete with the working threads for a shared CPU quota. */
static void *worker(void *a) {
  pool *p = (pool *)a;
  int64_t seen = 0;
  for (;;) {
    pthread_mutex_lock(&p->mu);
    while (p->gen == seen && !p->quit) pthread_cond_wait(&p->work, &p->mu);
    if (p->quit) {
      pthread_mutex_unlock(&p->mu);
      return NULL;
    }
    seen = p->gen;
    pthread_mutex_unlock(&p->mu);
    run_pieces(p);
    pthread_mutex_lock(&p->mu);
    if (++p->done == p->nthreads - 1) pthread_cond_signal(&p->idle);
    pthread_mutex_unlock(&p->mu);
  }
}

static int pool_init(pool *p, int32_t nthreads) {
  memset(p, 0, sizeof(*p));
  p->nthreads = nthreads;
  if (nthreads <= 1) return 0;
  pthread_mutex_init(&p->mu, NULL);
  pthread_cond_init(&p->work, NULL);
  pthread_cond_init(&p->idle, NULL);
  p->tid = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
  for (int32_t t = 0; t < nthreads - 1; t++) /* the caller is the last worker */
    if (pthread_create(&p->tid[t], NULL, worker, p)) return -1;
  return 0;
}

static void pool_free(pool *p) {
  if (p->nthreads > 1) {
    pthread_mutex_lock(&p->mu);
    p->quit = 1;
    pthread_cond_broadcast(&p->work);
    pthread_mutex_unlock(&p->mu);
    for (int32_t t = 0; t < p->nthreads - 1; t++) pthread_join(p->tid[t], NULL);
    free(p->tid);
    pthread_mutex_destroy(&p->mu);
    pthread_cond_destroy(&p->work);
    pthread_cond_destroy(&p->idle);
  }
}

/* Until(ctx, pieces, f) with `nthreads` workers and the reference chunking. */
static void pool_until(pool *p, int32_t pieces, piece_fn fn, void *arg) {
  if (pieces <= 0) return;
  if (p->nthreads <= 1) {
    fn(arg, 0, pieces);
    return;
  }
  p->pieces = pieces;
  p->chunk = chunk_size_for(pieces, 16);
  p->fn = fn;
  p->arg = arg;
  atomic_store(&p->next, 0);
  pthread_mutex_lock(&p->mu);
  p->done = 0;
  p->gen++;
  pthread_cond_broadcast(&p->work);
  pthread_mutex_unlock(&p->mu);
  run_pieces(p);
  pthread_mutex_lock(&p->mu);
  while (p->done < p->nthreads - 1) pthread_cond_wait(&p->idle, &p->mu);
  pthread_mutex_unlock(&p->mu);
}

/* ------------------------------------------------------------------------ */
/* Greedy stream with the reference loop structure                           */
/* ------------------------------------------------------------------------ */

typedef struct stream_ctx {
  const koordhip_config *cfg;
  const orc_state *st;
  const koordhip_pod *pod;
  const koordhip_pod_ext *ext;
  _Atomic int32_t nfeasible;
  int32_t *feasible;      /* node ids (unordered, like upstream's atomic append) */
  int resv_score;         /* the Reservation plugin scores (its PreScore nominates) */
  int64_t *plugin_scores; /* [KOORDHIP_NPLUGINS][nfeasible] */
  orc_pts *pts;           /* PodTopologySpread PreFilter / PreScore state of the pod */
  orc_ipa *ipa;           /* InterPodAffinity PreFilter / PreScore state of the pod */
} stream_ctx;

/* (upstream) findNodesThatPassFilters checkNode: RunFilterPlugins, append on success. */
static void filter_piece(void *a, int32_t lo, int32_t hi) {
  stream_ctx *c = (stream_ctx *)a;
  for (int32_t i = lo; i < hi; i++)
    if (orc_feasible(c->cfg, c->st, c->pod, c->ext, c->pts, c->ipa, i))
      c->feasible[atomic_fetch_add(&c->nfeasible, 1)] = i;
}

/* (upstream) framework.RunScorePlugins: one Until over nodes, every score plugin per node. */
static void score_piece(void *a, int32_t lo, int32_t hi) {
  stream_ctx *c = (stream_ctx *)a;
  int32_t nf = atomic_load(&c->nfeasible);
  for (int32_t j = lo; j < hi; j++) {
    int32_t i = c->feasible[j];
    c->plugin_scores[j] =
        (c->cfg->score_plugins & KOORDHIP_PLUGIN_FIT) ? orc_fit_score(c->cfg, c->st, c->pod, i) : 0;
    c->plugin_scores[(size_t)nf + j] =
        (c->cfg->score_plugins & KOORDHIP_PLUGIN_LOADAWARE) ? orc_la_score(c->cfg, c->st, c->pod, i) : 0;
    c->plugin_scores[2 * (size_t)nf + j] =
        (c->cfg->score_plugins & KOORDHIP_PLUGIN_NUMA) ? orc_numa_score(c->cfg, c->st, c->pod, i) : 0;
    c->plugin_scores[3 * (size_t)nf + j] =
        (c->cfg->score_plugins & KOORDHIP_PLUGIN_BALANCED) ? orc_bal_score(c->cfg, c->st, c->pod, i) : 0;
    /* the normalized plugins' raw scores (planes NPLUGINS..; the Reservation
     * plugin's normalized plane follows them) */
    if (c->cfg->score_plugins & (KOORDHIP_PLUGIN_DEVICESHARE | KOORDHIP_PLUGIN_AFFINITY_SCORE |
                                 KOORDHIP_PLUGIN_TAINT_SCORE)) {
      int64_t *x = c->plugin_scores + (size_t)KOORDHIP_NPLUGINS * nf;
      const int nom = c->resv_score && orc_resv_nominated(c->st, c->pod, i);
      x[j] = (c->cfg->score_plugins & KOORDHIP_PLUGIN_DEVICESHARE) ? orc_dev_score(c->cfg, c->st, c->pod, c->ext, i, nom) : 0;
      x[(size_t)nf + j] =
          (c->cfg->score_plugins & KOORDHIP_PLUGIN_AFFINITY_SCORE) ? orc_static_score(c->st, c->pod, i, 0) : 0;
      x[2 * (size_t)nf + j] =
          (c->cfg->score_plugins & KOORDHIP_PLUGIN_TAINT_SCORE) ? orc_static_score(c->st, c->pod, i, 1) : 0;
    }
    if (c->cfg->score_plugins & KOORDHIP_PLUGIN_PTS)
      c->plugin_scores[(size_t)(KOORDHIP_NPLUGINS + 3) * nf + j] = orc_pts_score(c->st, c->ext, c->pts, i);
    if (c->cfg->score_plugins & KOORDHIP_PLUGIN_IPA)
      c->plugin_scores[(size_t)(KOORDHIP_NPLUGINS + 4) * nf + j] = orc_ipa_score(c->st, c->ipa, i);
  }
}

int orc_place_stream(const koordhip_config *cfg, orc_state *st, const koordhip_pod *pods, int32_t n_pods,
                     int32_t *out_node, int32_t threads) {
  st->cur_ext = NULL;
  return orc_place_stream_ext(cfg, st, pods, NULL, n_pods, out_node, threads);
}

void orc_set_dev_out(orc_state *st, uint32_t *devs) { st->dev_out = devs; }

static const uint32_t k_ext_bits[KOORDHIP_NEXT_PLUGINS] = {KOORDHIP_PLUGIN_DEVICESHARE, KOORDHIP_PLUGIN_AFFINITY_SCORE,
                                                           KOORDHIP_PLUGIN_TAINT_SCORE, KOORDHIP_PLUGIN_PTS,
                                                           KOORDHIP_PLUGIN_IPA};

int orc_place_stream_ext(const koordhip_config *cfg, orc_state *st, const koordhip_pod *pods,
                         const koordhip_pod_ext *ext, int32_t n_pods, int32_t *out_node, int32_t threads) {
  const int32_t n = st->n;
  pool pl;
  if (pool_init(&pl, threads)) return -1;
  stream_ctx c;
  c.cfg = cfg;
  c.st = st;
  c.feasible = (int32_t *)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
  /* planes: NPLUGINS plugins, NEXT_PLUGINS normalized ones, the Reservation's normalized */
  c.plugin_scores = (int64_t *)malloc(sizeof(int64_t) * (KOORDHIP_NPLUGINS + KOORDHIP_NEXT_PLUGINS + 1) *
                                      (size_t)(n > 0 ? n : 1));
  const int rv = orc_resv_on(cfg, st);
  const int rs = rv && (cfg->score_plugins & KOORDHIP_PLUGIN_RESERVATION);
  c.resv_score = rs;
  orc_pts ps;
  memset(&ps, 0, sizeof(ps));
  c.pts = &ps;
  orc_ipa ia;
  memset(&ia, 0, sizeof(ia));
  c.ipa = &ia;
  for (int32_t p = 0; p < n_pods; p++) {
    c.ext = ext ? &ext[p] : NULL;
    const koordhip_pod pp = orc_devshare_pod(cfg, &pods[p], c.ext);
    c.pod = &pp;
    st->cur_ext = c.ext;
    st->resv_restore = rv;
    uint32_t *devs = st->dev_out ? st->dev_out + (size_t)p * KOORDHIP_DEV_TYPES : NULL;
    if (devs) memset(devs, 0, sizeof(uint32_t) * KOORDHIP_DEV_TYPES);
    orc_pts_free(&ps);
    orc_ipa_free(&ia);
    if (orc_pts_prefilter(cfg, st, c.ext, &ps)) return -1; /* PodTopologySpread PreFilter */
    if (orc_ipa_prefilter(cfg, st, c.ext, &ia)) return -1; /* InterPodAffinity PreFilter */
    /* Reservation BeforePreFilter: the cycle's NodeInfos are the restored ones */
    if (rv) orc_resv_restore(st, c.pod, +1);
    atomic_store(&c.nfeasible, 0);
    pool_until(&pl, n, filter_piece, &c);
    int32_t nf = atomic_load(&c.nfeasible);
    if (nf == 0) {
      if (rv) orc_resv_restore(st, c.pod, -1);
      out_node[p] = KOORDHIP_UNSCHEDULABLE;
      if (st->cpuset_out) memset(st->cpuset_out + (size_t)p * KOORDHIP_NUMA_WORDS, 0, 8 * KOORDHIP_NUMA_WORDS);
      continue;
    }
    /* PodTopologySpread PreScore over the feasible list (before the Score Until) */
    if ((cfg->score_plugins & KOORDHIP_PLUGIN_PTS) && orc_pts_prescore(st, c.ext, &ps, c.feasible, nf)) return -1;
    if ((cfg->score_plugins & KOORDHIP_PLUGIN_IPA) && orc_ipa_prescore(st, c.ext, &ia)) return -1;
    pool_until(&pl, nf, score_piece, &c);
    /* NormalizeScore of the normalized plugins (DefaultNormalizeScore over the
     * feasible list: DeviceShare scoring.go:78-80, upstream NodeAffinity, and
     * TaintToleration reversed), Reservation PreScore + Score + NormalizeScore */
    int64_t *xs = c.plugin_scores + (size_t)KOORDHIP_NPLUGINS * nf;
    for (int e = 0; e < 3; e++)
      if (cfg->score_plugins & k_ext_bits[e]) orc_default_normalize(xs + (size_t)e * nf, nf, e == 2);
    if (cfg->score_plugins & KOORDHIP_PLUGIN_PTS) orc_pts_normalize(&ps, c.feasible, xs + 3 * (size_t)nf, nf);
    if (cfg->score_plugins & KOORDHIP_PLUGIN_IPA) orc_ipa_normalize(xs + 4 * (size_t)nf, nf);
    int64_t *norm = c.plugin_scores + (size_t)(KOORDHIP_NPLUGINS + KOORDHIP_NEXT_PLUGINS) * nf;
    if (rs) orc_resv_normalized(st, c.pod, c.feasible, nf, norm);
    /* (upstream) prioritizeNodes: sum of score x weight; selectHost: max,
     * reservoir-random tie-break REPLACED by lowest node index (BASELINE.json). */
    int64_t best = -1;
    int32_t best_node = -1, best_j = -1;
    for (int32_t j = 0; j < nf; j++) {
      int32_t i = c.feasible[j];
      int64_t t = cfg->plugin_weight[0] * c.plugin_scores[j] + cfg->plugin_weight[1] * c.plugin_scores[(size_t)nf + j] +
                  cfg->plugin_weight[2] * c.plugin_scores[2 * (size_t)nf + j] +
                  cfg->plugin_weight[3] * c.plugin_scores[3 * (size_t)nf + j];
      for (int e = 0; e < KOORDHIP_NEXT_PLUGINS; e++)
        if (cfg->score_plugins & k_ext_bits[e]) t += (int64_t)cfg->ext_weight[e] * xs[(size_t)e * nf + j];
      if (rs) t += (int64_t)cfg->reservation_weight * norm[j];
      if (t > best || (t == best && i < best_node)) {
        best = t;
        best_node = i;
        best_j = j;
      }
    }
    (void)best_j;
    /* One feasible node: (upstream) schedulePod returns it without
     * prioritizeNodes, so PreScore nominates no reservation */
    const int nominated = rs && nf > 1 && orc_resv_nominated(st, c.pod, best_node);
    if (rv) orc_resv_restore(st, c.pod, -1);
    uint64_t *cs = st->cpuset_out ? st->cpuset_out + (size_t)p * KOORDHIP_NUMA_WORDS : NULL;
    /* Reserve (+ AssumePod); a failed Reserve leaves no state and is not retried. */
    st->no_prescore = nf == 1;
    out_node[p] = orc_commit_ext(cfg, st, c.pod, c.ext, best_node, cs, nominated, devs) ? KOORDHIP_RESERVE_FAILED
                                                                                            : best_node;
    st->no_prescore = 0;
  }
  orc_pts_free(&ps);
  orc_ipa_free(&ia);
  free(c.feasible);
  free(c.plugin_scores);
  pool_free(&pl);
  return 0;
}
