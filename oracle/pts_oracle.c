/* TEST INFRASTRUCTURE: CPU restatement of upstream PodTopologySpread
 * (k8s.io/kubernetes v1.24.15 pkg/scheduler/framework/plugins/podtopologyspread,
 * go.mod:57,275 of the reference; the module is not vendored, so parity with
 * upstream is UNPINNED: the rules follow the published sources as cited per
 * function, restated over the engine's columns).  It is the checker of the
 * sequential cycle (csrc/seq.hip), never the thing measured.
 *
 * Columns (include/koordhip.h): pts_dom [keys][n] (domain of the node for
 * topology key k, -1 = no such label; the node index for
 * kubernetes.io/hostname), pts_cnt [cons][n] (the node's pods in constraint c's
 * namespace that its selector matches: countPodsMatchSelector), pts_elig [n]
 * (bit 2s: the node matches spread class s's required node affinity and has
 * every DoNotSchedule key; bit 2s+1: ... every ScheduleAnyway key).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "koord_oracle.h"

static int32_t pts_dsize(const orc_state *st, int k) {
  return ((st->soa->pts_hostname >> k) & 1u) ? st->n : st->soa->pts_ndom[k];
}
static int32_t pts_dom(const orc_state *st, int k, int32_t i) { return st->soa->pts_dom[(size_t)k * st->n + i]; }
static int pts_key_of(const orc_state *st, const koordhip_pod_ext *x, int j) { return st->soa->pts_cons_key[x->pts_c[j]]; }
static int pts_hostname(const orc_state *st, int k) { return (st->soa->pts_hostname >> k) & 1u; }

int orc_pts_active(const koordhip_config *cfg, const orc_state *st, const koordhip_pod_ext *x) {
  return ((cfg->filter_plugins | cfg->score_plugins) & KOORDHIP_PLUGIN_PTS) && st->soa->pts_keys > 0 && x &&
         x->pts_n > 0;
}

void orc_pts_free(orc_pts *ps) {
  for (int k = 0; k < KOORDHIP_PTS_KEYS; k++) {
    free(ps->fpres[k]);
    free(ps->fmatch[k]);
    free(ps->spres[k]);
    free(ps->scount[k]);
  }
  free(ps->ignored);
  memset(ps, 0, sizeof(*ps));
}

/* PreFilter, filtering.go calPreFilterState: the DoNotSchedule constraints;
 * TpPairToMatchNum over the (key, value) pairs of the nodes that match the
 * pod's required node affinity and carry every hard key, summed over EVERY
 * node of such a pair (two constraints of one key share the pair's counter),
 * and per key the minimum over its pairs (criticalPaths[0], MaxInt32 when no
 * pair exists). */
int orc_pts_prefilter(const koordhip_config *cfg, const orc_state *st, const koordhip_pod_ext *x, orc_pts *ps) {
  memset(ps, 0, sizeof(*ps));
  if (!orc_pts_active(cfg, st, x)) return 0;
  ps->on = 1;
  const int32_t n = st->n;
  const int cls = x->pts_class;
  for (int j = 0; j < x->pts_n; j++) {
    if (x->pts_fl[j] & KOORDHIP_PTS_HARD) ps->hj[ps->nh++] = j;
    else ps->sj[ps->ns++] = j;
  }
  if (!(cfg->filter_plugins & KOORDHIP_PLUGIN_PTS)) ps->nh = 0;
  for (int q = 0; q < ps->nh; q++) {
    const int k = pts_key_of(st, x, ps->hj[q]);
    if (!ps->fpres[k]) {
      const int32_t D = pts_dsize(st, k);
      ps->fpres[k] = (uint8_t *)calloc((size_t)(D > 0 ? D : 1), 1);
      ps->fmatch[k] = (int64_t *)calloc((size_t)(D > 0 ? D : 1), sizeof(int64_t));
      if (!ps->fpres[k] || !ps->fmatch[k]) return -1;
    }
  }
  for (int32_t i = 0; i < n; i++) {
    if (!((st->soa->pts_elig[i] >> (2 * cls)) & 1u)) continue;
    for (int q = 0; q < ps->nh; q++) {
      const int k = pts_key_of(st, x, ps->hj[q]);
      const int32_t d = pts_dom(st, k, i);
      if (d >= 0) ps->fpres[k][d] = 1; /* (the class's eligibility implies the key) */
    }
  }
  for (int32_t i = 0; i < n; i++)
    for (int q = 0; q < ps->nh; q++) {
      const int j = ps->hj[q], k = pts_key_of(st, x, j);
      const int32_t d = pts_dom(st, k, i);
      if (d < 0 || !ps->fpres[k][d]) continue;
      ps->fmatch[k][d] += st->pts_cnt[(size_t)x->pts_c[j] * n + i];
    }
  for (int k = 0; k < KOORDHIP_PTS_KEYS; k++) {
    ps->fmin[k] = INT32_MAX;
    if (!ps->fpres[k]) continue;
    const int32_t D = pts_dsize(st, k);
    for (int32_t d = 0; d < D; d++)
      if (ps->fpres[k][d] && ps->fmatch[k][d] < ps->fmin[k]) ps->fmin[k] = ps->fmatch[k][d];
  }
  return 0;
}

/* Filter, filtering.go Filter: every hard constraint's key on the node
 * (else UnschedulableAndUnresolvable), and matchNum + selfMatch - minMatch <=
 * maxSkew (a pair absent from TpPairToMatchNum counts 0). 1 = passes. */
int orc_pts_filter(const orc_state *st, const koordhip_pod_ext *x, const orc_pts *ps, int32_t i) {
  if (!ps || !ps->on) return 1;
  for (int q = 0; q < ps->nh; q++) {
    const int j = ps->hj[q], k = pts_key_of(st, x, j);
    const int32_t d = pts_dom(st, k, i);
    if (d < 0) return 0;
    const int64_t self = (x->pts_fl[j] & KOORDHIP_PTS_SELF) ? 1 : 0;
    const int64_t match = ps->fpres[k][d] ? ps->fmatch[k][d] : 0;
    if (match + self - ps->fmin[k] > x->pts_skew[j]) return 0;
  }
  return 1;
}

/* PreScore, scoring.go initPreScoreState + the processAllNode pass: over the
 * feasible nodes, those lacking a ScheduleAnyway key are IgnoredNodes
 * (requireAllTopologies: the pod has explicit constraints); every other one
 * creates its (key, value) pair -- credited to topoSize of the first soft
 * constraint of that key in the pod's order -- except for hostname; weights
 * log(topoSize + 2) (hostname: feasible - ignored); then every node that
 * matches the pod's required affinity and carries the soft keys adds its
 * selector counts to its pair, if the pair exists. */
int orc_pts_prescore(const orc_state *st, const koordhip_pod_ext *x, orc_pts *ps, const int32_t *feas, int32_t nf) {
  if (!ps || !ps->on) return 0;
  const int32_t n = st->n;
  const int cls = x->pts_class;
  ps->scored = 1;
  ps->ignored = (uint8_t *)calloc((size_t)(n > 0 ? n : 1), 1);
  if (!ps->ignored) return -1;
  for (int q = 0; q < ps->ns; q++) {
    const int k = pts_key_of(st, x, ps->sj[q]);
    if (pts_hostname(st, k) || ps->spres[k]) continue;
    const int32_t D = pts_dsize(st, k);
    ps->spres[k] = (uint8_t *)calloc((size_t)(D > 0 ? D : 1), 1);
    ps->scount[k] = (int64_t *)calloc((size_t)(D > 0 ? D : 1), sizeof(int64_t));
    if (!ps->spres[k] || !ps->scount[k]) return -1;
  }
  int64_t topo[KOORDHIP_PTS_POD] = {0, 0, 0, 0};
  int32_t nign = 0;
  for (int32_t f = 0; f < nf; f++) {
    const int32_t i = feas[f];
    int all = 1;
    for (int q = 0; q < ps->ns; q++)
      if (pts_dom(st, pts_key_of(st, x, ps->sj[q]), i) < 0) all = 0;
    if (!all) {
      ps->ignored[i] = 1;
      nign++;
      continue;
    }
    for (int q = 0; q < ps->ns; q++) {
      const int k = pts_key_of(st, x, ps->sj[q]);
      if (pts_hostname(st, k)) continue;
      const int32_t d = pts_dom(st, k, i);
      if (!ps->spres[k][d]) {
        ps->spres[k][d] = 1;
        topo[q]++;
      }
    }
  }
  for (int q = 0; q < ps->ns; q++) {
    const int k = pts_key_of(st, x, ps->sj[q]);
    const int64_t sz = pts_hostname(st, k) ? (int64_t)nf - nign : topo[q];
    ps->weight[q] = log((double)(sz + 2)); /* topologyNormalizingWeight */
  }
  for (int32_t i = 0; i < n; i++) {
    if (!((st->soa->pts_elig[i] >> (2 * cls + 1)) & 1u)) continue;
    for (int q = 0; q < ps->ns; q++) {
      const int j = ps->sj[q], k = pts_key_of(st, x, j);
      if (pts_hostname(st, k)) continue;
      const int32_t d = pts_dom(st, k, i);
      if (d < 0 || !ps->spres[k][d]) continue;
      ps->scount[k][d] += st->pts_cnt[(size_t)x->pts_c[j] * n + i];
    }
  }
  return 0;
}

/* Score, scoring.go Score: 0 on an ignored node; else per soft constraint
 * scoreForCount(cnt, maxSkew, weight) = cnt * weight + (maxSkew - 1) with cnt
 * the node's own selector count for hostname, the pair's count otherwise;
 * int64(math.Round(sum)).  The raw score (before NormalizeScore). */
int64_t orc_pts_score(const orc_state *st, const koordhip_pod_ext *x, const orc_pts *ps, int32_t i) {
  if (!ps || !ps->scored || ps->ignored[i]) return 0;
  double score = 0.0;
  for (int q = 0; q < ps->ns; q++) {
    const int j = ps->sj[q], k = pts_key_of(st, x, j);
    const int32_t d = pts_dom(st, k, i);
    if (d < 0) continue;
    const int64_t cnt = pts_hostname(st, k) ? (int64_t)st->pts_cnt[(size_t)x->pts_c[j] * st->n + i] : ps->scount[k][d];
    score += (double)cnt * ps->weight[q] + (double)(x->pts_skew[j] - 1);
  }
  return (int64_t)round(score);
}

/* NormalizeScore, scoring.go: min / max over the non-ignored nodes; ignored
 * -> 0; max 0 -> MaxNodeScore; else MaxNodeScore * (max + min - s) / max. */
void orc_pts_normalize(const orc_pts *ps, const int32_t *feas, int64_t *scores, int32_t nf) {
  int64_t mn = INT64_MAX, mx = 0;
  for (int32_t f = 0; f < nf; f++) {
    if (ps && ps->scored && ps->ignored[feas[f]]) continue;
    if (scores[f] < mn) mn = scores[f];
    if (scores[f] > mx) mx = scores[f];
  }
  for (int32_t f = 0; f < nf; f++) {
    if (ps && ps->scored && ps->ignored[feas[f]]) {
      scores[f] = 0;
      continue;
    }
    if (mx == 0) {
      scores[f] = 100;
      continue;
    }
    scores[f] = 100 * (mx + mn - scores[f]) / mx;
  }
}

/* Reserve: the placed pod is one more pod on the node for every table
 * constraint whose namespace and selector match it (NodeInfo.AddPod). */
void orc_pts_commit(orc_state *st, const koordhip_pod_ext *x, int32_t i) {
  if (!x || !st->pts_cnt) return;
  for (int c = 0; c < st->soa->pts_cons; c++)
    if ((x->pts_match >> c) & 1u) st->pts_cnt[(size_t)c * st->n + i] += 1;
}
