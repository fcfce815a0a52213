/* TEST INFRASTRUCTURE: CPU restatement of upstream InterPodAffinity
 * (k8s.io/kubernetes v1.24.15 pkg/scheduler/framework/plugins/interpodaffinity,
 * go.mod:57,275 of the reference; the module is not vendored, so parity with
 * upstream is UNPINNED: the rules follow the published sources as cited per
 * function, restated over the engine's count entries; oracle/ipa_upstream.py
 * restates them over objects and checks this file on small cases).  It is the
 * checker of the sequential cycle (csrc/seq.hip), never the thing measured.
 *
 * Columns (include/koordhip.h): pts_dom [keys][n] (the topology keys shared with
 * PodTopologySpread), ipa_cnt [ents][n] (the node's pods entry e counts),
 * ipa_ent_key[e]; per pod the koordhip_pod_ext.ipa_* masks and weights.  The
 * pair maps below are keyed by (topology key, domain) as upstream's
 * topologyPair maps are.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "koord_oracle.h"

static int32_t ipa_dsize(const orc_state *st, int k) {
  return ((st->soa->pts_hostname >> k) & 1u) ? st->n : st->soa->pts_ndom[k];
}
static int32_t ipa_dom(const orc_state *st, int k, int32_t i) { return st->soa->pts_dom[(size_t)k * st->n + i]; }

int orc_ipa_active(const koordhip_config *cfg, const orc_state *st, const koordhip_pod_ext *x) {
  return ((cfg->filter_plugins | cfg->score_plugins) & KOORDHIP_PLUGIN_IPA) && st->soa->ipa_ents > 0 &&
         st->soa->pts_keys > 0 && x != NULL;
}

void orc_ipa_free(orc_ipa *ia) {
  for (int k = 0; k < KOORDHIP_PTS_KEYS; k++) {
    free(ia->aff[k]);
    free(ia->anti[k]);
    free(ia->score[k]);
  }
  memset(ia, 0, sizeof(*ia));
}

static int64_t *ipa_map(const orc_state *st, int k, int64_t **slot) {
  if (!*slot) {
    const int32_t D = ipa_dsize(st, k);
    *slot = (int64_t *)calloc((size_t)(D > 0 ? D : 1), sizeof(int64_t));
  }
  return *slot;
}

/* Add entry e's per-node counts (times w) into the pair map of its key over
 * every node carrying the key (topologyToMatchedTermCount.update /
 * scoreMap.processTerm: a node without the key label adds nothing). */
static int ipa_accumulate(const orc_state *st, int e, int64_t w, int64_t **maps) {
  const int k = st->soa->ipa_ent_key[e];
  int64_t *m = ipa_map(st, k, &maps[k]);
  if (!m) return -1;
  for (int32_t i = 0; i < st->n; i++) {
    const int32_t d = ipa_dom(st, k, i);
    if (d >= 0) m[d] += w * st->ipa_cnt[(size_t)e * st->n + i];
  }
  return 0;
}

/* PreFilter, filtering.go: affinityCounts over the pod's required affinity
 * terms (existing pods matching ALL of them, podMatchesAllAffinityTerms),
 * antiAffinityCounts over its anti-affinity terms and
 * existingAntiAffinityCounts over the running pods' anti-affinity terms that
 * match it -- the last two are checked alike, so one map holds both. */
int orc_ipa_prefilter(const koordhip_config *cfg, const orc_state *st, const koordhip_pod_ext *x, orc_ipa *ia) {
  memset(ia, 0, sizeof(*ia));
  if (!orc_ipa_active(cfg, st, x)) return 0;
  ia->on = 1;
  if (!(cfg->filter_plugins & KOORDHIP_PLUGIN_IPA)) return 0;
  ia->filt = 1;
  for (int e = 0; e < st->soa->ipa_ents; e++) {
    if (((x->ipa_aff >> e) & 1u) && ipa_accumulate(st, e, 1, ia->aff)) return -1;
    if (((x->ipa_anti >> e) & 1u) && ipa_accumulate(st, e, 1, ia->anti)) return -1;
  }
  /* len(affinityCounts) == 0: no pair with a nonzero count (update deletes pairs at 0) */
  ia->aff_empty = 1;
  for (int k = 0; k < KOORDHIP_PTS_KEYS; k++)
    if (ia->aff[k])
      for (int32_t d = 0; d < ipa_dsize(st, k); d++)
        if (ia->aff[k][d] != 0) ia->aff_empty = 0;
  return 0;
}

/* Filter, filtering.go: satisfyPodAffinity (every term's key on the node and
 * its pair counted, or -- no pair counted anywhere and the pod matching its own
 * terms -- the first pod of a series), satisfyPodAntiAffinity and
 * satisfyExistingPodsAntiAffinity (a counted pair at the node's value).  1 = passes. */
int orc_ipa_filter(const orc_state *st, const koordhip_pod_ext *x, const orc_ipa *ia, int32_t i) {
  if (!ia || !ia->on || !ia->filt) return 1;
  if (x->ipa_aff) {
    int pods_exist = 1;
    for (int e = 0; e < st->soa->ipa_ents; e++) {
      if (!((x->ipa_aff >> e) & 1u)) continue;
      const int k = st->soa->ipa_ent_key[e];
      const int32_t d = ipa_dom(st, k, i);
      if (d < 0) return 0; /* all topology labels must exist on the node */
      if (ia->aff[k][d] <= 0) pods_exist = 0;
    }
    if (!pods_exist && !(ia->aff_empty && (x->ipa_flags & KOORDHIP_IPA_SELF))) return 0;
  }
  for (int k = 0; k < KOORDHIP_PTS_KEYS; k++) {
    if (!ia->anti[k]) continue;
    const int32_t d = ipa_dom(st, k, i);
    if (d >= 0 && ia->anti[k][d] > 0) return 0;
  }
  return 1;
}

/* PreScore, scoring.go: topologyScore[key][value] += weight x multiplier for
 * every (existing pod, term) pair processExistingPod credits -- the pod's
 * preferred terms matching an existing pod, and the existing pods' required
 * affinity (hardPodAffinityWeight) / preferred terms matching the pod; the
 * host folded each kind into entry weights ipa_w[e]. */
int orc_ipa_prescore(const orc_state *st, const koordhip_pod_ext *x, orc_ipa *ia) {
  if (!ia || !ia->on) return 0;
  ia->scored = 1;
  for (int e = 0; e < st->soa->ipa_ents; e++)
    if (((x->ipa_score >> e) & 1u) && x->ipa_w[e] != 0 && ipa_accumulate(st, e, x->ipa_w[e], ia->score)) return -1;
  return 0;
}

/* Score, scoring.go: the sum over topologyScore's keys of the node's pair value. */
int64_t orc_ipa_score(const orc_state *st, const orc_ipa *ia, int32_t i) {
  if (!ia || !ia->scored) return 0;
  int64_t s = 0;
  for (int k = 0; k < KOORDHIP_PTS_KEYS; k++) {
    if (!ia->score[k]) continue;
    const int32_t d = ipa_dom(st, k, i);
    if (d >= 0) s += ia->score[k][d];
  }
  return s;
}

/* NormalizeScore, scoring.go: MaxNodeScore x (s - min) / (max - min) in
 * float64, truncated; 0 when max == min.  (With an empty topologyScore every
 * raw score is 0 and upstream leaves them: the same 0.) */
void orc_ipa_normalize(int64_t *scores, int32_t nf) {
  int64_t mn = INT64_MAX, mx = INT64_MIN;
  for (int32_t j = 0; j < nf; j++) {
    if (scores[j] > mx) mx = scores[j];
    if (scores[j] < mn) mn = scores[j];
  }
  const int64_t diff = mx - mn;
  for (int32_t j = 0; j < nf; j++) {
    double f = 0.0;
    if (diff > 0) f = 100.0 * ((double)(scores[j] - mn) / (double)diff);
    scores[j] = (int64_t)f;
  }
}

/* Reserve (NodeInfo.AddPod): the placed pod counts in every entry it matches
 * or carries. */
void orc_ipa_commit(orc_state *st, const koordhip_pod_ext *x, int32_t i) {
  if (!x || !st->ipa_cnt) return;
  for (int e = 0; e < st->soa->ipa_ents; e++)
    if ((x->ipa_inc >> e) & 1u) st->ipa_cnt[(size_t)e * st->n + i] += 1;
}
