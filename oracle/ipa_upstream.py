"""TEST INFRASTRUCTURE: a literal Python restatement of upstream
InterPodAffinity (k8s.io/kubernetes v1.24.15 pkg/scheduler/framework/plugins/
interpodaffinity, go.mod:57,275 of the reference; not vendored, so parity
with upstream is UNPINNED -- this follows the published sources function by
function) over Kubernetes objects, the checker of the host's count entries
(koordinator_amd/interpodaffinity.py) and of the C oracle (ipa_oracle.c) on
small cases.  Nothing in the product imports it.

Maps are keyed by topologyPair (key, value) exactly as upstream."""
from __future__ import annotations

import math
from typing import Dict, List

from koordinator_amd.interpodaffinity import affinity_term


def _terms(pod):
    ra = [affinity_term(pod, t) for t in (pod.pod_affinity_required or [])]
    rn = [affinity_term(pod, t) for t in (pod.pod_anti_affinity_required or [])]
    pa = [(w.weight, affinity_term(pod, w.term)) for w in (pod.pod_affinity_preferred or [])]
    pn = [(w.weight, affinity_term(pod, w.term)) for w in (pod.pod_anti_affinity_preferred or [])]
    return ra, rn, pa, pn


def _update(m: Dict, node, key: str, value: int):
    """topologyToMatchedTermCount.update (filtering.go)."""
    tv = (node.labels or {}).get(key)
    if tv is not None:
        pair = (key, tv)
        m[pair] = m.get(pair, 0) + value
        if m[pair] == 0:
            del m[pair]


def _matches_all(terms, pod, ns_labels) -> bool:
    """podMatchesAllAffinityTerms."""
    if not terms:
        return False
    return all(t.matches(pod, ns_labels) for t in terms)


def prefilter(pod, nodes, node_pods, ns_labels):
    """PreFilter: getExistingAntiAffinityCounts + getIncomingAffinityAntiAffinityCounts."""
    ra, rn, _, _ = _terms(pod)
    existing_anti, aff, anti = {}, {}, {}
    for node in nodes:
        for ep in node_pods.get(node.name, []):
            _, ern, _, _ = _terms(ep)
            for t in ern:                                  # existing pods' required anti-affinity
                if t.matches(pod, ns_labels):
                    _update(existing_anti, node, t.topology_key, 1)
            if _matches_all(ra, ep, ns_labels):            # updateWithAffinityTerms
                for t in ra:
                    _update(aff, node, t.topology_key, 1)
            for t in rn:                                   # updateWithAntiAffinityTerms
                if t.matches(ep, ns_labels):
                    _update(anti, node, t.topology_key, 1)
    return {"ra": ra, "rn": rn, "existing_anti": existing_anti, "aff": aff, "anti": anti, "pod": pod}


def filter_node(state, node, ns_labels) -> bool:
    """Filter: satisfyPodAffinity, satisfyPodAntiAffinity, satisfyExistingPodsAntiAffinity."""
    labels = node.labels or {}
    pods_exist = True
    for t in state["ra"]:
        v = labels.get(t.topology_key)
        if v is None:
            return False
        if state["aff"].get((t.topology_key, v), 0) <= 0:
            pods_exist = False
    if not pods_exist:
        if not (len(state["aff"]) == 0 and _matches_all(state["ra"], state["pod"], ns_labels)):
            return False
    for t in state["rn"]:
        v = labels.get(t.topology_key)
        if v is not None and state["anti"].get((t.topology_key, v), 0) > 0:
            return False
    if state["existing_anti"]:
        for k, v in labels.items():
            if state["existing_anti"].get((k, v), 0) > 0:
                return False
    return True


def prescore(pod, nodes, node_pods, ns_labels, hard_weight: int = 1) -> Dict[str, Dict[str, int]]:
    """PreScore: topologyScore over every node's pods (processExistingPod)."""
    _, _, pa, pn = _terms(pod)
    score: Dict[str, Dict[str, int]] = {}

    def process_term(t, weight, target, node, mult):
        if t.matches(target, ns_labels):
            v = (node.labels or {}).get(t.topology_key)
            if v is not None:
                score.setdefault(t.topology_key, {})
                score[t.topology_key][v] = score[t.topology_key].get(v, 0) + weight * mult

    for node in nodes:
        for ep in node_pods.get(node.name, []):
            era, _, epa, epn = _terms(ep)
            for w, t in pa:
                process_term(t, w, ep, node, 1)
            for w, t in pn:
                process_term(t, w, ep, node, -1)
            if hard_weight > 0 and node.labels:
                for t in era:
                    process_term(t, hard_weight, pod, node, 1)
            for w, t in epa:
                process_term(t, w, pod, node, 1)
            for w, t in epn:
                process_term(t, w, pod, node, -1)
    return score


def score_node(topology_score, node) -> int:
    s = 0
    labels = node.labels or {}
    for k, vals in topology_score.items():
        v = labels.get(k)
        if v is not None:
            s += vals.get(v, 0)
    return s


def normalize(topology_score, scores: List[int]) -> List[int]:
    """NormalizeScore: min-max to [0, 100] with float64, truncated."""
    if not topology_score:
        return list(scores)
    mn, mx = min(scores), max(scores)
    d = mx - mn
    return [int(100.0 * (float(s - mn) / float(d))) if d > 0 else 0 for s in scores]


def evaluate(pod, nodes, node_pods, ns_labels=None, hard_weight: int = 1):
    """(feasible node indices, raw score per node, normalized score per feasible node)."""
    ns_labels = ns_labels or {}
    st = prefilter(pod, nodes, node_pods, ns_labels)
    feas = [i for i, nd in enumerate(nodes) if filter_node(st, nd, ns_labels)]
    ts = prescore(pod, nodes, node_pods, ns_labels, hard_weight)
    raw = [score_node(ts, nd) for nd in nodes]
    norm = normalize(ts, [raw[i] for i in feas]) if feas else []
    return feas, raw, dict(zip(feas, norm))


def place_stream(pods, nodes, node_pods, ns_labels=None, hard_weight: int = 1, weight: int = 1):
    """The cycle with InterPodAffinity alone: argmax of the normalized score over
    the feasible nodes (lowest index on ties), then the pod runs there."""
    node_pods = {k: list(v) for k, v in node_pods.items()}
    out = []
    for p in pods:
        feas, raw, norm = evaluate(p, nodes, node_pods, ns_labels, hard_weight)
        if not feas:
            out.append(-1)
            continue
        best = max(feas, key=lambda i: (weight * norm[i], -i))
        out.append(best)
        node_pods.setdefault(nodes[best].name, []).append(p)
    return out, node_pods
