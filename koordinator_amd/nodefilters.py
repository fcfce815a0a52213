"""The upstream static node filters of a koord-scheduler profile, resolved on
the host per (pod static class, node) into the snapshot's `static_allow`
column, and the raw Scores of NodeAffinity
(preferred terms) and TaintToleration (PreferNoSchedule) per (class, node)
into `static_score` (normalized over the feasible nodes on the device, in the
sequential cycle).

NodeUnschedulable, NodeName, NodeAffinity (required part) and TaintToleration
(Filter) read only the node's name, labels, taints and spec.unschedulable and
the pod's spec.nodeName, nodeSelector, required node affinity and tolerations
-- nothing a Reserve changes.  Pods sharing those fields form one static class; a node's
`static_allow` bit c says whether class c passes all enabled filters there, so
the device Filter is one bit test per (pod, node).

Restated from k8s v1.24.15 (go.mod:57,275), which is not vendored in the
reference: parity with upstream is unpinned by reference tests; the rules
follow the published plugin sources as cited per function.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np

from . import abi
from .config import PLUGIN_NODE_AFFINITY, PLUGIN_NODE_NAME, PLUGIN_NODE_UNSCHEDULABLE, PLUGIN_TAINT_TOLERATION
from .reservation import NodeSelectorRequirement, NodeSelectorTerm, _req_matches

NO_SCHEDULE, PREFER_NO_SCHEDULE, NO_EXECUTE = "NoSchedule", "PreferNoSchedule", "NoExecute"
TAINT_NODE_UNSCHEDULABLE = "node.kubernetes.io/unschedulable"


@dataclass(frozen=True)
class Taint:
    key: str
    value: str = ""
    effect: str = NO_SCHEDULE


@dataclass(frozen=True)
class Toleration:
    key: str = ""
    operator: str = ""      # "" = Equal, "Exists"
    value: str = ""
    effect: str = ""        # "" = every effect

    def tolerates(self, t: Taint) -> bool:
        """(upstream) api/core/v1 Toleration.ToleratesTaint."""
        if self.effect and self.effect != t.effect:
            return False
        if self.key and self.key != t.key:
            return False
        if self.operator in ("", "Equal"):
            return self.value == t.value
        return self.operator == "Exists"


@dataclass
class NodeStatic:
    """The node fields the static filters read."""
    labels: Dict[str, str] = field(default_factory=dict)
    taints: List[Taint] = field(default_factory=list)
    unschedulable: bool = False
    name: str = ""


@dataclass
class PodStatic:
    """The pod fields the static filters read (its static class key)."""
    node_selector: Dict[str, str] = field(default_factory=dict)
    required_terms: Optional[List[NodeSelectorTerm]] = None   # requiredDuringSchedulingIgnoredDuringExecution
    tolerations: List[Toleration] = field(default_factory=list)
    # preferredDuringSchedulingIgnoredDuringExecution: (weight, NodeSelectorTerm)
    preferred_terms: List[Tuple[int, NodeSelectorTerm]] = field(default_factory=list)
    node_name: str = ""                                       # spec.nodeName

    def key(self) -> Tuple:
        tk = lambda t: (tuple((r.key, r.operator, tuple(r.values)) for r in t.match_expressions),
                        tuple((r.key, r.operator, tuple(r.values)) for r in t.match_fields))
        terms = None if self.required_terms is None else tuple(tk(t) for t in self.required_terms)
        pref = tuple((int(w), tk(t)) for w, t in self.preferred_terms)
        return (tuple(sorted(self.node_selector.items())), terms, tuple(self.tolerations), pref, self.node_name)


def tolerates_all(tolerations: Sequence[Toleration], taints: Iterable[Taint], effects) -> bool:
    """(upstream) v1helper.FindMatchingUntoleratedTaint with a filter on the
    taint effect: True when every taint of those effects is tolerated."""
    return all(any(tol.tolerates(t) for tol in tolerations) for t in taints if t.effect in effects)


def node_unschedulable_ok(pod: PodStatic, node: NodeStatic) -> bool:
    """(upstream) nodeunschedulable/node_unschedulable.go Filter: a node with
    spec.unschedulable takes only pods tolerating the
    node.kubernetes.io/unschedulable:NoSchedule taint."""
    if not node.unschedulable:
        return True
    return any(tol.tolerates(Taint(TAINT_NODE_UNSCHEDULABLE, "", NO_SCHEDULE)) for tol in pod.tolerations)


def node_name_ok(pod: PodStatic, node: NodeStatic) -> bool:
    """(upstream) nodename/node_name.go Fits: no spec.nodeName, or the node's name."""
    return not pod.node_name or pod.node_name == node.name


def _term_matches(t: NodeSelectorTerm, node: NodeStatic) -> bool:
    """(upstream) component-helpers nodeSelectorTerm.match: expressions on the
    labels and fields (metadata.name) all match; an empty term matches nothing."""
    if not t.match_expressions and not t.match_fields:
        return False
    return all(_req_matches(r, node.labels) for r in t.match_expressions) and \
        all(_req_matches(r, {"metadata.name": node.name}) for r in t.match_fields)


def node_affinity_ok(pod: PodStatic, node: NodeStatic) -> bool:
    """(upstream) nodeaffinity/node_affinity.go Filter with
    component-helpers RequiredNodeAffinity.Match: every nodeSelector label,
    and, when required terms are set, at least one term whose expressions (on
    labels) and fields (metadata.name) all match; a term with neither matches
    nothing, an empty term list matches no node."""
    for k, v in pod.node_selector.items():
        if node.labels.get(k) != v:
            return False
    if pod.required_terms is None:
        return True
    return any(_term_matches(t, node) for t in pod.required_terms)


def taint_toleration_ok(pod: PodStatic, node: NodeStatic) -> bool:
    """(upstream) tainttoleration/taint_toleration.go Filter: every NoSchedule
    / NoExecute taint of the node is tolerated (PreferNoSchedule is Score-only)."""
    return tolerates_all(pod.tolerations, node.taints, (NO_SCHEDULE, NO_EXECUTE))


def node_affinity_score(pod: PodStatic, node: NodeStatic) -> int:
    """(upstream) nodeaffinity/node_affinity.go Score with component-helpers
    PreferredSchedulingTerms.Score: the sum of the weights of the preferred
    terms the node matches (weight-0 terms dropped).  NormalizeScore:
    DefaultNormalizeScore(100, reverse=false) over the feasible nodes."""
    return sum(int(w) for w, t in pod.preferred_terms if w and _term_matches(t, node))


def taint_toleration_score(pod: PodStatic, node: NodeStatic) -> int:
    """(upstream) tainttoleration/taint_toleration.go Score,
    countIntolerableTaintsPreferNoSchedule: the node's PreferNoSchedule taints
    no toleration of effect "" / PreferNoSchedule tolerates
    (getAllTolerationPreferNoSchedule).  NormalizeScore: DefaultNormalizeScore
    (100, reverse=true)."""
    tols = [t for t in pod.tolerations if t.effect in ("", PREFER_NO_SCHEDULE)]
    return sum(1 for t in node.taints if t.effect == PREFER_NO_SCHEDULE and not any(x.tolerates(t) for x in tols))


_CHECKS = {PLUGIN_NODE_UNSCHEDULABLE: node_unschedulable_ok, PLUGIN_NODE_NAME: node_name_ok,
           PLUGIN_NODE_AFFINITY: node_affinity_ok, PLUGIN_TAINT_TOLERATION: taint_toleration_ok}


class StaticClasses:
    """Distinct pod static specs -> class index (at most MAX_STATIC_CLASSES)."""

    def __init__(self):
        self.specs: List[PodStatic] = []
        self._index: Dict[Tuple, int] = {}
        self.frozen = abi.MAX_STATIC_CLASSES   # classes with node bits on the device (set by marshal.build_table)

    def classify(self, pod: PodStatic) -> int:
        k = pod.key()
        c = self._index.get(k)
        if c is None:
            if len(self.specs) >= abi.MAX_STATIC_CLASSES:
                raise ValueError(f"more than {abi.MAX_STATIC_CLASSES} distinct pod static classes")
            c = len(self.specs)
            self.specs.append(pod)
            self._index[k] = c
        return c


def static_allow(nodes: Sequence[NodeStatic], classes: StaticClasses, filters: Iterable[str]) -> np.ndarray:
    """The static_allow column: bit c of row i = class c passes every enabled
    static filter on node i (bits of unused classes set)."""
    checks = [_CHECKS[f] for f in filters if f in _CHECKS]
    out = np.full(len(nodes), 0xFFFFFFFF, dtype=np.uint32)
    for i, nd in enumerate(nodes):
        m = 0xFFFFFFFF
        for c, spec in enumerate(classes.specs):
            if not all(ck(spec, nd) for ck in checks):
                m &= ~(1 << c)
        out[i] = m & 0xFFFFFFFF
    return out


def node_static_ok(pod: PodStatic, node: NodeStatic, filters: Iterable[str]) -> bool:
    """Direct per-(pod, node) evaluation (the test's reference for static_allow)."""
    return all(_CHECKS[f](pod, node) for f in filters if f in _CHECKS)


def static_scores(nodes: Sequence[NodeStatic], classes: StaticClasses) -> np.ndarray:
    """The static_score column [n][2][MAX_STATIC_CLASSES] u16: plane 0 the
    NodeAffinity raw Score, plane 1 the TaintToleration raw Score of each
    class on each node (unused classes 0)."""
    out = np.zeros((len(nodes), 2, abi.MAX_STATIC_CLASSES), np.uint16)
    for i, nd in enumerate(nodes):
        for c, spec in enumerate(classes.specs):
            a, b = node_affinity_score(spec, nd), taint_toleration_score(spec, nd)
            if a > 0xFFFF or b > 0xFFFF:
                raise ValueError("a raw NodeAffinity / TaintToleration Score above 65535")
            out[i, 0, c], out[i, 1, c] = a, b
    return out
