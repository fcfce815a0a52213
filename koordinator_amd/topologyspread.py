"""PodTopologySpread on the host: the pods' spec.topologySpreadConstraints
turned into the engine's tables.

Upstream k8s v1.24.15 pkg/scheduler/framework/plugins/podtopologyspread
(go.mod:57,275 of the reference; not vendored, so parity with upstream is
UNPINNED and the rules follow the published sources):

  filtering.go   PreFilter / Filter over the DoNotSchedule constraints
  scoring.go     PreScore / Score / NormalizeScore over the ScheduleAnyway ones
  common.go      filterTopologySpreadConstraints, nodeLabelsMatchSpreadConstraints,
                 countPodsMatchSelector

The per-pod cycle runs on the device (csrc/seq.hip) and in the oracle
(oracle/pts_oracle.c); this module builds what they read:

  keys        the distinct topology keys of the constraints (<= PTS_KEYS); a
              kubernetes.io/hostname key's domain is the node itself
  cons        the distinct (label selector, namespace) pairs (<= PTS_CONS):
              pts_cnt[c][node] = countPodsMatchSelector(node's pods, selector, ns)
  classes     (required node affinity, DoNotSchedule keys, ScheduleAnyway keys)
              (<= PTS_CLASSES): pts_elig bit 2s / 2s+1 = the node matches the
              class's affinity and carries every hard / soft key

Only explicit constraints are taken: the system-default constraints
(buildDefaultConstraints) need the pod's Service / ReplicaSet / StatefulSet
selectors, which the shim would pass as explicit constraints.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import abi

HOSTNAME = "kubernetes.io/hostname"
DO_NOT_SCHEDULE, SCHEDULE_ANYWAY = "DoNotSchedule", "ScheduleAnyway"


class SpreadError(ValueError):
    """A constraint set outside the engine's envelope (keys, domains, table sizes)."""


@dataclass(frozen=True)
class LabelRequirement:
    key: str
    operator: str                  # In, NotIn, Exists, DoesNotExist
    values: Tuple[str, ...] = ()


@dataclass(frozen=True)
class LabelSelector:
    """metav1.LabelSelector: matchLabels AND matchExpressions (an empty selector matches every pod)."""
    match_labels: Tuple[Tuple[str, str], ...] = ()
    match_expressions: Tuple[LabelRequirement, ...] = ()

    @staticmethod
    def of(labels: Dict[str, str] = None, exprs: Sequence[LabelRequirement] = ()) -> "LabelSelector":
        return LabelSelector(tuple(sorted((labels or {}).items())), tuple(exprs))

    def matches(self, labels: Dict[str, str]) -> bool:
        """(upstream) labels.Selector.Matches of metav1.LabelSelectorAsSelector."""
        labels = labels or {}
        for k, v in self.match_labels:
            if labels.get(k) != v:
                return False
        for r in self.match_expressions:
            has = r.key in labels
            if r.operator == "In":
                ok = has and labels[r.key] in r.values
            elif r.operator == "NotIn":
                ok = not has or labels[r.key] not in r.values
            elif r.operator == "Exists":
                ok = has
            elif r.operator == "DoesNotExist":
                ok = not has
            else:
                raise SpreadError(f"label selector operator {r.operator!r}")
            if not ok:
                return False
        return True


@dataclass(frozen=True)
class TopologySpreadConstraint:
    """v1.TopologySpreadConstraint (minDomains / nodeAffinityPolicy / nodeTaintsPolicy are later than v1.24)."""
    max_skew: int
    topology_key: str
    when_unsatisfiable: str = DO_NOT_SCHEDULE
    label_selector: Optional[LabelSelector] = None   # None: labels.Nothing()

    def selector_matches(self, labels: Dict[str, str]) -> bool:
        return self.label_selector is not None and self.label_selector.matches(labels)


def _affinity_key(pod) -> Tuple:
    from .nodefilters import PodStatic
    ps = PodStatic(node_selector=dict(pod.node_selector or {}), required_terms=pod.required_node_affinity)
    return ps.key()[:2]


class SpreadRegistry:
    """The snapshot's keys, constraint table and spread classes, registered from
    the pods to schedule (like nodefilters.StaticClasses: a snapshot covers the
    registry as it was when built; a pod that needs more asks for a rebuild)."""

    def __init__(self):
        self.keys: List[str] = []
        self.cons: List[Tuple[Optional[LabelSelector], str, int]] = []   # (selector, namespace, key index)
        self.classes: List[Tuple[Tuple, int, int]] = []                 # (affinity key, hard key mask, soft key mask)
        self.class_affinity: List = []                                  # a pod of the class (its affinity)
        self.frozen = None                                              # (keys, cons, classes) covered by the snapshot
        self.domains: Optional["DomainIndex"] = None                    # the snapshot's label value -> domain maps

    def _key(self, k: str) -> int:
        if k not in self.keys:
            if len(self.keys) >= abi.PTS_KEYS:
                raise SpreadError(f"more than {abi.PTS_KEYS} distinct topology keys")
            self.keys.append(k)
        return self.keys.index(k)

    def _cons(self, sel, ns: str, k: int) -> int:
        e = (sel, ns, k)
        if e not in self.cons:
            if len(self.cons) >= abi.PTS_CONS:
                raise SpreadError(f"more than {abi.PTS_CONS} distinct (selector, namespace, key) constraints")
            self.cons.append(e)
        return self.cons.index(e)

    def register(self, pod):
        """(class, [(cons, flags, max_skew)]) of the pod; None when it has no constraints."""
        cs = list(getattr(pod, "topology_spread_constraints", None) or [])
        if not cs:
            return None
        if len(cs) > abi.PTS_POD:
            raise SpreadError(f"pod {pod.key}: more than {abi.PTS_POD} topology spread constraints")
        hard = soft = 0
        out = []
        for c in cs:
            if c.max_skew <= 0:
                raise SpreadError(f"pod {pod.key}: maxSkew must be positive")
            if c.when_unsatisfiable not in (DO_NOT_SCHEDULE, SCHEDULE_ANYWAY):
                raise SpreadError(f"pod {pod.key}: whenUnsatisfiable {c.when_unsatisfiable!r}")
            k = self._key(c.topology_key)
            ci = self._cons(c.label_selector, pod.namespace, k)
            fl = (abi.PTS_HARD if c.when_unsatisfiable == DO_NOT_SCHEDULE else 0) | \
                (abi.PTS_SELF if c.selector_matches(pod.labels) else 0)
            if fl & abi.PTS_HARD:
                hard |= 1 << k
            else:
                soft |= 1 << k
            out.append((ci, fl, int(c.max_skew)))
        ck = (_affinity_key(pod), hard, soft)
        if ck not in self.classes:
            if len(self.classes) >= abi.PTS_CLASSES:
                raise SpreadError(f"more than {abi.PTS_CLASSES} spread classes")
            self.classes.append(ck)
            self.class_affinity.append(pod)
        return self.classes.index(ck), out

    def freeze(self):
        self.frozen = (len(self.keys), len(self.cons), len(self.classes))

    def covers(self, pod) -> bool:
        """The pod's keys, constraints and class were in the registry when the snapshot was built."""
        r = self.register(pod)                      # (registered either way: the next snapshot covers it)
        if r is None:
            return True
        if self.frozen is None:
            return False
        nk, nc, ns = self.frozen
        cls, items = r
        return cls < ns and all(c < nc for c, _, _ in items) and \
            all(self.cons[c][2] < nk for c, _, _ in items)

    def match_mask(self, pod) -> int:
        """Bit c: table constraint c counts the pod (its namespace, its selector) once it is placed."""
        m = 0
        for c, (sel, ns, _) in enumerate(self.cons):
            if ns == pod.namespace and sel is not None and sel.matches(pod.labels):
                m |= 1 << c
        return m


def registry_for(pods) -> SpreadRegistry:
    """A registry holding the spread constraints of `pods` (the pods a snapshot
    will schedule): set it as ClusterState.spread before marshal.build_table."""
    reg = SpreadRegistry()
    for p in pods:
        reg.register(p)
    return reg


def pod_pts_fields(rec, pod, reg: SpreadRegistry):
    """Fill the pts_* fields of one koordhip_pod_ext record."""
    rec["pts_n"] = 0
    rec["pts_class"] = 0
    rec["pts_match"] = reg.match_mask(pod)
    rec["pts_c"][:] = 0
    rec["pts_fl"][:] = 0
    rec["pts_skew"][:] = 0
    r = reg.register(pod)
    if r is None:
        return rec
    cls, items = r
    rec["pts_n"] = len(items)
    rec["pts_class"] = cls
    for j, (c, fl, sk) in enumerate(items):
        rec["pts_c"][j] = c
        rec["pts_fl"][j] = fl
        rec["pts_skew"][j] = sk
    return rec


class DomainIndex:
    """Per topology key, label value -> domain index (first-seen node order)."""

    def __init__(self, reg: SpreadRegistry):
        self.reg = reg
        self.values: List[Dict[str, int]] = [dict() for _ in reg.keys]

    def build(self, nodes) -> np.ndarray:
        """pts_dom [keys][n] for the nodes."""
        n = len(nodes)
        dom = np.full((len(self.reg.keys), n), -1, np.int32)
        for k, key in enumerate(self.reg.keys):
            if key == HOSTNAME:
                seen = set()
                for i, nd in enumerate(nodes):
                    v = (nd.labels or {}).get(HOSTNAME)
                    if v is None:
                        continue
                    if v in seen:
                        raise SpreadError(f"two nodes share {HOSTNAME}={v!r} (the engine's hostname domain is the node)")
                    seen.add(v)
                    dom[k, i] = i
                continue
            vals = self.values[k]
            for i, nd in enumerate(nodes):
                v = (nd.labels or {}).get(key)
                if v is None:
                    continue
                if v not in vals:
                    if len(vals) >= abi.PTS_DOMAINS:
                        raise SpreadError(f"more than {abi.PTS_DOMAINS} values of topology key {key!r}")
                    vals[v] = len(vals)
                dom[k, i] = vals[v]
        return dom


def node_pts(reg: SpreadRegistry, node, pods_on_node) -> Tuple[np.ndarray, int]:
    """(pts_cnt column values [cons], pts_elig bits) of one node."""
    from .nodefilters import NodeStatic, PodStatic, node_affinity_ok
    cnt = np.zeros(abi.PTS_CONS, np.int32)
    for c, (sel, ns, _) in enumerate(reg.cons):
        if sel is None:
            continue
        cnt[c] = sum(1 for p in pods_on_node if p.namespace == ns and sel.matches(p.labels))
    labels = node.labels or {}
    ns_ = NodeStatic(labels=dict(labels), name=node.name)
    elig = 0
    for s, (_, hard, soft) in enumerate(reg.classes):
        pod = reg.class_affinity[s]
        aff = node_affinity_ok(PodStatic(node_selector=dict(pod.node_selector or {}),
                                         required_terms=pod.required_node_affinity), ns_)
        has = lambda mask: all(reg.keys[k] in labels for k in range(len(reg.keys)) if (mask >> k) & 1)
        if aff and has(hard):
            elig |= 1 << (2 * s)
        if aff and has(soft):
            elig |= 1 << (2 * s + 1)
    return cnt, elig
