"""InterPodAffinity on the host: the pods' spec.affinity.podAffinity /
podAntiAffinity turned into the engine's count entries (SURVEY.md section
8(f)#4).

Upstream k8s v1.24.15 pkg/scheduler/framework/plugins/interpodaffinity
(go.mod:57,275 of the reference; not vendored, so parity with upstream is
UNPINNED and the rules follow the published sources; oracle/ipa_upstream.py
restates them literally over objects as the test checker):

  filtering.go  PreFilter (existingAntiAffinityCounts, affinityCounts,
                antiAffinityCounts over (topology key, value) pairs) and Filter
                (satisfyExistingPodsAntiAffinity, satisfyPodAntiAffinity,
                satisfyPodAffinity with the first-pod-of-a-series exception)
  scoring.go    PreScore (topologyScore from the pod's preferred terms and the
                existing pods' required affinity (hardPodAffinityWeight) and
                preferred terms), Score, NormalizeScore (min-max)
  framework/types.go  AffinityTerm.Matches, newAffinityTerm (an empty namespace
                list and no namespaceSelector: the term owner's namespace)

Every one of those counts is a sum, over the nodes holding a (key, value)
pair, of per-node pod counts of one kind.  The engine keeps those per-node
counts as *count entries* (ipa_cnt [ents][n]) on the topology keys the
PodTopologySpread tables define (pts_dom), and each pod says in its
koordhip_pod_ext which entries its Filter and Score read:

  ("M", terms, key)              the pods that match every term (one term for
                                 a pod's anti-affinity / preferred terms, all of
                                 its required affinity terms for affinityCounts)
  ("C", term, role, weight, key) the pods that carry `term` as a required
                                 anti-affinity ("anti"), required affinity
                                 ("aff", scored with hardPodAffinityWeight) or
                                 preferred term ("pref", +/- weight)

Carried terms are catalogued for every existing pod, but an entry is only made
for a carried term that matches one of the registered pods to schedule (a term
no pending pod matches changes no Filter or Score), which keeps the table
within KOORDHIP_IPA_ENTRIES.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, FrozenSet, List, Optional, Sequence, Tuple

import numpy as np

from . import abi
from .topologyspread import LabelSelector, SpreadRegistry

ROLE_ANTI, ROLE_AFF, ROLE_PREF = "anti", "aff", "pref"


class IpaError(ValueError):
    """Affinity terms outside the engine's envelope."""


@dataclass(frozen=True)
class PodAffinityTerm:
    """v1.PodAffinityTerm.  label_selector None = labels.Nothing();
    namespace_selector None = unset (an empty LabelSelector selects every namespace)."""
    label_selector: Optional[LabelSelector]
    topology_key: str
    namespaces: Tuple[str, ...] = ()
    namespace_selector: Optional[LabelSelector] = None


@dataclass(frozen=True)
class WeightedPodAffinityTerm:
    weight: int
    term: PodAffinityTerm


@dataclass(frozen=True)
class AffinityTerm:
    """framework.AffinityTerm: the term with its namespaces resolved against its owner."""
    selector: Optional[LabelSelector]
    namespaces: FrozenSet[str]
    namespace_selector: Optional[LabelSelector]
    topology_key: str

    def matches(self, pod, ns_labels: Dict[str, Dict[str, str]]) -> bool:
        """AffinityTerm.Matches: the pod's namespace is listed or the namespace
        selector matches its labels, and the label selector matches the pod."""
        if not (pod.namespace in self.namespaces or
                (self.namespace_selector is not None and
                 self.namespace_selector.matches(ns_labels.get(pod.namespace, {})))):
            return False
        return self.selector is not None and self.selector.matches(pod.labels or {})


def affinity_term(owner, t: PodAffinityTerm) -> AffinityTerm:
    """newAffinityTerm / getNamespacesFromPodAffinityTerm."""
    if not t.namespaces and t.namespace_selector is None:
        ns = frozenset((owner.namespace,))
    else:
        ns = frozenset(t.namespaces)
    return AffinityTerm(t.label_selector, ns, t.namespace_selector, t.topology_key)


def pod_terms(pod):
    """(required affinity, required anti-affinity, preferred affinity [(w, term)],
    preferred anti-affinity [(w, term)]) resolved against the pod."""
    ra = [affinity_term(pod, t) for t in (pod.pod_affinity_required or [])]
    rn = [affinity_term(pod, t) for t in (pod.pod_anti_affinity_required or [])]
    pa = [(int(w.weight), affinity_term(pod, w.term)) for w in (pod.pod_affinity_preferred or [])]
    pn = [(int(w.weight), affinity_term(pod, w.term)) for w in (pod.pod_anti_affinity_preferred or [])]
    return ra, rn, pa, pn


def has_terms(pod) -> bool:
    return bool(pod.pod_affinity_required or pod.pod_anti_affinity_required or pod.pod_affinity_preferred
                or pod.pod_anti_affinity_preferred)


def carried(pod, hard_weight: int) -> List[Tuple[AffinityTerm, str, int]]:
    """The (term, role, weight) a pod carries once it runs: the terms other pods'
    Filter (required anti-affinity) and Score (hardPodAffinityWeight x required
    affinity, +/- preferred weights) read (processExistingPod)."""
    ra, rn, pa, pn = pod_terms(pod)
    out = [(t, ROLE_ANTI, 0) for t in rn]
    if hard_weight > 0:
        out += [(t, ROLE_AFF, hard_weight) for t in ra]
    out += [(t, ROLE_PREF, w) for w, t in pa]
    out += [(t, ROLE_PREF, -w) for w, t in pn]
    return out


class IpaRegistry:
    """The snapshot's count entries, built from the pods to schedule and the
    terms the running pods carry (keys shared with the SpreadRegistry)."""

    def __init__(self, topo: SpreadRegistry, ns_labels: Optional[Dict[str, Dict[str, str]]] = None,
                 hard_weight: int = 1):
        self.topo = topo
        self.ns_labels = dict(ns_labels or {})
        self.hard_weight = hard_weight
        self.entries: List[Tuple] = []
        self._index: Dict[Tuple, int] = {}
        self.carriers: Dict[Tuple, None] = {}   # every carried (term, role, weight) seen, in order
        self.incoming: Dict[Tuple, object] = {}  # (namespace, labels) -> a registered pod to schedule
        self.frozen: Optional[int] = None

    def _entry(self, e: Tuple) -> int:
        i = self._index.get(e)
        if i is None:
            if len(self.entries) >= abi.IPA_ENTRIES:
                raise IpaError(f"more than {abi.IPA_ENTRIES} InterPodAffinity count entries")
            i = self._index[e] = len(self.entries)
            self.entries.append(e)
        return i

    def _key(self, k: str) -> int:
        from .topologyspread import SpreadError
        try:
            return self.topo._key(k)
        except SpreadError as ex:
            raise IpaError(str(ex)) from None

    def _carrier_entry(self, c):
        term, role, w = c
        return ("C", term, role, w, self._key(term.topology_key))

    def _add_carrier(self, c):
        """Catalogue a carried term; make its entry if a pod to schedule matches it."""
        if c not in self.carriers:
            self.carriers[c] = None
        if any(c[0].matches(p, self.ns_labels) for p in self.incoming.values()):
            self._entry(self._carrier_entry(c))

    def register_existing(self, pod):
        for c in carried(pod, self.hard_weight):
            self._add_carrier(c)

    def register(self, pod):
        """A pod to schedule: its own terms' entries, the entries of the
        catalogued carried terms that match it, and its carried terms."""
        cls = (pod.namespace, tuple(sorted((pod.labels or {}).items())))
        if cls not in self.incoming:
            self.incoming[cls] = pod
            for c in list(self.carriers):
                if c[0].matches(pod, self.ns_labels):
                    self._entry(self._carrier_entry(c))
        ra, rn, pa, pn = pod_terms(pod)
        if ra:
            conj = tuple(ra)
            for k in dict.fromkeys(t.topology_key for t in ra):
                self._entry(("M", conj, self._key(k)))
        for t in rn:
            self._entry(("M", (t,), self._key(t.topology_key)))
        for _, t in pa + pn:
            self._entry(("M", (t,), self._key(t.topology_key)))
        self.register_existing(pod)

    def freeze(self):
        self.frozen = len(self.entries)

    def covers(self, pod) -> bool:
        """The snapshot (frozen) holds every entry the pod needs."""
        self.register(pod)
        return self.frozen is not None and self.frozen == len(self.entries)

    def ent_keys(self) -> List[int]:
        return [e[-1] if e[0] == "M" else e[4] for e in self.entries]

    # ---- per node / per pod -------------------------------------------------
    def entry_counts(self, pod, out: np.ndarray):
        """Add one pod's contribution to a node's counts (out [IPA_ENTRIES])."""
        car = {}
        for c in carried(pod, self.hard_weight):
            car[c] = car.get(c, 0) + 1
        for e, ent in enumerate(self.entries):
            if ent[0] == "M":
                if all(t.matches(pod, self.ns_labels) for t in ent[1]):
                    out[e] += 1
            else:
                out[e] += car.get(ent[1:4], 0)

    def pod_fields(self, rec, pod):
        """Fill the ipa_* fields of one koordhip_pod_ext record."""
        rec["ipa_inc"] = rec["ipa_aff"] = rec["ipa_anti"] = rec["ipa_score"] = rec["ipa_flags"] = 0
        rec["ipa_w"][:] = 0
        inc = aff = anti = 0
        w = [0] * abi.IPA_ENTRIES
        car = {}
        for c in carried(pod, self.hard_weight):
            car[c] = car.get(c, 0) + 1
        if any(v > 1 for v in car.values()):
            raise IpaError(f"pod {pod.key}: the same affinity term twice")
        ra, rn, pa, pn = pod_terms(pod)
        conj = tuple(ra)
        for e, ent in enumerate(self.entries):
            if ent[0] == "M":
                terms, k = ent[1], ent[2]
                if all(t.matches(pod, self.ns_labels) for t in terms):
                    inc |= 1 << e
                if ra and terms == conj:
                    aff |= 1 << e
                if len(terms) == 1:
                    t = terms[0]
                    if t in rn and t.topology_key == self.topo.keys[k]:
                        anti |= 1 << e
                    for wt, pt in pa:
                        if pt == t:
                            w[e] += wt
                    for wt, pt in pn:
                        if pt == t:
                            w[e] -= wt
            else:
                term, role, weight = ent[1], ent[2], ent[3]
                if (term, role, weight) in car:
                    inc |= 1 << e
                if term.matches(pod, self.ns_labels):
                    if role == ROLE_ANTI:
                        anti |= 1 << e
                    else:
                        w[e] += weight
        if ra and aff == 0:
            raise IpaError(f"pod {pod.key}: its required affinity terms are not in the snapshot: rebuild it")
        rec["ipa_inc"], rec["ipa_aff"], rec["ipa_anti"] = inc, aff, anti
        rec["ipa_flags"] = abi.IPA_SELF if ra and all(t.matches(pod, self.ns_labels) for t in ra) else 0
        sc = 0
        for e in range(abi.IPA_ENTRIES):
            rec["ipa_w"][e] = w[e]
            if w[e]:
                sc |= 1 << e
        rec["ipa_score"] = sc
        return rec


def registry_for(pods, existing=(), topo: Optional[SpreadRegistry] = None, ns_labels=None,
                 hard_weight: int = 1) -> IpaRegistry:
    """A registry for `pods` (to schedule) and the running `existing` pods."""
    reg = IpaRegistry(topo if topo is not None else SpreadRegistry(), ns_labels, hard_weight)
    for p in existing:
        reg.register_existing(p)
    for p in pods:
        reg.register(p)
    return reg


def node_ipa(reg: IpaRegistry, pods_on_node: Sequence) -> np.ndarray:
    """ipa_cnt row of one node."""
    cnt = np.zeros(abi.IPA_ENTRIES, np.int32)
    for p in pods_on_node:
        reg.entry_counts(p, cnt)
    return cnt
