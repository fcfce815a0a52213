"""Upstream default-profile plugins on the host and in the
oracle: the static node filters (NodeUnschedulable, NodeAffinity,
TaintToleration) resolved into static_allow, and
NodeResourcesBalancedAllocation.

The upstream sources (k8s v1.24.15) are not in the container: the rules are
restated from the published plugins and the vectors below are worked from
those rules (the BalancedAllocation ones are the worked examples of upstream
balanced_allocation_test.go's "resources requested" case) -- parity with the
reference's own tests is unpinned."""
import ctypes as C

import numpy as np
import pytest

import oracle
from koordinator_amd import abi, synth
from koordinator_amd.config import (PLUGIN_BALANCED, STATIC_FILTERS, ArgsError, shipped_profile, to_c_config,
                                    with_upstream)
from koordinator_amd.nodefilters import (NO_EXECUTE, NO_SCHEDULE, PREFER_NO_SCHEDULE, NodeStatic, PodStatic,
                                         StaticClasses, Taint, Toleration, node_affinity_ok, node_static_ok,
                                         node_unschedulable_ok, static_allow, taint_toleration_ok)
from koordinator_amd.reservation import NodeSelectorRequirement as R, NodeSelectorTerm as T
from koordinator_amd.snapshot import NodeTable, pod_array


# ------------------------------------------------------------ tolerations
@pytest.mark.parametrize("tol,taint,want", [
    (Toleration("k", "Equal", "v", NO_SCHEDULE), Taint("k", "v", NO_SCHEDULE), True),
    (Toleration("k", "", "v", NO_SCHEDULE), Taint("k", "v", NO_SCHEDULE), True),     # "" = Equal
    (Toleration("k", "Equal", "w", NO_SCHEDULE), Taint("k", "v", NO_SCHEDULE), False),
    (Toleration("k", "Exists", "", NO_SCHEDULE), Taint("k", "v", NO_SCHEDULE), True),
    (Toleration("k", "Exists", "", NO_EXECUTE), Taint("k", "v", NO_SCHEDULE), False),  # effect differs
    (Toleration("k", "Exists", "", ""), Taint("k", "v", NO_EXECUTE), True),           # every effect
    (Toleration("", "Exists", "", ""), Taint("any", "x", NO_SCHEDULE), True),         # tolerates everything
    (Toleration("", "Equal", "", ""), Taint("any", "", NO_SCHEDULE), True),           # empty key, Equal "" == ""
    (Toleration("j", "Exists"), Taint("k", "v", NO_SCHEDULE), False),
    (Toleration("k", "Bogus", "v"), Taint("k", "v", NO_SCHEDULE), False),
])
def test_toleration_tolerates_taint(tol, taint, want):
    assert tol.tolerates(taint) is want


def test_taint_toleration_filter_effects():
    node = NodeStatic(taints=[Taint("a", "1", NO_SCHEDULE), Taint("b", "", PREFER_NO_SCHEDULE)])
    assert not taint_toleration_ok(PodStatic(), node)
    assert taint_toleration_ok(PodStatic(tolerations=[Toleration("a", "Equal", "1")]), node)  # PreferNoSchedule ignored
    node2 = NodeStatic(taints=[Taint("m", "", NO_EXECUTE)])
    assert not taint_toleration_ok(PodStatic(tolerations=[Toleration("m", "Exists", "", NO_SCHEDULE)]), node2)
    assert taint_toleration_ok(PodStatic(tolerations=[Toleration("m", "Exists", "", NO_EXECUTE)]), node2)


def test_node_unschedulable_filter():
    cordoned = NodeStatic(unschedulable=True)
    assert node_unschedulable_ok(PodStatic(), NodeStatic())
    assert not node_unschedulable_ok(PodStatic(), cordoned)
    tol = Toleration("node.kubernetes.io/unschedulable", "Exists", "", NO_SCHEDULE)
    assert node_unschedulable_ok(PodStatic(tolerations=[tol]), cordoned)
    assert node_unschedulable_ok(PodStatic(tolerations=[Toleration(operator="Exists")]), cordoned)
    assert not node_unschedulable_ok(PodStatic(tolerations=[Toleration("node.kubernetes.io/unschedulable", "Exists",
                                                                        "", NO_EXECUTE)]), cordoned)


@pytest.mark.parametrize("pod,labels,name,want", [
    (PodStatic(node_selector={"a": "1"}), {"a": "1", "b": "2"}, "n", True),
    (PodStatic(node_selector={"a": "1", "c": "3"}), {"a": "1"}, "n", False),
    (PodStatic(required_terms=[T([R("a", "In", ["1", "2"])])]), {"a": "2"}, "n", True),
    (PodStatic(required_terms=[T([R("a", "NotIn", ["1"])])]), {}, "n", True),            # absent key passes NotIn
    (PodStatic(required_terms=[T([R("a", "Exists")]), T([R("b", "Exists")])]), {"b": ""}, "n", True),  # ORed terms
    (PodStatic(required_terms=[T([R("a", "Exists"), R("b", "Exists")])]), {"b": ""}, "n", False),      # ANDed parts
    (PodStatic(required_terms=[T([R("g", "Gt", ["3"])])]), {"g": "4"}, "n", True),
    (PodStatic(required_terms=[T([R("g", "Gt", ["3"])])]), {"g": "x"}, "n", False),     # not an integer
    (PodStatic(required_terms=[T([R("g", "Lt", ["3"])])]), {"g": "3"}, "n", False),
    (PodStatic(required_terms=[T([], [R("metadata.name", "In", ["n"])])]), {}, "n", True),
    (PodStatic(required_terms=[T([], [R("metadata.name", "NotIn", ["n"])])]), {}, "n", False),
    (PodStatic(required_terms=[T()]), {"a": "1"}, "n", False),                            # empty term: no match
    (PodStatic(required_terms=[]), {"a": "1"}, "n", False),                               # no terms: no node
    (PodStatic(required_terms=[T([R("a", "DoesNotExist")])], node_selector={"b": "1"}), {"b": "1"}, "n", True),
])
def test_node_affinity_required(pod, labels, name, want):
    assert node_affinity_ok(pod, NodeStatic(labels=labels, name=name)) is want


def test_static_allow_matches_direct_checks():
    n = 600
    prof = with_upstream(shipped_profile())
    t = synth.make_cluster(synth.ClusterSpec(n), prof)
    pods = synth.make_pods(synth.StreamSpec(400, be_frac=0.3), prof)
    nodes, cls = synth.add_static(t, pods, synth.StaticSpec(), prof)
    assert len(cls.specs) == len(synth.static_templates())
    for i in range(n):
        for c, spec in enumerate(cls.specs):
            assert bool((int(t["static_allow"][i]) >> c) & 1) == node_static_ok(spec, nodes[i], STATIC_FILTERS)
    # some class is filtered somewhere, none everywhere except the empty-terms one
    assert (t["static_allow"] != 0xFFFFFFFF).any()
    # a subset of the filters: only TaintToleration
    m = static_allow(nodes, cls, ["TaintToleration"])
    for i in range(0, n, 7):
        for c, spec in enumerate(cls.specs):
            assert bool((int(m[i]) >> c) & 1) == taint_toleration_ok(spec, nodes[i])


def test_static_class_limit():
    cls = StaticClasses()
    for j in range(abi.MAX_STATIC_CLASSES):
        cls.classify(PodStatic(node_selector={"k": str(j)}))
    assert cls.classify(PodStatic(node_selector={"k": "0"})) == 0   # an existing class
    with pytest.raises(ValueError):
        cls.classify(PodStatic(node_selector={"k": "new"}))


def test_static_score_rejected():
    """NodeUnschedulable has no Score; NodeAffinity / TaintToleration Scores
    lower to the sequential cycle's normalized planes (weights 1..100)."""
    p = with_upstream(shipped_profile())
    p.scores = dict(p.scores)
    p.scores["NodeUnschedulable"] = 1
    with pytest.raises(ArgsError):
        to_c_config(p)
    p.scores = {**with_upstream(shipped_profile()).scores, "TaintToleration": 101}
    with pytest.raises(ArgsError):
        to_c_config(p)
    p.scores["TaintToleration"] = 3
    assert to_c_config(p).ext_weight[2] == 3


# ------------------------------------------------------- BalancedAllocation
def _one_node(cpu, mem, rcpu, rmem):
    t = NodeTable.empty(1)
    t["alloc0"][0], t["alloc1"][0] = cpu, mem
    t["requested0"][0], t["requested1"][0] = rcpu, rmem
    t["alloc_pods"][0] = 110
    return t


@pytest.mark.parametrize("node,req,want", [
    # upstream balanced_allocation_test.go worked examples ("resources requested"):
    ((4000, 10000, 0, 0), (3000, 5000), 87),    # fractions 0.75 / 0.5: std 0.125
    ((6000, 10000, 0, 0), (3000, 5000), 100),   # 0.5 / 0.5
    # worked from the same rules
    ((4000, 8000, 1000, 6000), (2000, 1000), 93),   # 0.75 / 0.875: std 0.0625, 93.75 truncated
    ((4000, 8000, 5000, 0), (0, 0), 50),        # cpu fraction capped at 1, mem 0: std 0.5
    ((4000, 0, 1000, 0), (1000, 0), 100),       # memory Allocatable 0: one fraction, std 0
    ((0, 0, 0, 0), (0, 0), 100),
])
def test_balanced_allocation_oracle(node, req, want):
    t = _one_node(*node)
    p = pod_array(1)
    p["req"][0, 0], p["req"][0, 1] = req
    prof = shipped_profile()
    prof.scores = {PLUGIN_BALANCED: 1}
    cfg = to_c_config(prof)
    o = oracle.Oracle(cfg, t)
    got = o.eval(p, status=False, scores=True)["scores"][0, 3, 0]
    fc = min(1.0, (node[2] + req[0]) / node[0]) if node[0] else None
    fm = min(1.0, (node[3] + req[1]) / node[1]) if node[1] else None
    fr = [f for f in (fc, fm) if f is not None]
    std = abs((fr[0] - fr[1]) / 2) if len(fr) == 2 else 0.0
    assert got == int((1 - std) * 100) == want


def test_oracle_static_status_bit():
    prof = with_upstream(shipped_profile(), balanced_weight=5)
    t = synth.make_cluster(synth.ClusterSpec(300), prof)
    pods = synth.make_pods(synth.StreamSpec(60, be_frac=0.3), prof)
    nodes, cls = synth.add_static(t, pods, synth.StaticSpec(), prof)
    r = oracle.Oracle(to_c_config(prof), t).eval(pods, k=4)
    for j in range(len(pods)):
        spec = cls.specs[int(pods["static_class"][j])]
        for i in range(0, 300, 5):
            fail = bool(r["status"][j, i] & abi.ST_STATIC_FAIL)
            assert fail == (not node_static_ok(spec, nodes[i], STATIC_FILTERS))
    assert (r["scores"][:, 3, :] > 0).all()


# ------------------------------------------------- NodeAffinity / TaintToleration Scores
# Worked from the published k8s v1.24 plugins (parity unpinned, like the
# filters above): NodeAffinity sums the weights of the matched preferred terms
# and normalizes by the max; TaintToleration counts the intolerable
# PreferNoSchedule taints and normalizes reversed.
def _norm(raw, reverse=False):
    return oracle.default_normalize(raw, reverse=reverse).tolist()


def test_node_affinity_score_weights():
    from koordinator_amd.nodefilters import node_affinity_score
    pref = [(2, T([R("foo", "In", ["bar"])])), (4, T([R("key", "In", ["value"])])),
            (5, T([R("foo", "In", ["bar"]), R("key", "In", ["value"]), R("az", "In", ["az1"])]))]
    pod = PodStatic(preferred_terms=pref)
    nodes = [NodeStatic(labels={"foo": "bar"}), NodeStatic(labels={"foo": "bar", "key": "value", "az": "az1"}),
             NodeStatic(labels={"key": "value"})]
    raw = [node_affinity_score(pod, n) for n in nodes]
    assert raw == [2, 11, 4]
    assert _norm(raw) == [18, 100, 36]
    one = PodStatic(preferred_terms=pref[:1])
    assert _norm([node_affinity_score(one, n) for n in nodes]) == [100, 100, 0]
    assert _norm([node_affinity_score(PodStatic(), n) for n in nodes]) == [0, 0, 0]
    # weight-0 and empty terms score nothing; match_fields read the node name
    odd = PodStatic(preferred_terms=[(0, T([R("foo", "Exists")])), (9, T()),
                                     (3, T([], [R("metadata.name", "In", ["n1"])]))])
    assert node_affinity_score(odd, NodeStatic(labels={"foo": "x"}, name="n1")) == 3
    assert node_affinity_score(odd, NodeStatic(labels={"foo": "x"}, name="n2")) == 0


def test_taint_toleration_score_counts():
    from koordinator_amd.nodefilters import taint_toleration_score
    P = PREFER_NO_SCHEDULE
    nodes = [NodeStatic(taints=[]), NodeStatic(taints=[Taint("a", "1", P)]),
             NodeStatic(taints=[Taint("a", "1", P), Taint("b", "2", P), Taint("c", "", NO_SCHEDULE)])]
    raw = [taint_toleration_score(PodStatic(), n) for n in nodes]
    assert raw == [0, 1, 2]
    assert _norm(raw, reverse=True) == [100, 50, 0]
    tol = PodStatic(tolerations=[Toleration("a", "Equal", "1", P)])
    assert [taint_toleration_score(tol, n) for n in nodes] == [0, 0, 1]
    # a toleration of another effect does not count for the Score
    ns = PodStatic(tolerations=[Toleration("a", "Exists", "", NO_SCHEDULE)])
    assert [taint_toleration_score(ns, n) for n in nodes] == [0, 1, 2]
    # every node tolerated: all raw 0 -> reversed normalize gives 100 everywhere
    allt = PodStatic(tolerations=[Toleration(operator="Exists")])
    assert _norm([taint_toleration_score(allt, n) for n in nodes], reverse=True) == [100, 100, 100]


def test_static_score_columns_from_synth():
    from koordinator_amd.config import with_normalized_scores
    from koordinator_amd.nodefilters import node_affinity_score, taint_toleration_score
    prof = with_normalized_scores(with_upstream(shipped_profile()), affinity=2, taint=1)
    t = synth.make_cluster(synth.ClusterSpec(300), prof)
    t.enable_ext(0)
    pods = synth.make_pods(synth.StreamSpec(200, be_frac=0.3), prof)
    nodes, cls = synth.add_static(t, pods, synth.StaticSpec(), prof)
    ss = t["static_score"]
    assert ss[:, 0].any() and ss[:, 1].any()
    for i in range(0, 300, 5):
        for c, spec in enumerate(cls.specs):
            assert ss[i, 0, c] == node_affinity_score(spec, nodes[i])
            assert ss[i, 1, c] == taint_toleration_score(spec, nodes[i])


def test_static_class_key_includes_preferred_terms():
    cls = StaticClasses()
    a = cls.classify(PodStatic(preferred_terms=[(1, T([R("a", "Exists")]))]))
    b = cls.classify(PodStatic(preferred_terms=[(2, T([R("a", "Exists")]))]))
    c = cls.classify(PodStatic(preferred_terms=[(1, T([R("a", "Exists")]))]))
    assert a != b and a == c


def test_node_name_filter():
    """(upstream) nodename/node_name.go Fits: a pod naming a node passes only
    that node; the name is part of the static class key only when the profile
    enables NodeName (with_upstream does)."""
    from koordinator_amd import k8s
    from koordinator_amd.marshal import pod_static
    nodes = [NodeStatic(name=f"n{i}") for i in range(5)]
    cls = StaticClasses()
    a = cls.classify(PodStatic(node_name="n3"))
    b = cls.classify(PodStatic())
    m = static_allow(nodes, cls, ["NodeName"])
    assert [(int(x) >> a) & 1 for x in m] == [0, 0, 0, 1, 0]
    assert all((int(x) >> b) & 1 for x in m)
    pod = k8s.Pod(name="p", node_name="n3")
    assert pod_static(pod, with_upstream(shipped_profile())).node_name == "n3"
    assert pod_static(pod, shipped_profile()).node_name == ""
    assert "NodeName" in with_upstream(shipped_profile()).filters
