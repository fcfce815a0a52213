"""Reservation host logic and the ranking-total claim, on CPU.

The device ranks nodes by a per-node total (resv.hpp) instead of the
reference's score normalized over the feasible nodes; the oracle implements
both (orc_eval's top-k: the ranking total; orc_place_stream: PreScore + Score
+ DefaultNormalizeScore + the weighted sum).  Here they must pick the same
node for every pod on random states."""
import numpy as np
import pytest

from koordinator_amd.snapshot import slot_col

import golden_cases as G
import oracle
from koordinator_amd import abi, k8s, marshal, synth
from koordinator_amd import reservation as rv
from koordinator_amd.config import ArgsError, shipped_profile, to_c_config


@pytest.mark.parametrize("seed,ordered", [(1, 0.0), (2, 0.05), (3, 0.3)])
def test_ranking_total_argmax_equals_normalized(seed, ordered):
    prof = shipped_profile(reservation=True)
    t = synth.make_cluster(synth.ClusterSpec(400, seed=seed), prof)
    synth.add_reservations(t, synth.ResvSpec(node_frac=0.4, groups=3, ordered_frac=ordered), seed=seed)
    pods = synth.make_pods(synth.StreamSpec(120, be_frac=0.3, seed=seed, resv_match_frac=0.6, resv_groups=3), prof)
    cfg = to_c_config(prof)
    top = oracle.Oracle(cfg, t).eval(pods, status=False, scores=False, k=1)["topk"][:, 0]["node"]
    for j in range(len(pods)):
        got = oracle.Oracle(cfg, t).place_stream(pods[j:j + 1])[0]
        assert got == top[j], j


def test_parse_order():
    L = rv.LABEL_RESERVATION_ORDER
    assert rv.parse_order({}) == 0
    assert rv.parse_order({L: "123456"}) == 123456
    assert rv.parse_order({L: "-5"}) == -5
    assert rv.parse_order({L: "abc"}) == 0
    assert rv.parse_order({L: "1.5"}) == 0
    assert rv.parse_order({L: str(1 << 63)}) == 0  # ParseInt out of range


def test_reservation_columns():
    prof = G.resv_profile()
    sel = rv.ReservationOwner(label_selector=rv.LabelSelector(match_labels={"app": "a"}))
    bad = rv.ReservationOwner(label_selector=rv.LabelSelector(
        match_expressions=[rv.LabelSelectorRequirement("k", "In", [])]))
    rs = [
        rv.Reservation("r0", "n0", allocatable=G.rlist({"cpu": "4", "memory": "8Gi"}), owners=[sel],
                       labels={rv.LABEL_RESERVATION_ORDER: "7"}, allocate_policy="Restricted"),
        rv.Reservation("r1", "n1", allocatable=G.rlist({"cpu": "2"}), owners=[sel], allocate_once=False,
                       allocated=G.rlist({"cpu": "1", "memory": "1Gi"}), assigned=1),
        rv.Reservation("r2", "n2", allocatable=G.rlist({"cpu": "2"}), owners=[bad]),
        rv.Reservation("r3", "n3", allocatable=G.rlist({"cpu": "2"}), phase="Pending"),
    ]
    nodes = [(f"n{i}", {"cpu": "32", "memory": "64Gi", "pods": "110"}) for i in range(4)]
    t, idx = G.build_resv_nodes(nodes, [r for r in rs if r.is_available()], prof)
    f = t["resv_flags"]
    assert f[0] & abi.RESV_PRESENT and f[0] & abi.RESV_ORDERED and f[0] & abi.RESV_ALLOCATE_ONCE
    assert (f[0] >> abi.RESV_POLICY_SHIFT) & 3 == abi.RESV_POLICY_RESTRICTED
    assert f[0] & abi.RESV_KEY_CPU and f[0] & abi.RESV_KEY_MEM
    assert f[1] & abi.RESV_KEY_CPU and not f[1] & abi.RESV_KEY_MEM and not f[1] & abi.RESV_ALLOCATE_ONCE
    assert t["resv_allocated0"][1] == 1000 and t["resv_allocated1"][1] == 0  # masked to ResourceNames
    assert t["resv_nz1"][1] == 200 << 20  # the reserve pod lists no memory: the non-zero default
    assert not f[2] & abi.RESV_PRESENT    # invalid owner selector: ParseError
    assert f[3] == 0                      # not Available
    assert (f[0] >> abi.RESV_GROUP_SHIFT) & 63 == (f[1] >> abi.RESV_GROUP_SHIFT) & 63  # same owner spec
    # reserve pods are NodeInfo pods
    assert t["npods"][0] == 1 and t["requested0"][0] == 4000
    pa = G.resv_pod({"cpu": "1"}, labels={"app": "a"})
    pb = G.resv_pod({"cpu": "1"}, labels={"app": "b"})
    g = int((f[0] >> abi.RESV_GROUP_SHIFT) & 63)
    assert idx.pod_mask(pa) == 1 << g and idx.pod_mask(pb) == 0
    rec = marshal.pod_records([pa], prof, idx)
    assert rec["resv_match"][0] == 1 << g and rec["flags"][0] & abi.POD_KEY_CPU and not rec["flags"][0] & abi.POD_KEY_MEM


def test_reservations_fill_node_slots():
    """Several Available reservations on a node take its slots in the given
    order (the nomination tie rule: lowest slot); more than
    KOORDHIP_RESV_SLOTS_MAX are rejected (more than KOORDHIP_RESV_SLOTS run in
    the sequential cycle)."""
    prof = G.resv_profile()
    rs = [rv.Reservation(f"r{i}", "n0", allocatable=G.rlist({"cpu": str(2 + i)})) for i in range(3)]
    t, _ = G.build_resv_nodes([("n0", {"cpu": "32", "memory": "64Gi", "pods": "110"}),
                               ("n1", {"cpu": "32", "memory": "64Gi", "pods": "110"})], rs, prof)
    assert t.resv_slots == 3
    assert [int(t[slot_col("resv_alloc0", q)][0]) for q in range(3)] == [2000, 3000, 4000]
    assert all(int(t[slot_col("resv_flags", q)][1]) == 0 for q in range(3))
    soa = t.as_soa()
    assert soa.resv_slots == 3 and soa.resv_alloc[0][2] == 3000 and soa.resv_alloc[0][1] == 0   # slot-major [s * n + i]
    rs6 = [rv.Reservation(f"r{i}", "n0", allocatable=G.rlist({"cpu": "1"})) for i in range(6)]
    t6, _ = G.build_resv_nodes([("n0", {"cpu": "32", "memory": "64Gi", "pods": "110"})], rs6, prof)
    assert t6.resv_slots == 6 and int(t6[slot_col("resv_alloc0", 5)][0]) == 1000
    rs9 = [rv.Reservation(f"r{i}", "n0", allocatable=G.rlist({"cpu": "1"})) for i in range(abi.RESV_SLOTS_MAX + 1)]
    with pytest.raises(rv.ReservationError):
        G.build_resv_nodes([("n0", {"cpu": "32", "memory": "64Gi", "pods": "110"})], rs9, prof)


def test_reservation_weight_must_dominate():
    prof = shipped_profile(reservation=True)
    prof.scores["Reservation"] = 200  # <= 100 x (Fit 1 + LoadAware 1)
    with pytest.raises(ArgsError):
        to_c_config(prof)


def test_synth_reservations_match_objects():
    """add_reservations' columns equal reservation_columns of the same reservations as objects."""
    prof = G.resv_profile()
    t = synth.make_cluster(synth.ClusterSpec(200, seed=4), prof)
    base = t.copy()
    synth.add_reservations(t, synth.ResvSpec(node_frac=0.5, groups=3, ordered_frac=0.3, cpu_only_frac=0.3), seed=4)
    owners = [[rv.ReservationOwner(label_selector=rv.LabelSelector(match_labels={"g": str(g)}))] for g in range(3)]
    idx = rv.ReservationIndex()
    for o in owners:
        idx.group(o)
    objs = []
    for i in np.flatnonzero(t["resv_flags"]):
        f = int(t["resv_flags"][i])
        alloc = {"cpu": f"{int(t['resv_alloc0'][i])}m"}
        if f & abi.RESV_KEY_MEM:
            alloc["memory"] = str(int(t["resv_alloc1"][i]))
        allocated = {"cpu": f"{int(t['resv_allocated0'][i])}m", "memory": str(int(t["resv_allocated1"][i]))}
        pol = ["", "Aligned", "Restricted"][(f >> abi.RESV_POLICY_SHIFT) & 3]
        labels = {}
        if f & abi.RESV_ORDERED:
            labels[rv.LABEL_RESERVATION_ORDER] = str(100 + int(t["resv_order_rank"][i]))
        objs.append(rv.Reservation(f"r{i}", t.names[i], allocatable=G.rlist(alloc), allocated=G.rlist(allocated),
                                   owners=owners[(f >> abi.RESV_GROUP_SHIFT) & 63], labels=labels,
                                   allocate_policy=pol, allocate_once=bool(f & abi.RESV_ALLOCATE_ONCE),
                                   unschedulable=bool(f & abi.RESV_UNSCHEDULABLE), assigned=int(t["resv_assigned"][i])))
    rv.reservation_columns(base, {n: i for i, n in enumerate(base.names)}, objs, idx)
    for c in ("resv_flags", "resv_order_rank", "resv_alloc0", "resv_alloc1", "resv_nz0", "resv_nz1",
              "resv_allocated0", "resv_allocated1", "resv_assigned"):
        assert np.array_equal(base[c], t[c]), c


@pytest.mark.parametrize("loaded", [0, 1])
def test_same_order_reservations_tie_to_lowest_index(loaded):
    """Two matched reservations with the same order label: upstream
    PreScore makes the FIRST node of the smallest order the preferred node
    (scoring.go:89-98, strict '>' keeps the first) whatever its other plugins'
    total; the harness's node list is in index order, so the lower index wins.
    The device's ranking total gives both nodes the same key (resv.hpp), so its
    argmax is the lower index too -- checked against the oracle's literal
    PreScore + Score + DefaultNormalizeScore cycle."""
    prof = G.resv_profile()
    sel = rv.ReservationOwner(label_selector=rv.LabelSelector(match_labels={"app": "a"}))
    L = rv.LABEL_RESERVATION_ORDER
    nodes = [(f"n{i}", {"cpu": "32", "memory": "64Gi", "pods": "110"}) for i in range(4)]
    busy = {"n1": [G.resv_pod({"cpu": "20", "memory": "40Gi"}, name="load")]} if loaded else None
    rs = [rv.Reservation("r1", "n1", allocatable=G.rlist({"cpu": "4", "memory": "8Gi"}), owners=[sel], labels={L: "5"}),
          rv.Reservation("r2", "n2", allocatable=G.rlist({"cpu": "4", "memory": "8Gi"}), owners=[sel], labels={L: "5"}),
          rv.Reservation("r3", "n3", allocatable=G.rlist({"cpu": "4", "memory": "8Gi"}), owners=[sel], labels={L: "9"})]
    t, idx = G.build_resv_nodes(nodes, rs, prof, node_pods=busy)
    pods = marshal.pod_records([G.resv_pod({"cpu": "1", "memory": "1Gi"}, labels={"app": "a"})], prof, idx)
    cfg = to_c_config(prof)
    placed = oracle.Oracle(cfg, t).place_stream(pods)[0]
    top = oracle.Oracle(cfg, t).eval(pods, status=False, scores=False, k=4)["topk"][0]
    assert placed == 1
    assert top["node"][0] == 1 and top["score"][0] == top["score"][1] and top["node"][1] == 2


# ------------------------------------------------------------ reservation affinity
def _aff_pod(aff_json, labels=None):
    return k8s.Pod(name="p", labels=dict(labels or {}), priority=9500,
                   annotations={rv.ANNOTATION_RESERVATION_AFFINITY: aff_json},
                   containers=[k8s.Container(requests=G.rlist({"cpu": "1"}))])


def test_match_reservation_kat():
    """Test_matchReservation (reservation/transformer_test.go:345-442): owners
    only, and owners + a required affinity term on the reservation's labels."""
    sel = rv.ReservationOwner(label_selector=rv.LabelSelector(match_labels={"app": "test"}))
    r = rv.Reservation("r", "n0", labels={"reservation-type": "reservation-test"}, owners=[sel],
                       allocatable=G.rlist({"cpu": "1"}))
    pod = k8s.Pod(name="p", labels={"app": "test"})
    idx = rv.ReservationIndex()
    idx.group(r.owners, {}, r)
    assert idx.pod_mask(pod) == 1                                   # :355-377 only match reservation owners
    aff = ('{"requiredDuringSchedulingIgnoredDuringExecution": {"reservationSelectorTerms": [{"matchExpressions": '
           '[{"key": "reservation-type", "operator": "In", "values": ["reservation-test"]}]}]}}')
    p2 = _aff_pod(aff, {"app": "test"})
    idx = rv.ReservationIndex()
    assert idx.register_affinities([p2])
    idx.group(r.owners, {}, r)
    assert idx.pod_mask(p2) == 1                                    # :378-422 owners + affinity
    assert rv.pod_keys(p2) & abi.POD_RESV_AFFINITY


def test_reservation_affinity_selects_by_labels_and_name():
    """matchReservation's fake node (transformer.go:340-356): node labels
    overlaid with the reservation's, the reservation's name for matchFields."""
    own = [rv.ReservationOwner(label_selector=rv.LabelSelector(match_labels={"app": "a"}))]
    rs = [rv.Reservation("ra", "n0", labels={"tier": "gold"}, owners=own, allocatable=G.rlist({"cpu": "2"})),
          rv.Reservation("rb", "n1", labels={"tier": "silver"}, owners=own, allocatable=G.rlist({"cpu": "2"})),
          rv.Reservation("rc", "n2", owners=own, allocatable=G.rlist({"cpu": "2"}))]
    node_labels = {"n0": {"zone": "z1"}, "n1": {"zone": "z2", "tier": "gold"}, "n2": {"zone": "z1", "tier": "gold"}}
    pods = [_aff_pod('{"reservationSelector": {"tier": "gold"}}', {"app": "a"}),
            _aff_pod('{"requiredDuringSchedulingIgnoredDuringExecution": {"reservationSelectorTerms": ['
                     '{"matchFields": [{"key": "metadata.name", "operator": "In", "values": ["rb"]}]}]}}', {"app": "a"}),
            _aff_pod('{"requiredDuringSchedulingIgnoredDuringExecution": {"reservationSelectorTerms": ['
                     '{"matchExpressions": [{"key": "zone", "operator": "In", "values": ["z1"]}]}]}}', {"app": "b"}),
            k8s.Pod(name="plain", labels={"app": "a"})]
    idx = rv.ReservationIndex()
    idx.register_affinities(pods)
    prof = G.resv_profile()
    nodes = [(f"n{i}", {"cpu": "32", "memory": "64Gi", "pods": "110"}) for i in range(3)]
    from koordinator_amd import marshal
    cluster = marshal.ClusterState(nodes=[k8s.Node(name=n, allocatable=G.rlist(a), labels=node_labels[n]) for n, a in nodes])
    for r in rs:
        cluster.node_pods.setdefault(r.node_name, []).append(r.reserve_pod())
    t = marshal.build_table(cluster, prof, G.NOW)
    rv.reservation_columns(t, {n: i for i, (n, _) in enumerate(nodes)}, rs, idx, node_labels)
    recs = marshal.pod_records(pods, prof, idx)
    grp = [(int(t["resv_flags"][i]) >> abi.RESV_GROUP_SHIFT) & 63 for i in range(3)]
    matched = [[bool((int(recs["resv_match"][j]) >> grp[i]) & 1) for i in range(3)] for j in range(4)]
    # reservation labels win over the node's (ra gold; rb silver although n1 is gold; rc takes n2's gold)
    assert matched[0] == [True, False, True]
    assert matched[1] == [False, True, False]                       # matchFields metadata.name
    assert matched[2] == [False, False, False]                      # owners do not match app=b
    assert matched[3] == [True, True, True]                         # no affinity: owners only
    # the Filter: an affinity pod fits only where a reservation matched it (plugin.go:378-381)
    cfg = to_c_config(prof)
    st = oracle.Oracle(cfg, t).eval(recs, status=True, scores=False)["status"]
    assert [(st[0, i] & abi.ST_RESV_FAIL) != 0 for i in range(3)] == [False, True, False]
    assert all(st[2, i] & abi.ST_RESV_FAIL for i in range(3))
    assert not any(st[3, i] & abi.ST_RESV_FAIL for i in range(3))


def test_unregistered_affinity_is_an_error():
    idx = rv.ReservationIndex()
    with pytest.raises(rv.ReservationError):
        idx.pod_mask(_aff_pod('{"reservationSelector": {"x": "y"}}'))
    with pytest.raises(rv.ReservationError):
        rv.parse_reservation_affinity({rv.ANNOTATION_RESERVATION_AFFINITY: "{bad"})
