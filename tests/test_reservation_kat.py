"""Reservation plugin pinned by the reference's table tests
(tests/golden/reservation_cases.json, written by
tests/golden/make_reservation_golden.py): the oracle on CPU, libkoordhip.so on
the GPU.  On the device the Reservation score is visible through the ranking
total of koordhip_eval's top-k (resv.hpp): raw score s > 0 -> s * (B + 1) + b,
an ordered matched reservation above every such total."""
import numpy as np
import pytest

import golden_cases as G
import oracle
from koordinator_amd import abi, marshal
from koordinator_amd import reservation as rv
from koordinator_amd.config import to_c_config

D = G.reservation_cases()
NODE = ("test-node", {"cpu": "32", "memory": "64Gi", "pods": "110"})


def _resv(name, node, alloc, allocated=None, owners=None, order=None, policy="", allocate_once=None, assigned=0):
    labels = {rv.LABEL_RESERVATION_ORDER: order} if order else {}
    return rv.Reservation(name=name, node_name=node, allocatable=G.rlist(alloc), allocated=G.rlist(allocated or {}),
                          owners=G.match_all_owner() if owners is None else owners, labels=labels,
                          allocate_policy=policy, allocate_once=allocate_once, assigned=assigned)


def _one(case_res, pod_req, policy="", node=NODE, node_pods=None):
    prof = G.resv_profile()
    r = _resv("r", node[0], case_res["allocatable"], case_res.get("allocated"), policy=policy)
    table, idx = G.build_resv_nodes([node], [r], prof, node_pods)
    pod = marshal.pod_records([G.resv_pod(pod_req)], prof, idx)
    return prof, table, pod


def _b1(prof):
    cfg = to_c_config(prof)
    return 100 * sum(cfg.plugin_weight[i] for i in range(abi.NPLUGINS)) + 1


# ------------------------------------------------------------------ TestScore
@pytest.mark.parametrize("case", D["score"], ids=[c["name"] for c in D["score"]])
def test_score_kat_oracle(case):
    prof, t, pod = _one(case["reservation"], case["pod"])
    o = oracle.Oracle(to_c_config(prof), t)
    raw = o.resv_score(pod, 0) if o.resv_nominated(pod, 0) else 0
    assert raw == case["want_raw"], case["source"]
    # the ranking total koordhip_eval reports: raw * (B + 1) + the Fit score
    ev = o.eval(pod, k=1)
    assert ev["topk"][0, 0]["score"] == raw * _b1(prof) + ev["scores"][0, 0, 0], case["source"]


# ------------------------------------------------------------------ TestScoreWithOrder
def _order_case():
    c = D["order"]
    prof = G.resv_profile()
    nodes = [(r["node"], dict(NODE[1])) for r in c["reservations"]]
    rs = [_resv(f"r{i}", r["node"], r["allocatable"], order=r.get("order")) for i, r in enumerate(c["reservations"])]
    table, idx = G.build_resv_nodes(nodes, rs, prof)
    pod = marshal.pod_records([G.resv_pod(c["pod"])], prof, idx)
    return c, prof, table, pod


def test_score_with_order_oracle():
    c, prof, t, pod = _order_case()
    o = oracle.Oracle(to_c_config(prof), t)
    assert o.resv_normalized(pod, [0, 1, 2, 3]).tolist() == c["want_normalized"], c["source"]
    raw = [o.resv_score(pod, i) for i in range(3)]
    assert raw == c["want_raw"][:3], c["source"]
    want = [n for n, _ in [(r["node"], 0) for r in c["reservations"]]].index(c["want_preferred"])
    assert o.place_stream(pod).tolist() == [want], c["source"]


# ------------------------------------------------------------------ filterWithReservations
def _filter_case(c):
    req = c["pod_requested"]
    # NodeInfo pods: the reserve pod (its Allocatable) and a pod holding the rest of podRequested
    rest = {k: str(G.rlist(req)[k].v - G.rlist(c["reservation"]["allocatable"]).get(k, G.rlist({"x": "0"})["x"]).v)
            for k in req}
    filler = G.resv_pod({k: v for k, v in rest.items()}, name="filler")
    node = ("test-node", {"cpu": "32", "memory": "32Gi", "pods": "100"})
    return _one(c["reservation"], c["pod"], policy=c["policy"], node=node, node_pods={"test-node": [filler]})


@pytest.mark.parametrize("case", D["filter"], ids=[c["name"] for c in D["filter"]])
def test_filter_kat_oracle(case):
    prof, t, pod = _filter_case(case)
    o = oracle.Oracle(to_c_config(prof), t)
    assert o.resv_filter(pod, 0) == case["want"], case["source"]
    st = o.eval(pod)["status"][0, 0]
    assert (st & abi.ST_RESV_FAIL == 0) == case["want"], case["source"]


# ------------------------------------------------------------------ FilterReservation
@pytest.mark.parametrize("case", D["nominate"], ids=[c["name"] for c in D["nominate"]])
def test_nominate_kat_oracle(case):
    prof, t, pod = _one(case["reservation"], case["pod"])
    assert oracle.Oracle(to_c_config(prof), t).resv_nominated(pod, 0) == case["want"], case["source"]


# ------------------------------------------------------------------ TestRestoreReservation
def _restore_nodes():
    c = D["restore"]
    prof = G.resv_profile()
    base = [G.resv_pod(p, name=f"p{i}") for i, p in enumerate(c["pods"])]
    u, m = c["unmatched"], c["matched"]
    held = [G.resv_pod(a, name=f"held{i}") for i, a in enumerate(u["assigned"])]
    owner_m = [rv.ReservationOwner(label_selector=rv.LabelSelector(match_labels=m["owner_labels"]))]
    owner_u = [rv.ReservationOwner(label_selector=rv.LabelSelector(match_labels={"other": "owner"}))]
    alloc_u = {}
    for a in u["assigned"]:
        for k, v in G.rlist(a).items():
            alloc_u[k] = str((G.rlist(alloc_u).get(k, G.rlist({"x": "0"})["x"]).v + v.v))
    ru = _resv("ru", "node-u", u["allocatable"], alloc_u, owners=owner_u, allocate_once=u["allocate_once"],
               assigned=len(u["assigned"]))
    rm = _resv("rm", "node-m", m["allocatable"], owners=owner_m)
    node = dict(c["node"], pods="110")
    t, idx = G.build_resv_nodes([("node-u", node), ("node-m", node)], [ru, rm], prof,
                                {"node-u": base + held, "node-m": list(base)})
    pod = marshal.pod_records([G.resv_pod({}, labels=c["pod_labels"])], prof, idx)
    return c, prof, t, pod


def test_restore_kat_oracle():
    c, prof, t, pod = _restore_nodes()
    o = oracle.Oracle(to_c_config(prof), t)
    q = lambda d: [G.rlist(d)["cpu"].milli_value(), G.rlist(d)["memory"].value()]
    du, nu, pu = o.resv_restore_delta(pod, 0)
    dm, nm, pm = o.resv_restore_delta(pod, 1)
    assert du.tolist() == q(c["unmatched"]["want_delta"]) and pu == 0, c["source"]
    assert dm.tolist() == q(c["matched"]["want_delta"]) and pm == c["matched"]["want_pods_delta"], c["source"]
    assert nu.tolist() == du.tolist() and nm.tolist() == dm.tolist()  # NonZeroRequested moves with Requested here
    before = np.array(q(c["requested_before"]))
    assert (before + du).tolist() == q(c["want_pod_requested"]), c["source"]
    assert (before + du + dm).tolist() == q(c["want_requested_after"]), c["source"]


# ------------------------------------------------------------------ matchReservation
@pytest.mark.parametrize("case", D["match"], ids=[c["name"] for c in D["match"]])
def test_match_kat(case):
    owners = [rv.ReservationOwner(label_selector=rv.LabelSelector(match_labels=case["owner_labels"]))]
    pod = G.resv_pod({}, labels=case["pod_labels"])
    assert rv.match_owners(pod, owners) == case["want"], case["source"]


def test_reservation_affinity_rejected():
    idx = rv.ReservationIndex()
    idx.group([rv.ReservationOwner()])
    pod = G.resv_pod({})
    pod.annotations[rv.ANNOTATION_RESERVATION_AFFINITY] = '{"reservationSelector": {"a": "b"}}'
    with pytest.raises(rv.ReservationError):
        idx.pod_mask(pod)


# ------------------------------------------------------------------ the same on the GPU
@pytest.fixture(scope="module")
def Engine():
    import torch  # noqa: F401
    from koordinator_amd.engine import PlacementEngine
    return PlacementEngine


def _gpu_eval(Engine, prof, t, pod, k=1):
    with Engine(prof, device=0) as e:
        e.load_snapshot(t)
        return e.eval(pod, k=k)


@pytest.mark.gpu
@pytest.mark.parametrize("case", D["score"], ids=[c["name"] for c in D["score"]])
def test_score_kat_gpu(Engine, case):
    prof, t, pod = _one(case["reservation"], case["pod"])
    ev = _gpu_eval(Engine, prof, t, pod)
    assert ev["topk"][0, 0]["score"] == case["want_raw"] * _b1(prof) + ev["scores"][0, 0, 0], case["source"]


@pytest.mark.gpu
def test_score_with_order_gpu(Engine):
    c, prof, t, pod = _order_case()
    with Engine(prof, device=0) as e:
        e.load_snapshot(t)
        tk = e.eval(pod, k=4)["topk"][0]
        got = e.place_stream(pod)
    names = [r["node"] for r in c["reservations"]]
    assert int(tk[0]["node"]) == names.index(c["want_preferred"]) and int(got[0]) == names.index(c["want_preferred"])
    # the other three rank by raw score 100 (all equal), then node index
    assert [int(x) for x in tk["node"][1:]] == [0, 1, 2]


@pytest.mark.gpu
@pytest.mark.parametrize("case", D["filter"], ids=[c["name"] for c in D["filter"]])
def test_filter_kat_gpu(Engine, case):
    prof, t, pod = _filter_case(case)
    st = _gpu_eval(Engine, prof, t, pod)["status"][0, 0]
    assert (st & abi.ST_RESV_FAIL == 0) == case["want"], case["source"]


@pytest.mark.gpu
@pytest.mark.parametrize("case", D["nominate"], ids=[c["name"] for c in D["nominate"]])
def test_nominate_kat_gpu(Engine, case):
    prof, t, pod = _one(case["reservation"], case["pod"])
    ev = _gpu_eval(Engine, prof, t, pod)
    assert (ev["topk"][0, 0]["score"] >= _b1(prof)) == case["want"], case["source"]


@pytest.mark.gpu
def test_restore_kat_gpu(Engine):
    c, prof, t, pod = _restore_nodes()
    ref = oracle.Oracle(to_c_config(prof), t).eval(pod, k=2)
    got = _gpu_eval(Engine, prof, t, pod, k=2)
    for key in ("status", "scores"):
        assert np.array_equal(ref[key], got[key]), key
    assert np.array_equal(ref["topk"], got["topk"])
