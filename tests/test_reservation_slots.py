"""Several Available reservations per node (koordhip_node_soa.resv_slots).

Known answers: reservation/nominator_test.go:35-304 (TestNominateReservation)
-- a node's matched reservations, the one NominateReservation picks:
  * "preferred reservation" (:118-204): an ordered one (order 100) beside an
    unordered one, both 2C4G, pod 2C4G -> the ordered one;
  * "allocated reservation" (:205-248): 4C8G and 2C4G with 2C4G fully
    allocated, pod 2C4G -> 4C8G (the other fails FilterReservation:
    nothing remains, plugin.go:530-533);
  * "matched reservations" (:249-270): 4C8G and 2C4G, pod 2C4G -> 2C4G
    (scoreReservation MostAllocated: 100 vs 50, scoring.go:177-200);
  * "node without reservations" (:112-116) -> none.
The reference's tie order among a node's reservations is Go map order
(cache.go:236-252); here the lowest slot, pinned by the tie cases below.
The same cases run on the oracle (CPU) and through the device's Reserve
(GPU: the nominated slot's Allocated / assigned advance).  Random workloads
with up to KOORDHIP_RESV_SLOTS reservations per node compare the device's
evaluation and greedy streams with the oracle bit for bit."""
import numpy as np
import pytest

import golden_cases as G
import oracle
from koordinator_amd import abi, marshal, synth
from koordinator_amd import reservation as rv
from koordinator_amd.config import shipped_profile, to_c_config

NODE = [("test-node", {"cpu": "32", "memory": "64Gi", "pods": "110"})]


def _r(name, cpu, mem, order=None, allocated=None):
    labels = {rv.LABEL_RESERVATION_ORDER: str(order)} if order else {}
    return rv.Reservation(name, "test-node", allocatable=G.rlist({"cpu": cpu, "memory": mem}),
                          owners=G.match_all_owner(), labels=labels, allocate_once=False,
                          allocated=G.rlist(allocated or {}), assigned=1 if allocated else 0)


# (case, reservations in the node's slot order, expected nominated slot)
NOMINATOR_CASES = [
    ("preferred reservation", [_r("preferred-reservation", "2", "4Gi", order=100), _r("normal-reservation", "2", "4Gi")], 0),
    ("preferred reservation, slots swapped", [_r("normal-reservation", "2", "4Gi"),
                                              _r("preferred-reservation", "2", "4Gi", order=100)], 1),
    ("allocated reservation", [_r("reservation4C8G", "4", "8Gi"),
                               _r("reservation2C4G", "2", "4Gi", allocated={"cpu": "2", "memory": "4Gi"})], 0),
    ("matched reservations", [_r("reservation4C8G", "4", "8Gi"), _r("reservation2C4G", "2", "4Gi")], 1),
    ("node without reservations", [], -1),
    # ties (the reference: map order) -> the lowest slot
    ("equal scores", [_r("a", "4", "8Gi"), _r("b", "4", "8Gi")], 0),
    ("equal orders", [_r("a", "4", "8Gi", order=7), _r("b", "2", "4Gi", order=7)], 0),
    ("smaller order wins over the score", [_r("a", "2", "4Gi", order=9), _r("b", "4", "8Gi", order=3),
                                            _r("c", "2", "4Gi")], 1),
]


def _case(rs):
    prof = G.resv_profile()
    t, idx = G.build_resv_nodes(NODE, rs, prof)
    pod = marshal.pod_records([G.resv_pod({"cpu": "2", "memory": "4Gi"})], prof, idx)
    return prof, t, pod


@pytest.mark.parametrize("name,rs,want", NOMINATOR_CASES, ids=[c[0] for c in NOMINATOR_CASES])
def test_nominate_reservation_oracle(name, rs, want):
    prof, t, pod = _case(rs)
    assert oracle.Oracle(to_c_config(prof), t).resv_nominate(pod, 0) == want


@pytest.mark.gpu
@pytest.mark.parametrize("name,rs,want", NOMINATOR_CASES, ids=[c[0] for c in NOMINATOR_CASES])
def test_nominate_reservation_gpu(name, rs, want):
    """The device's Reserve goes into the nominated slot (and the oracle's too)."""
    import torch  # noqa: F401
    from koordinator_amd.engine import PlacementEngine
    prof, t, pod = _case(rs)
    o = oracle.Oracle(to_c_config(prof), t)
    with PlacementEngine(prof, device=0) as e:
        e.load_snapshot(t)
        before = e.read_reservations()
        e.commit(pod[0], 0)
        after = e.read_reservations()
    o.commit(pod[0], 0)
    ref = o.resv_state()
    assert np.array_equal(after["allocated"], ref["allocated"]) and np.array_equal(after["assigned"], ref["assigned"])
    grew = np.flatnonzero(after["assigned"] != before["assigned"])
    n = t.n
    assert (grew // n).tolist() == ([want] if want >= 0 else [])


def _workload(n, p, seed=7, slots=4, multi=0.6, numa=False, ordered=0.1, match=0.6):
    prof = shipped_profile(numa=numa, reservation=True)
    t = synth.make_cluster(synth.ClusterSpec(n, seed=seed), prof)
    if numa:
        synth.add_numa(t, synth.NumaSpec(), prof, seed=seed)
    synth.add_reservations(t, synth.ResvSpec(node_frac=0.4, groups=3, ordered_frac=ordered, slots=slots,
                                             multi_frac=multi, allocate_once_frac=0.3), seed=seed)
    pods = synth.make_pods(synth.StreamSpec(p, be_frac=0.3, seed=seed, resv_match_frac=match, resv_groups=3), prof)
    return prof, t, pods


def test_synth_slots_fill_in_order():
    _, t, _ = _workload(2000, 10)
    from koordinator_amd.snapshot import slot_col
    has = [t[slot_col("resv_flags", q)] & abi.RESV_PRESENT != 0 for q in range(4)]
    assert has[1].sum() > 50 and has[3].sum() > 5
    for q in range(1, 4):
        assert not (has[q] & ~has[q - 1]).any()


@pytest.mark.parametrize("seed,ordered", [(1, 0.0), (2, 0.1), (3, 0.4)])
def test_slots_ranking_total_argmax_equals_normalized(seed, ordered):
    """The per-node ranking total (orc_eval top-k) and the reference's
    normalized Reservation score (orc_place_stream) pick the same node with
    several reservations per node."""
    prof, t, pods = _workload(300, 80, seed=seed, ordered=ordered)
    cfg = to_c_config(prof)
    top = oracle.Oracle(cfg, t).eval(pods, status=False, scores=False, k=1)["topk"][:, 0]["node"]
    for j in range(len(pods)):
        assert oracle.Oracle(cfg, t).place_stream(pods[j:j + 1])[0] == top[j], j


def test_one_slot_table_equals_plain_columns():
    """slots = 1 keeps the one-per-node layout bit for bit (config 5's fixture)."""
    prof = shipped_profile(reservation=True)
    a = synth.make_cluster(synth.ClusterSpec(500, seed=3), prof)
    b = a.copy()
    synth.add_reservations(a, synth.ResvSpec(node_frac=0.3), seed=3)
    synth.add_reservations(b, synth.ResvSpec(node_frac=0.3, slots=1, multi_frac=0.9), seed=3)
    for c in a.cols:
        assert np.array_equal(a[c], b[c]), c
    assert a.as_soa().resv_slots == 0


@pytest.mark.gpu
@pytest.mark.parametrize("numa", [False, True])
def test_gpu_slots_eval_parity(numa):
    import torch  # noqa: F401
    from koordinator_amd.engine import PlacementEngine
    prof, t, pods = _workload(1500, 48, numa=numa)
    ref = oracle.Oracle(to_c_config(prof), t).eval(pods, k=16)
    with PlacementEngine(prof, device=0) as e:
        e.load_snapshot(t)
        got = e.eval(pods, k=16)
    assert np.array_equal(ref["status"], got["status"])
    assert (got["status"] & abi.ST_RESV_FAIL).any()
    assert np.array_equal(ref["scores"], got["scores"])
    assert np.array_equal(ref["topk"], got["topk"])


@pytest.mark.gpu
@pytest.mark.parametrize("numa,mode", [(False, "fused"), (False, "split"), (True, "fused"), (False, "rounds")])
def test_gpu_slots_stream_parity(numa, mode, monkeypatch):
    import torch  # noqa: F401
    from koordinator_amd.engine import PlacementEngine
    if mode == "split":
        monkeypatch.setenv("KOORDHIP_EVAL", "split")
    if mode == "rounds":
        monkeypatch.setenv("KOORDHIP_ROUND_LAUNCH", "1")
    prof, t, pods = _workload(3000, 2500, numa=numa)
    o = oracle.Oracle(to_c_config(prof), t)
    ref = o.place_stream(pods, threads=8)
    with PlacementEngine(prof, device=0) as e:
        e.load_snapshot(t)
        got = e.place_stream(pods)
        assert np.array_equal(ref, got), np.flatnonzero(ref != got)[:10]
        gr, rr = e.read_reservations(), o.resv_state()
        assert np.array_equal(gr["allocated"], rr["allocated"]) and np.array_equal(gr["assigned"], rr["assigned"])
        gs, rs = e.read_nodes(), o.state()
        for k in ("requested", "nz", "npods", "la_used"):
            assert np.array_equal(gs[k], rs[k]), k
    # Reserves went into slots >= 1 too
    n = t.n
    took = np.flatnonzero(rr["assigned"] != np.concatenate(
        [t[c] for c in ["resv_assigned"] + [f"resv_assigned@{q}" for q in range(1, 4)]]))
    assert (took >= n).sum() > 10 and (took < n).sum() > 10
