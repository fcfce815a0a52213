"""Reservation on the GPU vs the oracle (bit-exact): Filter status / scores /
top-k on random reservation nodes, and greedy streams whose Reserves go into
reservations (reservation Allocated / assigned pods advance) -- with and
without NodeNUMAResource, in the persistent pipeline and with one resolve
launch per round.  The oracle selects with the reference's normalized
Reservation score (DefaultNormalizeScore over the feasible nodes, weight
5000); the device with its per-node ranking total: equal placements are the
proof that the two orders agree on the argmax."""
import os

import numpy as np
import pytest

import oracle
from koordinator_amd import abi, synth
from koordinator_amd.config import shipped_profile, to_c_config

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def Engine():
    import torch  # noqa: F401
    from koordinator_amd.engine import PlacementEngine
    return PlacementEngine


def _workload(n, p, numa, seed=5, node_frac=0.3, match=0.4, ordered=0.05, cpuset=0.0):
    prof = shipped_profile(numa=numa, reservation=True)
    t = synth.make_cluster(synth.ClusterSpec(n, seed=seed), prof)
    if numa:
        synth.add_numa(t, synth.NumaSpec(), prof, seed=seed)
    synth.add_reservations(t, synth.ResvSpec(node_frac=node_frac, groups=4, ordered_frac=ordered), seed=seed)
    pods = synth.make_pods(synth.StreamSpec(p, be_frac=0.3, seed=seed, cpuset_frac=cpuset, resv_match_frac=match,
                                            resv_groups=4), prof)
    return prof, t, pods


def _state_eq(e, o, numa):
    got, ref = e.read_nodes(), o.state()
    for k in ("requested", "nz", "npods", "la_used"):
        assert np.array_equal(got[k], ref[k]), k
    gr, rr = e.read_reservations(), o.resv_state()
    assert np.array_equal(gr["allocated"], rr["allocated"])
    assert np.array_equal(gr["assigned"], rr["assigned"])
    if numa:
        gn, rn = e.read_numa(), o.numa_state()
        for k in ("free", "excl_pcpu", "excl_numa", "alloc_cnt"):
            assert np.array_equal(gn[k], rn[k]), k


@pytest.mark.parametrize("numa", [False, True])
def test_gpu_resv_eval_parity(Engine, numa):
    prof, t, pods = _workload(1500, 48, numa)
    ref = oracle.Oracle(to_c_config(prof), t).eval(pods, k=16)
    with Engine(prof, device=0) as e:
        e.load_snapshot(t)
        got = e.eval(pods, k=16)
    assert np.array_equal(ref["status"], got["status"])
    assert (got["status"] & abi.ST_RESV_FAIL).any()
    assert np.array_equal(ref["scores"], got["scores"])
    assert np.array_equal(ref["topk"], got["topk"])


@pytest.mark.parametrize("numa,mode", [(False, "persistent"), (True, "persistent"), (False, "rounds"),
                                       (True, "cpuset"), (True, "r1")])
def test_gpu_resv_stream_parity(Engine, numa, mode, monkeypatch):
    if mode == "rounds":
        monkeypatch.setenv("KOORDHIP_ROUND_LAUNCH", "1")
    if mode == "r1":  # one node per scan lane
        monkeypatch.setenv("KOORDHIP_TOPK_R", "1")
    prof, t, pods = _workload(3000, 2500, numa, cpuset=0.2 if mode == "cpuset" else 0.0)
    o = oracle.Oracle(to_c_config(prof), t)
    ref = o.place_stream(pods, threads=8)
    with Engine(prof, device=0) as e:
        e.load_snapshot(t)
        got = e.place_stream(pods)
        assert np.array_equal(ref, got), np.flatnonzero(ref != got)[:10]
        _state_eq(e, o, numa)
    # the stream took reservations
    assert (o.resv_state()["assigned"] > t["resv_assigned"]).sum() > 20


def test_gpu_resv_contended(Engine):
    """Few large reservations, most pods matching: pods pile into the same
    reservations round after round (reusable ones fill up; Restricted /
    Aligned filters flip as Allocated grows)."""
    prof, t, pods = _workload(800, 3000, False, seed=9, node_frac=0.6, match=0.8, ordered=0.02)
    t["resv_flags"][:] &= np.uint32(~abi.RESV_ALLOCATE_ONCE & 0xFFFFFFFF)  # every reservation reusable
    o = oracle.Oracle(to_c_config(prof), t)
    ref = o.place_stream(pods, threads=8)
    with Engine(prof, device=0) as e:
        e.load_snapshot(t)
        got = e.place_stream(pods)
        assert np.array_equal(ref, got), np.flatnonzero(ref != got)[:10]
        _state_eq(e, o, False)


def test_gpu_resv_commit_uncommit(Engine):
    prof, t, pods = _workload(300, 64, False)
    o = oracle.Oracle(to_c_config(prof), t)
    with Engine(prof, device=0) as e:
        e.load_snapshot(t)
        nodes = np.flatnonzero(t["resv_flags"] & abi.RESV_PRESENT)
        for j, pod in enumerate(pods[:32]):
            nd = int(nodes[j % len(nodes)])
            rc, _ = o.commit(pod, nd)
            assert rc == 0
            e.commit(pod, nd)
        _state_eq(e, o, False)
        # Unreserve of a pod the node's reservation matches is refused on both sides
        m = [(p, int(nd)) for p in pods for nd in nodes
             if p["resv_match"] >> np.uint64((int(t["resv_flags"][nd]) >> abi.RESV_GROUP_SHIFT) & 63) & np.uint64(1)]
        assert m
        p, nd = m[0]
        assert o.commit(p, nd, sign=-1)[0] == abi.E_INVAL
        with pytest.raises(Exception):
            e.uncommit(p, nd)


def test_gpu_resv_update_nodes(Engine):
    """Informer deltas of reservation rows (a reservation appears / fills up)."""
    prof, t, pods = _workload(1000, 600, False)
    t2 = t.copy()
    rng = np.random.default_rng(3)
    idx = np.sort(rng.choice(t.n, 40, replace=False)).astype(np.int32)
    for i in idx:  # flip: drop a reservation or give a node a fresh one of group 1
        if t2["resv_flags"][i]:
            t2["resv_flags"][i] = 0
        else:
            t2["resv_flags"][i] = abi.RESV_PRESENT | abi.RESV_KEY_CPU | abi.RESV_KEY_MEM | (1 << abi.RESV_GROUP_SHIFT)
            t2["resv_alloc0"][i], t2["resv_alloc1"][i] = 8000, 16 << 30
            t2["resv_nz0"][i], t2["resv_nz1"][i] = 8000, 16 << 30
    ref = oracle.Oracle(to_c_config(prof), t2).place_stream(pods, threads=8)
    with Engine(prof, device=0) as e:
        e.load_snapshot(t)
        e.update_nodes(idx, t2.rows(idx))
        got = e.place_stream(pods)
    assert np.array_equal(ref, got)


@pytest.mark.parametrize("world", [2, 3])
def test_gpu_resv_sharded_group(Engine, world):
    """Node-index shards (the multi-GPU layout, here `world` contexts on one
    GPU): per-shard top-k of the Reservation ranking totals merged, then the
    replicated resolve -- every rank returns the unsharded placements."""
    from koordinator_amd.engine import place_stream_group
    prof, t, pods = _workload(2000, 800, True)
    engines = [Engine(prof, device=0) for _ in range(world)]
    try:
        for e in engines:
            e.load_snapshot(t)
        Engine.comm_init_local(engines)
        outs = place_stream_group(engines, pods)
        resv = [e.read_reservations() for e in engines]
    finally:
        for e in engines:
            e.close()
    o = oracle.Oracle(to_c_config(prof), t)
    ref = o.place_stream(pods, threads=8)
    for r in range(world):
        assert np.array_equal(outs[r], ref), (r, int(np.flatnonzero(outs[r] != ref)[0]))
        assert np.array_equal(resv[r]["allocated"], o.resv_state()["allocated"])


@pytest.mark.parametrize("numa,evalpath", [(False, "fused"), (True, "fused"), (False, "split")])
def test_gpu_resv_affinity_stream(Engine, numa, evalpath, monkeypatch):
    """Pods with a required reservation affinity (KOORDHIP_POD_RESV_AFFINITY):
    feasible only on nodes where a reservation matched them
    (reservation/plugin.go:378-381), through both evaluation paths; status,
    top-k and the placement stream vs the oracle."""
    monkeypatch.setenv("KOORDHIP_EVAL", evalpath)
    prof = shipped_profile(numa=numa, reservation=True)
    t = synth.make_cluster(synth.ClusterSpec(2500, seed=17), prof)
    if numa:
        synth.add_numa(t, synth.NumaSpec(), prof, seed=17)
    synth.add_reservations(t, synth.ResvSpec(node_frac=0.3, groups=4), seed=17)
    pods = synth.make_pods(synth.StreamSpec(2000, be_frac=0.3, seed=17, resv_match_frac=0.5, resv_groups=4,
                                            resv_affinity_frac=0.3), prof)
    assert (pods["flags"] & abi.POD_RESV_AFFINITY).sum() > 200
    o = oracle.Oracle(to_c_config(prof), t)
    rev = oracle.Oracle(to_c_config(prof), t).eval(pods[:32], k=16)
    ref = o.place_stream(pods, threads=8)
    with Engine(prof, device=0) as e:
        e.load_snapshot(t)
        got_eval = e.eval(pods[:32], k=16)
        got = e.place_stream(pods)
        assert np.array_equal(ref, got), np.flatnonzero(ref != got)[:10]
        _state_eq(e, o, numa)
    assert np.array_equal(rev["status"], got_eval["status"])
    assert np.array_equal(rev["topk"], got_eval["topk"])
    aff = (pods["flags"] & abi.POD_RESV_AFFINITY) != 0
    assert (ref[aff] >= 0).sum() > 50 and (ref[aff] < 0).sum() > 10
