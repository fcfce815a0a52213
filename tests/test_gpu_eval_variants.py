"""Compile-time variants of the fused evaluation kernel k_eval_topk that the
defaults do not run: G = 2 / 4 pods per workgroup (KOORDHIP_ETK_G, DESIGN.md
§4) on the plain (config-4 plugin set, forced fused), NUMA and Reservation
plugin sets, and lag 2 with NodeNUMAResource (KOORDHIP_LAG2).  Each stream is
bit-exact against the oracle."""
import numpy as np
import pytest

import oracle
from koordinator_amd import synth
from koordinator_amd.config import shipped_profile, to_c_config

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def Engine():
    import torch  # noqa: F401
    from koordinator_amd.engine import PlacementEngine
    return PlacementEngine


def _workload(kind, n, p, seed=11):
    numa, resv = kind in ("numa", "resv"), kind == "resv"
    prof = shipped_profile(numa=numa, reservation=resv)
    t = synth.make_cluster(synth.ClusterSpec(n, seed=seed), prof)
    if numa:
        synth.add_numa(t, synth.NumaSpec(), prof, seed=seed)
    if resv:
        synth.add_reservations(t, synth.ResvSpec(node_frac=0.3, groups=4), seed=seed)
    pods = synth.make_pods(synth.StreamSpec(p, be_frac=0.3, seed=seed, cpuset_frac=0.4 if kind == "numa" else 0.0,
                                            resv_match_frac=0.4 if resv else 0.0, resv_groups=4), prof)
    return prof, t, pods


@pytest.mark.parametrize("kind,g", [("plain", 2), ("plain", 4), ("numa", 4), ("resv", 2), ("resv", 4)])
def test_gpu_pods_per_workgroup_stream(Engine, kind, g, monkeypatch):
    monkeypatch.setenv("KOORDHIP_ETK_G", str(g))
    if kind == "plain":
        monkeypatch.setenv("KOORDHIP_EVAL", "fused")
    prof, t, pods = _workload(kind, 6000, 3000)
    ref = oracle.Oracle(to_c_config(prof), t).place_stream(pods, threads=8)
    with Engine(prof, device=0) as e:
        e.load_snapshot(t)
        got = e.place_stream(pods)
    assert np.array_equal(ref, got), np.flatnonzero(ref != got)[:10]


def test_gpu_numa_lag2_stream(Engine, monkeypatch):
    monkeypatch.setenv("KOORDHIP_LAG2", "1")
    prof, t, pods = _workload("numa", 3000, 3000)
    ref = oracle.Oracle(to_c_config(prof), t).place_stream(pods, threads=8)
    with Engine(prof, device=0) as e:
        e.load_snapshot(t)
        got = e.place_stream(pods)
        assert e.kernel_stats()["lag"] == 2
    assert np.array_equal(ref, got), np.flatnonzero(ref != got)[:10]


def test_gpu_wide_totals_asked_split_run_fused(Engine, monkeypatch):
    """BalancedAllocation weight 5 beside Reservation: ranking totals beyond the
    split path's u16 matrix (2^15).  KOORDHIP_EVAL=split no longer fails the
    create: the context runs the fused path (32-bit keys), bit-exact."""
    from koordinator_amd.config import with_upstream
    monkeypatch.setenv("KOORDHIP_EVAL", "split")
    prof0, t, pods = _workload("resv", 3000, 2000)
    prof = with_upstream(prof0, static_filters=(), balanced_weight=5)
    ref = oracle.Oracle(to_c_config(prof), t).place_stream(pods, threads=8)
    with Engine(prof, device=0) as e:
        e.load_snapshot(t)
        got = e.place_stream(pods)
        assert "eval_topk" in e.kernel_names()["eval"]
    assert np.array_equal(ref, got), np.flatnonzero(ref != got)[:10]
