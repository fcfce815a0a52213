"""Pins for the pipeline faults fixed in round 2 (VERDICT r02 "What's weak" 7).

1. The profiled-stream stall: with profile_kernels on, every timed event held
   a runtime signal and the host thread could wait for one queued behind the
   persistent resolve, which itself waited for rounds the thread had not
   enqueued yet.  A >= 4k-round stream under the config-5 plugin set
   (Fit + LoadAware + NUMA + Reservation, reduced nodes) with the per-launch
   timing on must finish and place exactly like the oracle.
2. The lag-2 batch fallback: lag 2 needs 3 x batch list slots per pod in the
   resolve; a batch of 33-64 pods must fall back to lag 1 (not an invalid
   launch) and still place exactly like the oracle.
"""
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


def test_profiled_4k_round_config5_stream(Engine):
    prof = shipped_profile(numa=True, reservation=True)
    prof.batch_pods = 8
    n_nodes, n_pods = 1200, 33000
    t = synth.make_cluster(synth.ClusterSpec(n_nodes, seed=11), prof)
    synth.add_numa(t, synth.NumaSpec(), prof, seed=11)
    synth.add_reservations(t, synth.ResvSpec(node_frac=0.1, groups=4, ordered_frac=0.05), seed=11)
    pods = synth.make_pods(synth.StreamSpec(n_pods, be_frac=0.3, seed=11, resv_match_frac=0.2, resv_groups=4), prof)
    o = oracle.Oracle(to_c_config(prof), t)
    ref = o.place_stream(pods, threads=8)
    with Engine(prof, device=0, profile_kernels=True) as e:
        e.load_snapshot(t)
        got = e.place_stream(pods)
        ks = e.kernel_stats()
    assert ks["rounds"] >= 4000, ks
    assert ks["scan_launches"] > 0 and ks["resolve_launches"] >= 1, ks
    assert np.array_equal(got, ref), int(np.flatnonzero(got != ref)[0])


@pytest.mark.parametrize("batch", [33, 48, 64])
def test_lag2_large_batch_falls_back_to_lag1(Engine, batch):
    prof = shipped_profile()
    prof.batch_pods = batch
    t = synth.make_cluster(synth.ClusterSpec(2000, seed=3), prof)
    pods = synth.make_pods(synth.StreamSpec(3000, be_frac=0.3, seed=3), prof)
    ref = oracle.Oracle(to_c_config(prof), t).place_stream(pods)
    with Engine(prof, device=0, profile_kernels=True) as e:
        e.load_snapshot(t)
        got = e.place_stream(pods)
        ks = e.kernel_stats()
    assert ks["round_pods"] == batch, ks
    assert ks["lag"] == 1, ks
    assert np.array_equal(got, ref), int(np.flatnonzero(got != ref)[0])
