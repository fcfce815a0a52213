"""The lag-1 round pipeline of koordhip_place_staged, modelled on CPU with the
oracle (tests/lag_model.py): lists built two rounds stale, refreshed on the
previous round's nodes, resolved with k_resolve's rules -- must equal the
sequential greedy bit for bit.  Checks the algorithm independently of the
kernels (the GPU parity tests check the kernels against the oracle)."""
import numpy as np
import pytest

import oracle
from koordinator_amd import synth
from koordinator_amd.config import shipped_profile, to_c_config
from lag_model import place_lagged


@pytest.mark.parametrize("n_nodes,n_pods,batch,be", [(300, 600, 8, 0.3), (40, 300, 16, 0.5), (5, 120, 4, 0.3),
                                                     (500, 400, 64, 0.3)])
def test_lag_model_fit_loadaware(n_nodes, n_pods, batch, be):
    prof = shipped_profile()
    table = synth.make_cluster(synth.ClusterSpec(n_nodes), prof)
    pods = synth.make_pods(synth.StreamSpec(n_pods, be_frac=be), prof)
    cfg = to_c_config(prof)
    ref = oracle.Oracle(cfg, table).place_stream(pods)
    assert np.array_equal(place_lagged(cfg, table, pods, batch), ref)


@pytest.mark.parametrize("n_nodes,n_pods,batch,cpuset_frac,scoring", [
    (600, 1000, 64, 0.5, "LeastAllocated"), (300, 800, 17, 0.8, "LeastAllocated"),
    (60, 400, 8, 0.9, "LeastAllocated"), (300, 800, 17, 0.6, "MostAllocated")])
def test_lag_model_numa(n_nodes, n_pods, batch, cpuset_frac, scoring):
    prof = shipped_profile(numa=True)
    prof.numa.scoring_type = scoring
    table = synth.make_cluster(synth.ClusterSpec(n_nodes), prof)
    synth.add_numa(table, synth.NumaSpec(), prof)
    pods = synth.make_pods(synth.StreamSpec(n_pods, be_frac=0.2, cpuset_frac=cpuset_frac), prof)
    cfg = to_c_config(prof)
    ref = oracle.Oracle(cfg, table).place_stream(pods)
    assert np.array_equal(place_lagged(cfg, table, pods, batch), ref)
