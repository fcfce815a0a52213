"""Full-size parity of the BASELINE configurations through libkoordhip.so.

* config 4 (the headline: 50k nodes x 100k pods) and config 5 (200k nodes
  with reservations + NUMA x 100k pods) against committed golden placements +
  final-state digests (tests/golden/make_stream_golden.py ran the oracle on
  the exact bench.py workloads);
* config 2 (5k x 10k) and config 3 (5k 2-socket nodes x 10k pods with
  NodeNUMAResource cpusets) against the live oracle;
* the size-dependent launch shapes the small streams never reach: the split
  select with several tiles per workgroup (KOORDHIP_SEL_G=1/2 on 20k nodes),
  thousands of rounds of the persistent resolve.
"""
import hashlib
import os

import numpy as np
import pytest

import oracle
from koordinator_amd import abi, synth
from koordinator_amd.config import shipped_profile, to_c_config

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def Engine():
    import torch  # noqa: F401  (device discovery only; the engine is plain HIP)
    from koordinator_amd.engine import PlacementEngine
    return PlacementEngine


def pods_v4(pods):
    """The records as the fixture's ABI wrote them: the POD_KEY_* bits (ABI v5,
    read only by the Reservation plugin, which this workload does not enable)
    masked out."""
    from koordinator_amd import abi
    p = pods.copy()
    p["flags"] &= np.uint32(~(abi.POD_KEY_CPU | abi.POD_KEY_MEM) & 0xFFFFFFFF)
    return p


def _sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _first_diff(a, b):
    bad = np.flatnonzero(a != b)
    return None if len(bad) == 0 else (int(bad[0]), int(a[bad[0]]), int(b[bad[0]]), len(bad))


def test_config4_headline_stream_matches_golden(Engine):
    """50k nodes x 100k pods, the stream bench.py times: every placement and
    every final mutable node column equal the oracle's."""
    g = np.load(os.path.join(GOLDEN, "stream_config4.npz"))
    prof = shipped_profile()
    table, pods = synth.config_workload(4, prof)
    # the generator must reproduce the bytes the golden file was made from
    want_in = dict(zip(g["input_keys"].tolist(), g["input_sha"].tolist()))
    got_in = {c: _sha(table[c]) for c in table.cols if c in want_in}
    got_in["__pods__"] = _sha(pods_v4(pods))
    assert got_in == want_in
    from koordinator_amd.snapshot import NodeTable
    blank = NodeTable.empty(1)
    for c in set(table.cols) - set(want_in):  # columns added since: their defaults for this workload
        assert (table[c] == blank[c].flat[0]).all(), c
    with Engine(prof, device=0) as e:
        e.load_snapshot(table)
        got = e.place_stream(pods)
        state = e.read_nodes()
    ref = g["placements"]
    assert len(got) == 100000 and table.n == 50000
    assert np.array_equal(got, ref), _first_diff(got, ref)
    want_st = dict(zip(g["state_keys"].tolist(), g["state_sha"].tolist()))
    assert {k: _sha(v) for k, v in state.items()} == want_st


def test_config4_repeated_steps_identical(Engine):
    """bench.py's step (restore + place_staged) gives the golden placements on
    every repetition (the device restore and the pipeline state reset)."""
    g = np.load(os.path.join(GOLDEN, "stream_config4.npz"))
    prof = shipped_profile()
    table, pods = synth.config_workload(4, prof)
    with Engine(prof, device=0) as e:
        e.load_snapshot(table)
        e.checkpoint()
        e.stage_pods(pods)
        for _ in range(3):
            e.restore()
            e.place_staged()
            got = e.fetch_placements(len(pods))
            assert np.array_equal(got, g["placements"]), _first_diff(got, g["placements"])


def test_config5_stream_matches_golden(Engine):
    """BASELINE config 5: 200k nodes (10% holding an Available Reservation) x
    100k pods (20% matching a reservation owner), Fit + LoadAware +
    NodeNUMAResource + Reservation: every placement and the digests of every
    final node / NUMA / reservation column equal the oracle's (fixture made by
    tests/golden/make_stream_golden.py --config 5, ~45 min of oracle time)."""
    g = np.load(os.path.join(GOLDEN, "stream_config5.npz"))
    prof = shipped_profile(numa=True, reservation=True)
    table, pods = synth.config_workload(5, prof)
    want_in = dict(zip(g["input_keys"].tolist(), g["input_sha"].tolist()))
    got_in = {c: _sha(table[c]) for c in table.cols if c in want_in}
    got_in["__pods__"] = _sha(pods)
    assert got_in == want_in
    with Engine(prof, device=0) as e:
        e.load_snapshot(table)
        got = e.place_stream(pods)
        cpus = e.fetch_cpusets(len(pods))
        state = e.read_nodes()
        state.update({"numa." + k: v for k, v in e.read_numa().items()})
        state.update({"resv." + k: v for k, v in e.read_reservations().items()})
    state["__cpusets__"] = cpus
    ref = g["placements"]
    assert len(got) == 100000 and table.n == 200000
    assert np.array_equal(got, ref), _first_diff(got, ref)
    want_st = dict(zip(g["state_keys"].tolist(), g["state_sha"].tolist()))
    assert {k: _sha(state[k]) for k in want_st} == want_st


def test_config2_full_stream(Engine):
    """BASELINE config 2: 5k nodes x 10k LS pods, the whole stream + final state."""
    prof = shipped_profile()
    table, pods = synth.config_workload(2, prof)
    with Engine(prof, device=0) as e:
        e.load_snapshot(table)
        got = e.place_stream(pods)
        state = e.read_nodes()
    o = oracle.Oracle(to_c_config(prof), table)
    ref = o.place_stream(pods)
    assert np.array_equal(got, ref), _first_diff(got, ref)
    rs = o.state()
    for k in rs:
        assert np.array_equal(state[k], rs[k]), k


def test_config3_full_numa_stream(Engine):
    """BASELINE config 3: 5k 2-socket nodes x 10k pods (50% of LS pods LSR/LSE
    cpuset): placements, Reserve failures, the exact cpusets, final state."""
    prof = shipped_profile(numa=True)
    table, pods = synth.config_workload(3, prof)
    assert (pods["flags"] & abi.POD_CPUSET).sum() > 3000
    with Engine(prof, device=0) as e:
        e.load_snapshot(table)
        got = e.place_stream(pods)
        cpus = e.fetch_cpusets(len(pods))
        state = e.read_nodes()
        nstate = e.read_numa()
    o = oracle.Oracle(to_c_config(prof), table)
    ref, rcpus = o.place_stream(pods, cpusets=True)
    assert np.array_equal(got, ref), _first_diff(got, ref)
    assert np.array_equal(cpus, rcpus)
    rs = o.state()
    for k in rs:
        assert np.array_equal(state[k], rs[k]), k
    rn = o.numa_state()
    for k in rn:
        assert np.array_equal(nstate[k], rn[k]), k


@pytest.mark.parametrize("sel_g", ["1", "2"])
def test_split_select_multi_tile(Engine, monkeypatch, sel_g):
    """20k nodes = 5 select tiles: with 1-2 workgroups per pod each walks
    several tiles (the pass-1 / pass-2 reloads and the early break)."""
    monkeypatch.setenv("KOORDHIP_SEL_G", sel_g)
    prof = shipped_profile()
    table = synth.make_cluster(synth.ClusterSpec(20000), prof)
    pods = synth.make_pods(synth.StreamSpec(2000, be_frac=0.3), prof)
    with Engine(prof, device=0) as e:
        e.load_snapshot(table)
        got = e.place_stream(pods)
    ref = oracle.Oracle(to_c_config(prof), table).place_stream(pods)
    assert np.array_equal(got, ref), _first_diff(got, ref)
