"""NodeNUMAResource Filter / Reserve pinned by the reference's TestPlugin_Filter
and TestPlugin_Reserve (tests/golden/numa_plugin_cases.json, written by
tests/golden/make_numa_plugin_golden.py): the oracle on CPU, libkoordhip.so on
the GPU."""
import numpy as np
import pytest

import golden_cases as G
import oracle
from koordinator_amd import abi
from koordinator_amd.config import to_c_config
from koordinator_amd.numa import format_cpuset

FILTER = G.numa_plugin_cases("filter")
RESERVE = G.numa_plugin_cases("reserve")


@pytest.mark.parametrize("name,case", FILTER, ids=[c[0] for c in FILTER])
def test_filter_kat_oracle(name, case):
    prof, t, pod, _ = G.build_numa_plugin_case(case)
    st = oracle.Oracle(to_c_config(prof), t).eval(pod)["status"][0, 0]
    assert (st & abi.ST_NUMA_FAIL == 0) == case["want"], case["source"]


@pytest.mark.parametrize("name,case", RESERVE, ids=[c[0] for c in RESERVE])
def test_reserve_kat_oracle(name, case):
    prof, t, pod, topo = G.build_numa_plugin_case(case)
    rc, cpus = oracle.Oracle(to_c_config(prof), t).commit(pod, 0)
    assert (rc == 0) == case["want"], case["source"]
    if case["want"]:
        got = topo.cpus(cpus) if topo is not None else []
        assert format_cpuset(got) == format_cpuset(case["want_cpuset"]), case["source"]


@pytest.fixture(scope="module")
def Engine():
    import torch  # noqa: F401
    from koordinator_amd.engine import PlacementEngine
    return PlacementEngine


@pytest.mark.gpu
@pytest.mark.parametrize("name,case", FILTER, ids=[c[0] for c in FILTER])
def test_filter_kat_gpu(Engine, name, case):
    prof, t, pod, _ = G.build_numa_plugin_case(case)
    with Engine(prof, device=0) as e:
        e.load_snapshot(t)
        st = e.eval(pod)["status"][0, 0]
    assert (st & abi.ST_NUMA_FAIL == 0) == case["want"], case["source"]


@pytest.mark.gpu
@pytest.mark.parametrize("name,case", RESERVE, ids=[c[0] for c in RESERVE])
def test_reserve_kat_gpu(Engine, name, case):
    prof, t, pod, topo = G.build_numa_plugin_case(case)
    with Engine(prof, device=0) as e:
        e.load_snapshot(t)
        try:
            cpus = e.commit(pod, 0)
            ok = True
        except abi.KoordhipError as err:
            assert err.code == abi.E_RESERVE
            ok = False
    assert ok == case["want"], case["source"]
    if ok:
        got = topo.cpus(cpus) if topo is not None else []
        assert format_cpuset(got) == format_cpuset(case["want_cpuset"]), case["source"]


SCORE1 = G.numa_plugin_cases("score_node1")


@pytest.mark.parametrize("name,case", SCORE1, ids=[c[0] for c in SCORE1])
def test_score_node1_kat_oracle(name, case):
    """TestScoreWithAmplifiedCPUs, ratio-1.0 node: the Least/MostAllocated scorer."""
    prof, t, pod = G.build_numa_score_node1_case(case)
    assert oracle.Oracle(to_c_config(prof), t).eval(pod)["scores"][0, 2, 0] == case["want"], case["source"]


@pytest.mark.gpu
@pytest.mark.parametrize("name,case", SCORE1, ids=[c[0] for c in SCORE1])
def test_score_node1_kat_gpu(Engine, name, case):
    prof, t, pod = G.build_numa_score_node1_case(case)
    with Engine(prof, device=0) as e:
        e.load_snapshot(t)
        got = e.eval(pod)["scores"][0, 2, 0]
    assert got == case["want"], case["source"]


SCORE2 = G.numa_plugin_cases("score_node2")
FAMP = G.numa_plugin_cases("filter_amp")


@pytest.mark.parametrize("name,case", SCORE2, ids=[c[0] for c in SCORE2])
def test_score_node2_amplified_kat_oracle(name, case):
    """TestScoreWithAmplifiedCPUs, ratio-2.0 node: scoreWithAmplifiedCPUs and the
    amplified cpuset requests (scoring.go:95-168)."""
    prof, t, pod = G.build_numa_score_node1_case(case, node=2)
    assert oracle.Oracle(to_c_config(prof), t).eval(pod)["scores"][0, 2, 0] == case["want"], case["source"]


@pytest.mark.parametrize("name,case", FAMP, ids=[c[0] for c in FAMP])
def test_filter_amplified_kat_oracle(name, case):
    """TestFilterWithAmplifiedCPUs (plugin.go:326-363)."""
    prof, t, pod = G.build_numa_filter_amp_case(case)
    st = oracle.Oracle(to_c_config(prof), t).eval(pod)["status"][0, 0]
    assert (st & abi.ST_NUMA_FAIL == 0) == case["want"], case["source"]


@pytest.mark.gpu
@pytest.mark.parametrize("name,case", SCORE2, ids=[c[0] for c in SCORE2])
def test_score_node2_amplified_kat_gpu(Engine, name, case):
    prof, t, pod = G.build_numa_score_node1_case(case, node=2)
    with Engine(prof, device=0) as e:
        e.load_snapshot(t)
        got = e.eval(pod)["scores"][0, 2, 0]
    assert got == case["want"], case["source"]


@pytest.mark.gpu
@pytest.mark.parametrize("name,case", FAMP, ids=[c[0] for c in FAMP])
def test_filter_amplified_kat_gpu(Engine, name, case):
    prof, t, pod = G.build_numa_filter_amp_case(case)
    with Engine(prof, device=0) as e:
        e.load_snapshot(t)
        st = e.eval(pod)["status"][0, 0]
    assert (st & abi.ST_NUMA_FAIL == 0) == case["want"], case["source"]
