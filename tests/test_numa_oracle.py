"""NodeNUMAResource oracle pinned by the reference's cpu_accumulator_test.go
tables (tests/golden/cpu_accumulator.json), plus the topology model."""
import json
import os

import numpy as np
import pytest

import oracle
import golden_cases as G
from koordinator_amd import abi
from koordinator_amd.config import to_c_config
from koordinator_amd.numa import (Topology, TopologyError, CPUInfo, format_cpuset, linux_topology, parse_cpuset,
                                  reference_test_topology)

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "cpu_accumulator.json")))
POL = {"FullPCPUs": abi.CPUBIND_FULL_PCPUS, "SpreadByPCPUs": abi.CPUBIND_SPREAD_BY_PCPUS}
EXCL = {"None": abi.CPUEXCL_NONE, "PCPULevel": abi.CPUEXCL_PCPU, "NUMANodeLevel": abi.CPUEXCL_NUMA}


@pytest.mark.parametrize("case", GOLDEN["take_cpus"], ids=[c["name"] for c in GOLDEN["take_cpus"]])
def test_take_cpus_golden(case):
    topo = reference_test_topology(*case["topology"])
    allocated = parse_cpuset(case["allocated"])
    avail = topo.mask([c for c in topo.cpu_of if c not in allocated])
    amask = topo.mask(allocated)
    ae = case["allocated_exclusive_policy"]
    got = oracle.take_cpus(topo.record, avail, case["need"], POL[case["bind_policy"]], EXCL[case["exclusive_policy"]],
                           case["strategy"] == "MostAllocated",
                           excl_pcpu=amask if ae == "PCPULevel" else None,
                           excl_numa=amask if ae == "NUMANodeLevel" else None)
    if case["want_error"]:
        assert got is None
        return
    assert got is not None, case["source"]
    assert format_cpuset(topo.cpus(got)) == format_cpuset(parse_cpuset(case["want"])), case["source"]


@pytest.mark.parametrize("case", GOLDEN["spread_order"], ids=[c["name"] for c in GOLDEN["spread_order"]])
def test_spread_order_golden(case):
    topo = reference_test_topology(*case["topology"])
    got = oracle.spread_order(topo.record, topo.all_mask(), case["strategy"] == "MostAllocated")
    assert got == case["want"], case["source"]


def test_topology_model():
    t = linux_topology(2, 1, 24, 2)
    assert (t.num_cpus, t.num_cores, t.num_nodes, t.num_sockets, t.cpus_per_core) == (96, 48, 2, 2, 2)
    # core-major positions: siblings (c, c + 48) adjacent
    assert t.cpu_of[:4] == [0, 48, 1, 49]
    assert t.cpus(t.mask([5, 53, 90])) == [5, 53, 90]
    assert parse_cpuset("0-3,8,10-11") == [0, 1, 2, 3, 8, 10, 11]
    assert format_cpuset([0, 1, 2, 3, 8, 10, 11]) == "0-3,8,10-11"
    with pytest.raises(TopologyError):
        Topology([CPUInfo(0, 0, 0, 0), CPUInfo(1, 0, 0, 0), CPUInfo(2, 1, 0, 0)])  # non-uniform cores


def test_take_cpus_never_exceeds_avail_and_counts():
    rng = np.random.default_rng(3)
    topo = linux_topology(2, 2, 8, 2)
    for _ in range(300):
        free = [c for c in topo.cpu_of if rng.random() < 0.6]
        need = int(rng.integers(1, 20))
        pol = int(rng.integers(1, 3))
        got = oracle.take_cpus(topo.record, topo.mask(free), need, pol, int(rng.integers(0, 3)), bool(rng.random() < .5))
        if need > len(free):
            assert got is None
        else:
            assert got is not None
            cs = topo.cpus(got)
            assert len(cs) == need and set(cs) <= set(free)


@pytest.mark.parametrize("name,case", G.numa_score_cases(), ids=[c[0] for c in G.numa_score_cases()])
def test_numa_score_kat(name, case):
    """TestPlugin_Score (scoring_test.go:373-595): MostAllocated NodeNUMAResource score."""
    prof, table, pod = G.build_numa_score_case(case)
    got = oracle.Oracle(to_c_config(prof), table).eval(pod)["scores"][0, 2, 0]
    assert got == case["want"], case["source"]


def _seven_socket_case():
    """7 sockets x 1 node x 2 cores x 2 threads; sockets 0-5 have one free core
    (2 CPUs), socket 6 both (4 CPUs); MostAllocated orders the sockets 0..5, 6
    (fewest free first, id asc); need 8 FullPCPUs > CPUsPerSocket skips to the
    whole-socket pass (cpu_accumulator.go:141-155), whose len-desc sort.Slice
    in go 1.18 (go.mod:3) moves socket 0 to the END with its gap-6 shell pass:
    Go takes sockets 6, 1, 2 where a stable sort would take 6, 0, 1."""
    topo = reference_test_topology(7, 1, 2, 2)
    free = [24, 25, 26, 27] + [c for s in range(6) for c in (4 * s, 4 * s + 1)]
    return topo, free, [4, 5, 8, 9, 24, 25, 26, 27]


def test_take_cpus_go118_unstable_socket_sort():
    topo, free, want = _seven_socket_case()
    got = oracle.take_cpus(topo.record, topo.mask(free), 8, abi.CPUBIND_FULL_PCPUS, abi.CPUEXCL_NONE, True)
    assert got is not None
    assert topo.cpus(got) == want
