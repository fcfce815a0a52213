"""NUMA topology policies: the topology manager's Merge / admit pinned by the
reference's policy_test.go tables, and NodeNUMAResource Filter + Score on
policy nodes pinned by TestNUMANodeScore (tests/golden/topology_policy_cases.json,
written by tests/golden/make_topology_policy_golden.py)."""
import json
import os

import numpy as np
import pytest

import golden_cases as G
import oracle
from koordinator_amd import abi
from koordinator_amd.config import to_c_config

CASES = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "topology_policy_cases.json")))
POLICY = {"best-effort": abi.NUMA_TOPO_BEST_EFFORT, "restricted": abi.NUMA_TOPO_RESTRICTED,
          "single-numa-node": abi.NUMA_TOPO_SINGLE_NUMA_NODE, "none": abi.NUMA_TOPO_NONE}


def _mask(ids):
    return None if ids is None else sum(1 << i for i in ids)


def _entries(providers):
    """filterProvidersHints input order: providers in order, resources in the
    order listed (the merge result does not depend on it: the best hint is the
    unique minimum of (preferred, narrower))."""
    out = []
    for p in providers:
        if p == "provider-empty":
            out.append("provider-empty")
            continue
        for _, hints in p.items():
            if hints == "nil":
                out.append("nil")
            elif hints == []:
                out.append("empty")
            else:
                out.append([(_mask(m), pref) for m, pref in hints])
    return out


MERGE = [(pol, c) for pol, cs in CASES["merge"].items() for c in cs]


@pytest.mark.parametrize("pol,case", MERGE, ids=[f"{p}:{c['name']}" for p, c in MERGE])
def test_merge_kat(pol, case):
    admit, mask, pref = oracle.tm_merge(POLICY[pol], _mask(CASES["numa_nodes"]), _entries(case["providers"]))
    want_mask, want_pref = case["expected"]
    assert (mask, pref) == (_mask(want_mask), want_pref)
    want_admit = {"best-effort": True, "none": True}.get(pol, want_pref)
    assert admit == want_admit


@pytest.mark.parametrize("pol", sorted(CASES["admit"]))
def test_can_admit_pod_result(pol):
    """canAdmitPodResult on {nil, preferred}: merged from a single nil hint."""
    for pref, want in CASES["admit"][pol]:
        admit, _, _ = oracle.tm_merge(POLICY[pol], 0b11, [[(None, pref)]])
        assert admit == want, (pol, pref)


def test_merge_reference_quirk_intersection_of_two_resources():
    """Two identical resource lists can merge into a mask neither holds
    (mergePermutation ANDs one hint per list): 0011 & 0110 = 0010."""
    hints = [(0b0011, True), (0b0110, True), (0b1111, False)]
    admit, mask, pref = oracle.tm_merge(abi.NUMA_TOPO_RESTRICTED, 0b1111, [hints, hints])
    assert (admit, mask, pref) == (True, 0b0010, True)


@pytest.mark.parametrize("name,case", G.numa_node_score_cases(), ids=[c[0] for c in G.numa_node_score_cases()])
def test_numa_node_score_kat(name, case):
    """TestNUMANodeScore (scoring_test.go:47-371): Filter passes on every node,
    MostAllocated scores over the hinted zones."""
    prof, table, pod = G.build_numa_node_score_case(case)
    r = oracle.Oracle(to_c_config(prof), table).eval(pod)
    assert not (r["status"][0] & abi.ST_NUMA_FAIL).any()
    assert r["scores"][0, 2].tolist() == case["want"]


def test_hint_alloc_zones_single_numa():
    """allocateResourcesByHint on the TestNUMANodeScore 'single numa' node 1:
    zone 0 takes the whole request; a 1-zone node's hint equals the default
    affinity and turns nil (policy_single_numa_node.go:70-72)."""
    _, case = G.numa_node_score_cases()[0]
    prof, table, pod = G.build_numa_node_score_case(case)
    o = oracle.Oracle(to_c_config(prof), table)
    ok, mask, admit, zones = o.hint_alloc(pod, 0)
    assert ok and admit and mask == 0b01
    assert zones[0, 0] == 21000 and zones[1, 0] == 40 * 2**30 and not zones[:, 1:].any()
    ok, mask, admit, zones = o.hint_alloc(pod, 1)
    assert ok and admit and mask is None and not zones.any()


def test_reserve_advances_zone_used_and_cpus():
    """Reserve on a Restricted node: the zone amounts land in NodeAllocation
    (node_allocation.go:92-102) and the cpuset stays inside the hinted zone."""
    _, case = G.numa_node_score_cases()[4]
    prof, table, pod = G.build_numa_node_score_case(case)
    o = oracle.Oracle(to_c_config(prof), table)
    before = o.numa_state()["zone_used"][0].copy()
    rc, cpus = o.commit(pod, 0)
    assert rc == 0
    after = o.numa_state()["zone_used"][0]
    assert after[0, 0] - before[0, 0] == 4000 and after[1, 0] - before[1, 0] == 40 * 2**30
    from koordinator_amd.numa import reference_test_topology
    topo = reference_test_topology(2, 1, 26, 2)
    got = topo.cpus(cpus)
    assert len(got) == 4 and all(topo.details[c].node == 0 for c in got)
    rc, _ = o.commit(pod, 0, sign=-1, cpus=cpus)
    assert rc == abi.E_INVAL


def test_oracle_8_zone_streams_self_consistent():
    """The oracle on 2-socket NPS4 nodes (8 NUMA zones, every policy): a stream's
    final zone allocations equal the sum of what each pod's Reserve took."""
    import oracle
    from koordinator_amd import abi, synth
    from koordinator_amd.config import shipped_profile, to_c_config
    prof = shipped_profile(numa=True)
    t = synth.make_cluster(synth.ClusterSpec(200, seed=17), prof)
    synth.add_numa(t, synth.NumaSpec(policy_frac=0.9, nodes_per_socket=4), prof, seed=17)
    pods = synth.make_pods(synth.StreamSpec(300, be_frac=0.2, cpuset_frac=0.5), prof)
    o = oracle.Oracle(to_c_config(prof), t)
    out = o.place_stream(pods)
    assert (out >= 0).sum() > 200
    zu = o.numa_state()["zone_used"]
    assert zu[:, :, 4:].sum() > t["numa_zone_used"][:, :, 4:].sum()
