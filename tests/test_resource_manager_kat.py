"""resourceManager.Allocate and NodeAllocation pinned by the reference's
resource_manager_test.go / node_allocation_test.go tables
(tests/golden/resource_manager_cases.json, written by
tests/golden/make_resource_manager_golden.py): the oracle's Allocate with a
given hint (allocateResourcesByHint + allocateCPUSet) and the host's
getAvailableCPUs.  The device reaches the same Allocate through its
topology-manager merge; tests/test_gpu_topology_policy.py holds it to the
oracle on random streams."""
import numpy as np
import pytest

import golden_cases as G
import oracle
from koordinator_amd import abi
from koordinator_amd import numa as nm
from koordinator_amd.config import PLUGIN_NUMA, Profile, to_c_config
from koordinator_amd.snapshot import NodeTable, pod_array

CASES = G.load("resource_manager_cases.json")
ALLOCATE = [(c["name"], c) for c in CASES["allocate"]]
AVAILABLE = [(c["name"], c) for c in CASES["available"]]
BIND = {"": 0, "FullPCPUs": 1, "SpreadByPCPUs": 2}
GI = 2**30


def _allocate_case(c):
    """resource_manager_test.go:538-582: one node, topology (2, 1, 26, 2), NUMA
    nodes of 52 cpu / 128Gi, NUMALeastAllocated, the case's earlier allocation."""
    prof = Profile(filters=(PLUGIN_NUMA,), scores={PLUGIN_NUMA: 1})
    topo = nm.reference_test_topology(2, 1, 26, 2)
    t = NodeTable.empty(1)
    t["alloc0"][0], t["alloc1"][0] = 104000, 256 * GI
    t["alloc_pods"][0] = 110
    ct = nm.ClassTable()
    t["numa_class"][0] = ct.add(topo)
    t.numa_classes = ct.records()
    alloc = nm.NodeAllocation()
    held = [x for x in nm.parse_cpuset(c["allocated_cpuset"]) if x in topo.pos_of] if c["allocated_cpuset"] else []
    zres = [(k, {"cpu": v}) for k, v in enumerate(c["allocated_zone_cpu_m"])]
    if held or zres:
        alloc.add("123456", held, "", zres)
    free = topo.mask(nm.available_cpus(topo, alloc))
    for w in range(abi.NUMA_WORDS):
        t[f"numa_free{w}"][0] = free[w]
    t["numa_alloc_cnt"][0] = len(held)
    t["numa_zone_alloc"][0] = nm.zone_row([(52000, 128 * GI)] * 2)
    t["numa_zone_used"][0] = nm.zone_row([(alloc.resources.get(k, {}).get("cpu", 0), 0) for k in range(2)])
    t["numa_flags"][0] = nm.node_numa_flags({}, None, False)   # NUMALeastAllocated
    p = pod_array(1)
    p["req"][0, abi.RES_CPU] = c["req_cpu_m"]
    p["nz_cpu_m"][0] = c["req_cpu_m"]
    p["flags"][0] = abi.POD_HAS_REQ | (abi.POD_CPUSET if c["request_cpu_bind"] else 0)
    if c["request_cpu_bind"]:
        p["numa_cpus"][0] = c["need"]
        p["numa_policy"][0] = abi.numa_policy(BIND[c["policy"]], BIND[c["policy"]], 0)
    return prof, t, p, topo


@pytest.mark.parametrize("name,c", ALLOCATE, ids=[x[0] for x in ALLOCATE])
def test_allocate_with_hint_kat(name, c):
    prof, t, p, topo = _allocate_case(c)
    mask = sum(1 << k for k in c["hint"])
    ok, zones, cpus = oracle.Oracle(to_c_config(prof), t).numa_allocate_hint(p, 0, mask)
    assert ok == c["want"], c["source"]
    if not ok:
        return
    assert nm.format_cpuset(topo.cpus(cpus)) == (c["want_cpuset"] or ""), c["source"]
    got = {str(k): int(zones[0, k]) for k in range(abi.NUMA_MAX_NODES) if zones[0, k]}
    assert got == c["want_zone_cpu_m"], c["source"]


@pytest.mark.parametrize("name,c", AVAILABLE, ids=[x[0] for x in AVAILABLE])
def test_available_cpus_kat(name, c):
    topo = nm.reference_test_topology(*c["topology"])
    alloc = nm.NodeAllocation()
    for j, (cs, ex) in enumerate(c["allocations"]):
        alloc.add(f"pod-{j}", nm.parse_cpuset(cs), ex, [])
    for j in c["released"]:
        alloc.release(f"pod-{j}")
    pref = nm.parse_cpuset(c["preferred"]) if c["preferred"] else []
    got = nm.available_cpus(topo, alloc, preferred=pref)
    assert nm.format_cpuset(got) == c["want"], c["source"]


def test_node_allocation_add_release():
    """TestNodeAllocationAddCPUs / ReleaseCPUs (node_allocation_test.go:33-120):
    an allocation is added once (a second add of the same UID is a no-op),
    RefCount counts the pods holding a CPU, the exclusive policy is the last
    pod's, and release drops CPUs whose count reaches 0."""
    alloc = nm.NodeAllocation()
    alloc.add("a", nm.parse_cpuset("1-4"), "PCPULevel", [])
    alloc.add("a", nm.parse_cpuset("1-4"), "PCPULevel", [])
    assert {c: v[0] for c, v in alloc.cpus.items()} == {1: 1, 2: 1, 3: 1, 4: 1}
    alloc.add("b", nm.parse_cpuset("2-5"), "PCPULevel", [])
    assert {c: v[0] for c, v in alloc.cpus.items()} == {1: 1, 2: 2, 3: 2, 4: 2, 5: 1}
    assert all(v[1] == "PCPULevel" for v in alloc.cpus.values())
    alloc.release("a")
    alloc.release("b")
    assert alloc.cpus == {} and alloc.pods == {}
