"""Writes resource_manager_cases.json: NodeNUMAResource resourceManager.Allocate
and NodeAllocation known-answer tests transcribed from the reference's table
tests (data only):

  plugins/nodenumaresource/resource_manager_test.go:34-589  TestResourceManagerAllocate
  plugins/nodenumaresource/node_allocation_test.go:122-169  getAvailableCPUs (maxRefCount 1 rows,
                                                            with and without preferred CPUs)

Allocate runs on the test's node (resource_manager_test.go:538-582): topology
buildCPUTopologyForTest(2, 1, 26, 2), NUMA nodes 0 / 1 with 52 cpu and 128Gi
each, NUMALeastAllocated, the case's earlier allocation (cpuset + per-NUMA
cpu; CPU 104 of "4-104" is outside the topology and ignored there too) and the
case's hint (NUMANodeAffinity).  Left out: the three amplification-ratio rows
(:338-477; the engine rejects CPU amplification on nodes with NUMA zones), and
from the first row the gpu-memory request (no NUMA zone holds it, so
allocateResourcesByHint skips it: :191-200).
"""
import json
import os


def case(name, src, hint, req_cpu, want, cpu_bind=False, policy="", need=0, allocated="", allocated_zones=(),
         want_cpuset=None, want_zones=None):
    return {"name": name, "source": src, "hint": list(hint), "req_cpu_m": req_cpu, "request_cpu_bind": cpu_bind,
            "policy": policy, "need": need, "allocated_cpuset": allocated, "allocated_zone_cpu_m": list(allocated_zones),
            "want": want, "want_cpuset": want_cpuset, "want_zone_cpu_m": want_zones}


R = "resource_manager_test.go:"
ALLOCATE = [
    case("allocate with non-existing resources in NUMA", R + "44-72", [0], 4000, True, want_zones={"0": 4000}),
    case("allocate with insufficient resources", R + "73-91", [0], 54000, False),
    case("allocate with required CPUBindPolicyFullPCPUs", R + "92-122", [0], 4000, True, True, "FullPCPUs", 4,
         want_cpuset="0-3", want_zones={"0": 4000}),
    case("allocate with required CPUBindPolicyFullPCPUs and allocated", R + "123-173", [0], 4000, True, True,
         "FullPCPUs", 4, "4-104", (48000, 52000), want_cpuset="0-3", want_zones={"0": 4000}),
    case("failed to allocate with required CPUBindPolicyFullPCPUs and allocated", R + "174-214", [0], 4000, False,
         True, "FullPCPUs", 4, "1,3,5,7-104", (48000, 52000)),
    case("allocate with required CPUBindPolicySpreadByPCPUs", R + "215-245", [0], 4000, True, True, "SpreadByPCPUs",
         4, want_cpuset="0,2,4,6", want_zones={"0": 4000}),
    case("allocate with required CPUBindPolicySpreadByPCPUs and allocated", R + "246-296", [0], 4000, True, True,
         "SpreadByPCPUs", 4, "1,3,5,7-104", (48000, 52000), want_cpuset="0,2,4,6", want_zones={"0": 4000}),
    case("failed to allocate with required CPUBindPolicySpreadByPCPUs and allocated", R + "297-337", [0], 4000, False,
         True, "SpreadByPCPUs", 4, "4-104", (48000, 52000)),
    case("allocate by numa hint on mixed cpuset/share node", R + "478-534", [0, 1], 8000, True, True, "FullPCPUs", 8,
         "0-43,53-96", (48000, 48000), want_cpuset="44-47,98-101", want_zones={"0": 4000, "1": 4000}),
]

N = "node_allocation_test.go:"
# (topology, allocations [(cpuset, exclusive policy)], released indices, preferred, want available), maxRefCount 1
AVAILABLE = [
    {"name": "getAvailableCPUs after a release", "source": N + "122-149", "topology": [2, 1, 4, 2],
     "allocations": [["1-4", "PCPULevel"], ["2-5", "PCPULevel"]], "released": [0], "preferred": "",
     "want": "0-1,6-15"},
    {"name": "getAvailableCPUs", "source": N + "151-164", "topology": [2, 1, 4, 2],
     "allocations": [["0-4", "PCPULevel"]], "released": [], "preferred": "", "want": "5-15"},
    {"name": "getAvailableCPUs with preferred cpus", "source": N + "166-168", "topology": [2, 1, 4, 2],
     "allocations": [["0-4", "PCPULevel"]], "released": [], "preferred": "1-2", "want": "1-2,5-15"},
]

if __name__ == "__main__":
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "resource_manager_cases.json")
    with open(out, "w") as f:
        json.dump({"allocate": ALLOCATE, "available": AVAILABLE}, f, indent=1)
    print(out)
