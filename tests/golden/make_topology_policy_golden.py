"""Writes topology_policy_cases.json: the topology manager's Merge known-answer
tests, transcribed from the reference's own table tests (data only):

  frameworkext/topologymanager/policy_test.go:60-342   commonPolicyMergeTestCases
  frameworkext/topologymanager/policy_test.go:344-610  bestEffortPolicy.mergeTestCases
                                                       (restrictedPolicy embeds it)
  frameworkext/topologymanager/policy_test.go:612-883  singleNumaNodePolicy.mergeTestCases
  frameworkext/topologymanager/policy_none_test.go:53-96
  policy_{best_effort,restricted,single_numa_node,none}_test.go canAdmitPodResult tables
  plugins/nodenumaresource/scoring_test.go:47-371      TestNUMANodeScore

Each provider is "provider-empty" (a nil or empty hint map) or a dict resource
-> "nil" | [] | [[numa ids | None, preferred], ...].  Expected hints are
[numa ids | None, preferred]; numaNodes = [0, 1] throughout.
"""
import json
import os

P = lambda *ids: list(ids)
E = "provider-empty"

COMMON = [  # policy_test.go:60-342
    ("Two providers, 1 hint each, same mask, both preferred 1/2",
     [{"resource1": [[P(0), True]]}, {"resource2": [[P(0), True]]}], [P(0), True]),
    ("Two providers, 1 hint each, same mask, both preferred 2/2",
     [{"resource1": [[P(1), True]]}, {"resource2": [[P(1), True]]}], [P(1), True]),
    ("Two providers, 1 no hints, 1 single hint preferred 1/2", [E, {"resource": [[P(0), True]]}], [P(0), True]),
    ("Two providers, 1 no hints, 1 single hint preferred 2/2", [E, {"resource": [[P(1), True]]}], [P(1), True]),
    ("Two providers, 1 with 2 hints, 1 with single hint matching 1/2",
     [{"resource1": [[P(0), True], [P(1), True]]}, {"resource2": [[P(0), True]]}], [P(0), True]),
    ("Two providers, 1 with 2 hints, 1 with single hint matching 2/2",
     [{"resource1": [[P(0), True], [P(1), True]]}, {"resource2": [[P(1), True]]}], [P(1), True]),
    ("Two providers, both with 2 hints, matching narrower preferred hint from both",
     [{"resource1": [[P(0), True], [P(1), True]]}, {"resource2": [[P(0), True], [P(0, 1), False]]}], [P(0), True]),
    ("Ensure less narrow preferred hints are chosen over narrower non-preferred hints",
     [{"resource1": [[P(1), True], [P(0, 1), False]]},
      {"resource2": [[P(0), True], [P(1), True], [P(0, 1), False]]}], [P(1), True]),
    ("Multiple resources, same provider",
     [{"resource1": [[P(1), True], [P(0, 1), False]],
       "resource2": [[P(0), True], [P(1), True], [P(0, 1), False]]}], [P(1), True]),
]

BEST_EFFORT = [  # policy_test.go:344-610
    ("NUMATopologyHint not set", [], [P(0, 1), True]),
    ("NUMATopologyHintProvider returns empty non-nil map[string][]NUMATopologyHint", [E], [P(0, 1), True]),
    ("NUMATopologyHintProvider returns -nil map[string][]NUMATopologyHint from provider",
     [{"resource": "nil"}], [P(0, 1), True]),
    ("NUMATopologyHintProvider returns empty non-nil map[string][]NUMATopologyHint from provider",
     [{"resource": []}], [P(0, 1), False]),
    ("Single NUMATopologyHint with Preferred as true and NUMANodeAffinity as nil",
     [{"resource": [[None, True]]}], [P(0, 1), True]),
    ("Single NUMATopologyHint with Preferred as false and NUMANodeAffinity as nil",
     [{"resource": [[None, False]]}], [P(0, 1), False]),
    ("Two providers, 1 hint each, no common mask",
     [{"resource1": [[P(0), True]]}, {"resource2": [[P(1), True]]}], [P(0, 1), False]),
    ("Two providers, 1 hint each, same mask, 1 preferred, 1 not 1/2",
     [{"resource1": [[P(0), True]]}, {"resource2": [[P(0), False]]}], [P(0), False]),
    ("Two providers, 1 hint each, same mask, 1 preferred, 1 not 2/2",
     [{"resource1": [[P(1), True]]}, {"resource2": [[P(1), False]]}], [P(1), False]),
    ("Two providers, 1 hint each, 1 wider mask, both preferred 1/2",
     [{"resource1": [[P(0), True]]}, {"resource2": [[P(0, 1), True]]}], [P(0), True]),
    ("Two providers, 1 with 2 hints, 1 with single non-preferred hint matching",
     [{"resource1": [[P(0), True], [P(1), True]]}, {"resource2": [[P(0, 1), False]]}], [P(0), False]),
    ("Two providers, 1 hint each, 1 wider mask, both preferred 1/2 (second)",
     [{"resource1": [[P(1), True]]}, {"resource2": [[P(0, 1), True]]}], [P(1), True]),
]

SINGLE = [  # policy_test.go:612-883
    ("NUMATopologyHint not set", [], [None, True]),
    ("NUMATopologyHintProvider returns empty non-nil map[string][]NUMATopologyHint", [E], [None, True]),
    ("NUMATopologyHintProvider returns -nil map[string][]NUMATopologyHint from provider",
     [{"resource": "nil"}], [None, True]),
    ("NUMATopologyHintProvider returns empty non-nil map[string][]NUMATopologyHint from provider",
     [{"resource": []}], [None, False]),
    ("Single NUMATopologyHint with Preferred as true and NUMANodeAffinity as nil",
     [{"resource": [[None, True]]}], [None, True]),
    ("Single NUMATopologyHint with Preferred as false and NUMANodeAffinity as nil",
     [{"resource": [[None, False]]}], [None, False]),
    ("Two providers, 1 hint each, no common mask",
     [{"resource1": [[P(0), True]]}, {"resource2": [[P(1), True]]}], [None, False]),
    ("Two providers, 1 hint each, same mask, 1 preferred, 1 not 1/2",
     [{"resource1": [[P(0), True]]}, {"resource2": [[P(0), False]]}], [None, False]),
    ("Two providers, 1 hint each, same mask, 1 preferred, 1 not 2/2",
     [{"resource1": [[P(1), True]]}, {"resource2": [[P(1), False]]}], [None, False]),
    ("Two providers, 1 with 2 hints, 1 with single non-preferred hint matching",
     [{"resource1": [[P(0), True], [P(1), True]]}, {"resource2": [[P(0, 1), False]]}], [None, False]),
    ("Single NUMA hint generation",
     [{"resource1": [[P(0, 1), True]],
       "resource2": [[P(0), True], [P(1), True], [P(0, 1), False]]}], [None, False]),
    ("One no-preference provider",
     [{"resource1": [[P(0), True], [P(1), True], [P(0, 1), False]]}, E], [P(0), True]),
]

NONE = [  # policy_none_test.go:53-96
    ("merged empty providers hints", [], [None, False]),
    ("merge with a single provider with a single preferred resource",
     [{"resource": [[P(0, 1), True]]}], [None, False]),
    ("merge with a single provider with a single non-preferred resource",
     [{"resource": [[P(0, 1), False]]}], [None, False]),
]

# TestNUMANodeScore (nodenumaresource/scoring_test.go:47-371): MostAllocated
# over cpu 1 / memory 1.  node: [name, cpu cores, memory Gi, policy label, NUMA
# node count]; the topology is buildCPUTopologyForTest(count, 1, cores/2/count,
# 2) with count zones of capacity/count each (:312-330); an existing pod is a
# NodeAllocation entry on zone 0 holding its requests, plus CPUs 0..cpu-1 when
# it is LSR (:331-352) -- not part of NodeInfo.Requested (no pods in the
# snapshot, :304).  pod: [cpu cores, memory Gi, LSR].
NUMA_NODE_SCORE = [
    ("single numa nodes score",
     [["test-node-1", 104, 256, "SingleNUMANode", 2], ["test-node-2", 64, 128, "SingleNUMANode", 1]],
     [21, 40, False], [], [35, 31]),
    ("restricted numa nodes score",
     [["test-node-1", 104, 256, "Restricted", 2], ["test-node-2", 64, 128, "Restricted", 1]],
     [54, 40, False], [], [33, 57]),
    ("restricted numa nodes score with same capacity",
     [["test-node-1", 104, 256, "Restricted", 2], ["test-node-2", 104, 256, "Restricted", 2]],
     [54, 40, False], [], [33, 33]),
    ("single numa nodes score with same capacity but different requested",
     [["test-node-1", 104, 256, "Restricted", 2], ["test-node-2", 104, 256, "Restricted", 2],
      ["test-node-3", 104, 256, "Restricted", 2]],
     [4, 40, False], [[0, 4, 8, False], [1, 8, 32, False], [2, 32, 40, False]], [26, 39, 65]),
    ("single numa nodes score with same capacity but different requested and LSR",
     [["test-node-1", 104, 256, "Restricted", 2], ["test-node-2", 104, 256, "Restricted", 2],
      ["test-node-3", 104, 256, "Restricted", 2]],
     [4, 40, True], [[0, 4, 8, False], [0, 4, 8, True], [1, 8, 32, False], [1, 8, 32, True],
                     [2, 16, 40, False], [2, 16, 40, True]], [29, 52, 65]),
]

# canAdmitPodResult tables: policy -> [(preferred, expected)]
ADMIT = {
    "best-effort": [[False, True], [True, True]],
    "restricted": [[False, False], [True, True]],
    "single-numa-node": [[False, False]],
    "none": [[False, True], [True, True]],
}


def cases(rows):
    return [{"name": n, "providers": p, "expected": e} for n, p, e in rows]


def main():
    out = {
        "numa_nodes": [0, 1],
        "merge": {
            "best-effort": cases(COMMON + BEST_EFFORT),
            "restricted": cases(COMMON + BEST_EFFORT),
            "single-numa-node": cases(COMMON + SINGLE),
            "none": cases(NONE),
        },
        "admit": ADMIT,
        "numa_node_score": [{"name": n, "nodes": nodes, "pod": pod, "existing": ex, "want": want}
                            for n, nodes, pod, ex, want in NUMA_NODE_SCORE],
    }
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "topology_policy_cases.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
