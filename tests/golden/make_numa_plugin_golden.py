"""Writes numa_plugin_cases.json: NodeNUMAResource Filter and Reserve known-answer
tests transcribed from the reference's table tests (data only):

  plugins/nodenumaresource/plugin_test.go:544-812   TestPlugin_Filter
  plugins/nodenumaresource/plugin_test.go:927-1146  TestPlugin_Reserve
  plugins/nodenumaresource/scoring_test.go:597-852  TestScoreWithAmplifiedCPUs, the node1
                                                    (ratio 1.0) and node2 (ratio 2.0) columns
  plugins/nodenumaresource/plugin_test.go:814-925   TestFilterWithAmplifiedCPUs

Every case runs on the tests' node (allocatable cpu 96, memory 512Gi) with the
case's CPU topology (buildCPUTopologyForTest args; "invalid" = &CPUTopology{},
null = none) and, for a node with a topology policy, one NRT zone per NUMA
node of CPUsPerNode cores and 32Gi (:775-782).  The pod is the case's
preFilterState: requests cpu = numCPUsNeeded cores (:795-797), bind policies.
Left out: the missing-preFilterState rows (a framework error before any plugin
logic), the amplification-ratio rows (:705-738; the engine rejects ratios > 1
at marshal time) and the reservation-reserved-CPUs row (:1044-1058).
"""
import json
import os

NODE_BIND = "node.koordinator.sh/cpu-bind-policy"
NUMA_POLICY = "node.koordinator.sh/numa-topology-policy"
NUMA_STRATEGY = "node.koordinator.sh/numa-allocate-strategy"
KUBELET_FULL = {"policy": "static", "options": {"full-pcpus-only": "true"}}


def case(name, src, want, topology=(2, 1, 4, 2), labels=None, kubelet=None, cpu_bind=True, required="",
         preferred="", need=0, allocated=(), want_cpuset=None):
    return {"name": name, "source": src, "topology": list(topology) if isinstance(topology, tuple) else topology,
            "labels": labels or {}, "kubelet_policy": kubelet, "request_cpu_bind": cpu_bind, "required": required,
            "preferred": preferred, "need": need, "allocated_cpus": list(allocated), "want": want,
            "want_cpuset": want_cpuset}


F = "plugin_test.go:"
FILTER = [
    case("error with missing CPUTopology", F + "560-565", False, topology=None),
    case("error with invalid cpu topology", F + "566-574", False, topology="invalid"),
    case("succeed with valid cpu topology", F + "575-583", True),
    case("succeed with skip", F + "584-590", True, topology=None, cpu_bind=False),
    case("verify FullPCPUsOnly with SMTAlignmentError", F + "591-604", False,
         labels={NODE_BIND: "FullPCPUsOnly"}, preferred="FullPCPUs", need=5),
    case("verify required FullPCPUs SMTAlignmentError", F + "605-616", False, required="FullPCPUs",
         preferred="FullPCPUs", need=5),
    case("verify FullPCPUsOnly with preferred SpreadByPCPUs", F + "617-630", False,
         labels={NODE_BIND: "FullPCPUsOnly"}, preferred="SpreadByPCPUs", need=4),
    case("verify FullPCPUsOnly with required SpreadByPCPUs", F + "631-645", False,
         labels={NODE_BIND: "FullPCPUsOnly"}, required="SpreadByPCPUs", preferred="SpreadByPCPUs", need=4),
    case("verify Kubelet FullPCPUsOnly with SMTAlignmentError", F + "646-662", False, kubelet=KUBELET_FULL,
         preferred="FullPCPUs", need=5),
    case("verify Kubelet FullPCPUsOnly with RequiredFullPCPUsPolicy", F + "663-679", False, kubelet=KUBELET_FULL,
         preferred="SpreadByPCPUs", need=4),
    case("verify required FullPCPUs with none NUMA topology policy", F + "680-690", True, required="FullPCPUs",
         preferred="FullPCPUs", need=4),
    case("verify FullPCPUs with NUMA Topology Policy", F + "691-704", True,
         labels={NUMA_POLICY: "SingleNUMANode"}, required="FullPCPUs", preferred="FullPCPUs", need=4),
]

RESERVE = [
    case("error with missing allocationState", F + "945-952", False, topology=None),
    case("error with invalid cpu topology", F + "953-961", False, topology="invalid"),
    case("succeed with skip", F + "962-969", True, topology=None, cpu_bind=False, want_cpuset=[]),
    case("succeed with valid cpu topology", F + "970-981", True, preferred="FullPCPUs", need=4,
         want_cpuset=[0, 1, 2, 3]),
    case("allocated by node cpu bind policy", F + "982-1001", True, labels={NODE_BIND: "SpreadByPCPUs"},
         preferred="FullPCPUs", need=4, want_cpuset=[0, 2, 4, 6]),
    case("error with big request cpu", F + "1002-1011", False, need=24),
    case("succeed with valid cpu topology and node numa least allocate strategy", F + "1012-1027", True,
         topology=(2, 1, 8, 2), labels={NUMA_STRATEGY: "LeastAllocated"}, preferred="FullPCPUs", need=4,
         allocated=(0, 1, 2, 3), want_cpuset=[16, 17, 18, 19]),
    case("succeed with valid cpu topology and node numa most allocate strategy", F + "1028-1043", True,
         topology=(2, 1, 8, 2), labels={NUMA_STRATEGY: "MostAllocated"}, preferred="FullPCPUs", need=4,
         allocated=(0, 1, 2, 3), want_cpuset=[4, 5, 6, 7]),
]


# TestScoreWithAmplifiedCPUs node1: allocatable cpu 32 / memory 40Gi, the
# requested pod cpu 8 / memory 16Gi at prod priority (cpuset = LSR, default
# preferred FullPCPUs), an existing pod cpu 20 / memory 4Gi in NodeInfo (LSR:
# CPUs 0-19 allocated, plugin_test.go:117-130), buildCPUTopologyForTest(2, 1, 8, 2)
# when the node has an NRT (scoring_test.go:807-830).
S = "scoring_test.go:"
SCORE_NODE1 = [
    {"name": "ScoringStrategy MostAllocated, no cpuset pod", "source": S + "609-624", "scoring": "MostAllocated",
     "has_nrt": False, "existing": False, "existing_cpuset": False, "pod_cpuset": False, "want": 0},
    {"name": "ScoringStrategy MostAllocated, cpuset pods on node", "source": S + "625-649",
     "scoring": "MostAllocated", "has_nrt": True, "existing": True, "existing_cpuset": True, "pod_cpuset": False,
     "want": 68},
    {"name": "ScoringStrategy MostAllocated, scheduling cpuset pod", "source": S + "650-674",
     "scoring": "MostAllocated", "has_nrt": True, "existing": True, "existing_cpuset": False, "pod_cpuset": True,
     "want": 37},
    {"name": "ScoringStrategy MostAllocated, cpuset pods on node, scheduling cpuset pod", "source": S + "675-699",
     "scoring": "MostAllocated", "has_nrt": True, "existing": True, "existing_cpuset": True, "pod_cpuset": True,
     "want": 68},
    {"name": "ScoringStrategy LeastAllocated, no cpuset pod", "source": S + "700-719", "scoring": "LeastAllocated",
     "has_nrt": False, "existing": True, "existing_cpuset": False, "pod_cpuset": False, "want": 0},
    {"name": "ScoringStrategy LeastAllocated, cpuset pods on node", "source": S + "720-744",
     "scoring": "LeastAllocated", "has_nrt": True, "existing": True, "existing_cpuset": True, "pod_cpuset": False,
     "want": 31},
    {"name": "ScoringStrategy LeastAllocated, scheduling cpuset pod", "source": S + "745-769",
     "scoring": "LeastAllocated", "has_nrt": True, "existing": True, "existing_cpuset": False, "pod_cpuset": True,
     "want": 62},
    {"name": "ScoringStrategy LeastAllocated, cpuset pods on node,scheduling cpuset pod", "source": S + "770-794",
     "scoring": "LeastAllocated", "has_nrt": True, "existing": True, "existing_cpuset": True, "pod_cpuset": True,
     "want": 31},
]


# TestScoreWithAmplifiedCPUs node2: cpu 64 (= Amplify(32 CPUs, 2.0)), memory
# 60Gi, ratio 2.0, same pods and topology as node1 (scoring_test.go:610-794).
SCORE_NODE2 = [dict(c, want=w) for c, w in zip(SCORE_NODE1, [0, 54, 29, 60, 0, 45, 70, 39])]

# TestFilterWithAmplifiedCPUs (plugin_test.go:814-925): buildCPUTopologyForTest(2, 1, 8, 2)
# (32 CPUs), node cpu = Amplify(32, ratio), memory 40Gi; existing pod [cpu, LSR]
# (LSR: CPUs 0..cpu-1 allocated); NRT zones of Amplify(16, ratio) cpu and 20Gi
# when has_nrt (:894-909); pod [cpu, LSR].  want: Filter passes.
P = "plugin_test.go:"
FILTER_AMP = [
    {"name": "no resources requested always fits", "source": P + "825-830", "ratio": 2.0, "has_nrt": False,
     "existing": [4, False], "pod": None, "want": True},
    {"name": "no filtering without node cpu amplification", "source": P + "831-837", "ratio": 1.0,
     "has_nrt": False, "existing": [32, False], "pod": [32, False], "want": True},
    {"name": "cpu fits on no NRT node", "source": P + "838-844", "ratio": 2.0, "has_nrt": False,
     "existing": [32, False], "pod": [32, False], "want": True},
    {"name": "insufficient cpu", "source": P + "845-852", "ratio": 2.0, "has_nrt": False,
     "existing": [64, False], "pod": [32, False], "want": False},
    {"name": "insufficient cpu with cpuset pod on node", "source": P + "853-861", "ratio": 2.0, "has_nrt": True,
     "existing": [32, True], "pod": [32, False], "want": False},
    {"name": "insufficient cpu when scheduling cpuset pod", "source": P + "862-870", "ratio": 2.0,
     "has_nrt": True, "existing": [32, False], "pod": [32, True], "want": False},
    {"name": "insufficient cpu when scheduling cpuset pod with cpuset pod on node", "source": P + "871-879",
     "ratio": 2.0, "has_nrt": True, "existing": [32, True], "pod": [32, True], "want": False},
]


def main():
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "numa_plugin_cases.json")
    with open(path, "w") as f:
        json.dump({"filter": FILTER, "reserve": RESERVE, "score_node1": SCORE_NODE1, "score_node2": SCORE_NODE2,
                   "filter_amp": FILTER_AMP}, f, indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
