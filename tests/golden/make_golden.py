"""Writes the golden known-answer fixtures of this directory.

The reference path is Go and cannot be compiled or run in this image (no Go
toolchain), so these fixtures are TRANSCRIPTIONS of the known-answer tables in
the reference's own tests: inputs (objects) and expected outputs exactly as
the Go test tables state them, one JSON case per table row, each carrying the
reference file:line of its row.  Times are seconds relative to the evaluation
instant `now` (the Go tests use time.Now()).

Run:  python tests/golden/make_golden.py
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LA_TEST = "pkg/scheduler/plugins/loadaware/load_aware_test.go"
EST_TEST = "pkg/scheduler/plugins/loadaware/estimator/default_estimator_test.go"


def ctr(req=None, lim=None):
    return {"requests": req or {}, "limits": lim or {}}


def pod(name="test-pod-1", ns="default", priority=None, labels=None, containers=None, owner_kinds=None):
    return {"ns": ns, "name": name, "priority": priority, "labels": labels or {},
            "containers": containers if containers is not None else [ctr()], "owner_kinds": owner_kinds or []}


G16 = ctr({"cpu": "16", "memory": "32Gi"}, {"cpu": "16", "memory": "32Gi"})


def nm(update_dt=0.0, node_usage=None, aggregated=None, pods_metric=None, has_node_metric=None):
    return {"update_dt": update_dt, "report_interval_s": 60, "node_usage": node_usage,
            "aggregated": aggregated or [], "pods_metric": pods_metric or [], "has_node_metric": has_node_metric}


NODE_96 = {"name": "test-node-1", "allocatable": {"cpu": "96", "memory": "512Gi"}}

# ---------------------------------------------------------------- TestScore
score_cases = [
    dict(name="score node with expired nodeMetric", line=926, pod=None,
         node_metric=nm(update_dt=-180), want=0),
    dict(name="score empty node", line=947, pod=pod(containers=[G16]), node_metric=nm(), want=90),
    dict(name="score node missing NodeMetrics", line=991, pod=pod(containers=[G16]), node_metric=None, want=0),
    dict(name="score load node", line=1020, pod=pod(containers=[G16]),
         node_metric=nm(node_usage={"cpu": "32", "memory": "10Gi"}), want=72),
    dict(name="score load node with p95", line=1072, pod=pod(containers=[G16]),
         args={"aggregated": {"score_aggregation_type": "p95", "score_aggregated_duration_s": 300}},
         node_metric=nm(node_usage={"cpu": "0", "memory": "0Gi"},
                        aggregated=[{"duration_s": 300, "usage": {"p95": {"cpu": "32", "memory": "10Gi"},
                                                                  "p99": {"cpu": "50", "memory": "70Gi"}}}]),
         want=72),
    dict(name="score load node with p95 but have not reported usage", line=1147, pod=pod(containers=[G16]),
         args={"aggregated": {"score_aggregation_type": "p95", "score_aggregated_duration_s": 300}},
         node_metric=nm(node_usage={"cpu": "0", "memory": "0Gi"}), want=90),
    dict(name="score load node with p95 but have not reported usage and have assigned pods", line=1203,
         pod=pod(containers=[G16]),
         args={"aggregated": {"score_aggregation_type": "p95", "score_aggregated_duration_s": 300}},
         assigned=[{"dt": -600, "pod": pod(name="assigned-pod-1", containers=[G16])}],
         node_metric=nm(node_usage={"cpu": "0", "memory": "0Gi"},
                        pods_metric=[{"ns": "default", "name": "assigned-pod-1",
                                      "usage": {"cpu": "1", "memory": "1Gi"}}]),
         want=81),
    dict(name="score load node with just assigned pod", line=1300, pod=pod(containers=[G16]),
         assigned=[{"dt": -1e-6, "pod": pod(name="assigned-pod-1", containers=[G16])}],
         node_metric=nm(node_usage={"cpu": "32", "memory": "10Gi"}), want=63),
    dict(name="score load node with just assigned pod where after updateTime", line=1381,
         pod=pod(containers=[G16]),
         assigned=[{"dt": 0.0, "pod": pod(name="assigned-pod-1", containers=[G16])}],
         node_metric=nm(update_dt=-10, node_usage={"cpu": "32", "memory": "10Gi"}), want=63),
    dict(name="score load node with just assigned pod where before updateTime", line=1462,
         pod=pod(containers=[G16]),
         assigned=[{"dt": -10, "pod": pod(name="assigned-pod-1", containers=[G16])}],
         node_metric=nm(node_usage={"cpu": "32", "memory": "10Gi"}), want=63),
    dict(name="score batch Pod", line=1543,
         pod=pod(priority=5000, containers=[ctr(
             {"kubernetes.io/batch-cpu": "16000", "kubernetes.io/batch-memory": "32Gi"},
             {"kubernetes.io/batch-cpu": "16000", "kubernetes.io/batch-memory": "32Gi"})]),
         node_metric=nm(), want=90),
    dict(name="score prod Pod", line=1588, args={"score_according_prod_usage": True},
         pod=pod(name="prod-pod-1", priority=9999,
                 containers=[ctr({"cpu": "16000", "memory": "32Gi"}, {"cpu": "16000", "memory": "32Gi"})]),
         assigned=[{"dt": -1e-6, "pod": pod(name="assign-prod-pod-1", priority=9999, containers=[G16])}],
         node_metric=nm(pods_metric=[{"ns": "default", "name": "assign-prod-pod-1",
                                      "usage": {"cpu": "30", "memory": "100Gi"}}]),
         want=38),
    dict(name="score request less than limit", line=1676,
         pod=pod(containers=[ctr({"cpu": "8", "memory": "16Gi"}, {"cpu": "16", "memory": "32Gi"})]),
         node_metric=nm(), want=88),
    dict(name="score empty pod", line=1720, pod=pod(containers=[ctr()]), node_metric=nm(), want=99),
]
for c in score_cases:
    c.setdefault("args", {})
    c.setdefault("assigned", [])
    c["source"] = f"{LA_TEST}:{c.pop('line')}"
# "score node with expired nodeMetric": tt.pod is nil in the Go table -> an empty pod
score_cases[0]["pod"] = pod(containers=[])

# ---------------------------------------------------------- TestFilterUsage
PROD_PODS = [pod(name="prod-pod-1", priority=9999, containers=[]), pod(name="prod-pod-2", priority=9999, containers=[])]
PROD_METRICS = [{"ns": "default", "name": "prod-pod-1", "usage": {"cpu": "30", "memory": "200Gi"}},
                {"ns": "default", "name": "prod-pod-2", "usage": {"cpu": "33", "memory": "300Gi"}}]
filter_cases = [
    dict(name="filter normal usage", line=277, node_metric=nm(node_usage={"cpu": "60", "memory": "256Gi"}), want_ok=True),
    dict(name="filter node missing NodeMetrics", line=305, node_metric=None, want_ok=True),
    dict(name="filter exceed cpu usage", line=310, node_metric=nm(node_usage={"cpu": "70", "memory": "256Gi"}),
         want_ok=False),
    dict(name="filter exceed p95 cpu usage", line=338,
         args={"aggregated": {"usage_thresholds": {"cpu": 60}, "usage_aggregation_type": "p95",
                              "usage_aggregated_duration_s": 300}},
         node_metric=nm(node_usage={"cpu": "30", "memory": "100Gi"},
                        aggregated=[{"duration_s": 300, "usage": {"p95": {"cpu": "70", "memory": "256Gi"}}}]),
         want_ok=False),
    dict(name="filter exceed memory usage", line=386, node_metric=nm(node_usage={"cpu": "30", "memory": "500Gi"}),
         want_ok=False),
    dict(name="filter exceed memory usage by custom usage thresholds", line=414,
         annotation={"usageThresholds": {"memory": 60}},
         node_metric=nm(node_usage={"cpu": "30", "memory": "316Gi"}), want_ok=False),
    dict(name="filter exceed p95 cpu usage by custom usage", line=445,
         annotation={"aggregatedUsage": {"usageThresholds": {"cpu": 60}, "usageAggregationType": "p95",
                                         "usageAggregatedDuration": "5m0s"}},
         node_metric=nm(node_usage={"cpu": "30", "memory": "100Gi"},
                        aggregated=[{"duration_s": 300, "usage": {"p95": {"cpu": "70", "memory": "256Gi"}}}]),
         want_ok=False),
    dict(name="disable filter exceed memory usage", line=493, args={"usage_thresholds": {"memory": 0}},
         node_metric=nm(node_usage={"cpu": "30", "memory": "500Gi"}), want_ok=True),
    dict(name="prod usage filter is not enabled by default", line=524,
         args={"usage_thresholds": {"cpu": 100, "memory": 100}}, pods=PROD_PODS,
         node_metric=nm(node_usage={"cpu": "63", "memory": "500Gi"}, pods_metric=PROD_METRICS), want_ok=True),
    dict(name="filter prod cpu usage", line=582,
         args={"usage_thresholds": {"cpu": 100, "memory": 100}, "prod_usage_thresholds": {"cpu": 50, "memory": 100}},
         pods=PROD_PODS, test_pod=pod(name="prod-pod-3", priority=9999, containers=[]),
         node_metric=nm(node_usage={"cpu": "63", "memory": "500Gi"}, pods_metric=PROD_METRICS), want_ok=False),
    dict(name="filter prod memory usage", line=645,
         args={"usage_thresholds": {"cpu": 100, "memory": 100}, "prod_usage_thresholds": {"cpu": 100, "memory": 50}},
         pods=PROD_PODS, test_pod=pod(name="prod-pod-3", priority=9999, containers=[]),
         node_metric=nm(node_usage={"cpu": "63", "memory": "500Gi"}, pods_metric=PROD_METRICS), want_ok=False),
    dict(name="filter prod memory usage with custom usage configuration", line=708,
         args={"usage_thresholds": {"cpu": 100, "memory": 100}, "prod_usage_thresholds": {"cpu": 100, "memory": 100}},
         annotation={"prodUsageThresholds": {"cpu": 100, "memory": 50}},
         pods=PROD_PODS, test_pod=pod(name="prod-pod-3", priority=9999, containers=[]),
         node_metric=nm(node_usage={"cpu": "63", "memory": "500Gi"}, pods_metric=PROD_METRICS), want_ok=False),
    dict(name="filter daemonset pod exceed cpu usage", line=775,
         test_pod=pod(name="test-pod", priority=9999, containers=[], owner_kinds=["DaemonSet"]),
         node_metric=nm(node_usage={"cpu": "70", "memory": "256Gi"}), want_ok=True),
]
for c in filter_cases:
    c.setdefault("args", {})
    c["args"].setdefault("filter_expired_node_metrics", False)   # load_aware_test.go:807
    c.setdefault("pods", [])
    c.setdefault("test_pod", pod(name="", ns="", containers=[]))   # &corev1.Pod{} :902-905
    c.setdefault("annotation", None)
    c["source"] = f"{LA_TEST}:{c.pop('line')}"

# -------------------------------------------------- TestFilterExpiredNodeMetric
expired_cases = [
    dict(name="filter healthy nodeMetrics", line=147, node_metric=nm(update_dt=0), want_ok=True),
    dict(name="filter unhealthy nodeMetric with nil updateTime", line=167, node_metric=nm(update_dt=None),
         want_ok=True),
    dict(name="filter unhealthy nodeMetric with expired updateTime", line=181, node_metric=nm(update_dt=-180),
         want_ok=True),
]
for c in expired_cases:
    c["args"] = {}                                  # defaults: FilterExpiredNodeMetrics=true, 180 s
    c["node"] = {"name": "test-node-1", "allocatable": {}}   # load_aware_test.go:219-225
    c["test_pod"] = pod(name="", ns="", containers=[])
    c["source"] = f"{LA_TEST}:{c.pop('line')}"

# ------------------------------------------------------------------ estimator
G4 = {"cpu": "4", "memory": "8Gi"}
estimate_cases = [
    dict(name="estimate empty pod", line=40, pod=pod(containers=[ctr()]), factors=None,
         want={"cpu": 250, "memory": 209715200}),
    dict(name="estimate guaranteed pod", line=58, pod=pod(containers=[ctr(G4, G4)]), factors=None,
         want={"cpu": 3400, "memory": 6012954214}),
    dict(name="estimate burstable pod", line=82,
         pod=pod(containers=[ctr(G4, {"cpu": "8", "memory": "8Gi"})]), factors=None,
         want={"cpu": 8000, "memory": 6012954214}),
    dict(name="estimate guaranteed pod and zoomed cpu factors", line=106, pod=pod(containers=[ctr(G4, G4)]),
         factors={"cpu": 110}, want={"cpu": 4000, "memory": 6012954214}),
    dict(name="estimate guaranteed pod and zoomed memory factors", line=133, pod=pod(containers=[ctr(G4, G4)]),
         factors={"memory": 110}, want={"cpu": 3400, "memory": 8589934592}),
    dict(name="estimate Batch pod", line=160,
         pod=pod(priority=5000, labels={"koordinator.sh/qosClass": "BE"}, containers=[ctr(
             {"kubernetes.io/batch-cpu": "4000", "kubernetes.io/batch-memory": "8Gi"},
             {"kubernetes.io/batch-cpu": "4000", "kubernetes.io/batch-memory": "8Gi"})]),
         factors=None, want={"cpu": 3400, "memory": 6012954214}),
    dict(name="estimate pod only has request", line=193,
         pod=pod(priority=9999, labels={"koordinator.sh/qosClass": "LS"}, containers=[ctr(G4)]),
         factors={"cpu": 80, "memory": 80}, want={"cpu": 3200, "memory": 6871947674}),
]
for c in estimate_cases:
    c["source"] = f"{EST_TEST}:{c.pop('line')}"

estimate_node_cases = [
    dict(name="estimate empty node", line=259, allocatable={"cpu": "32"}, annotations={}, want={"cpu": "32"}),
    dict(name="estimate node with original allocatable", line=272, allocatable={"cpu": "32", "memory": "42Gi"},
         annotations={"node.koordinator.sh/raw-allocatable": '{"cpu":28,"memory":"32Gi"}'},
         want={"cpu": "28", "memory": "32Gi"}),
    dict(name="estimate node with original allocatable and sames", line=291,
         allocatable={"cpu": "32", "memory": "42Gi"},
         annotations={"node.koordinator.sh/raw-allocatable": '{"cpu":32,"memory":"42Gi"}'},
         want={"cpu": "32", "memory": "42Gi"}),
]
for c in estimate_node_cases:
    c["source"] = f"{EST_TEST}:{c.pop('line')}"


# --------------------------------------------------------------- cpu_accumulator_test.go
ACC_TEST = "pkg/scheduler/plugins/nodenumaresource/cpu_accumulator_test.go"


def acc(name, line, topo, need, want, allocated="", policy="FullPCPUs", excl="None", strategy="MostAllocated",
        allocated_excl="", error=False):
    """One takeCPUs call: topology = buildCPUTopologyForTest(sockets, nodesPerSocket, coresPerNode, cpusPerCore),
    available = all - allocated, allocatedCPUs = KeepOnly(allocated) with ExclusivePolicy allocated_excl."""
    return dict(name=name, source=f"{ACC_TEST}:{line}", topology=topo, allocated=allocated, need=need,
                bind_policy=policy, exclusive_policy=excl, strategy=strategy, allocated_exclusive_policy=allocated_excl,
                want=want, want_error=error)


_full_most = [  # TestTakeFullPCPUs, :59-173 (NUMAMostAllocated)
    ("allocate on non-NUMA node", 70, [1, 1, 4, 2], "", 2, "0-1"),
    ("with allocated cpus", 77, [1, 1, 4, 2], "0-1", 2, "2-3"),
    ("allocate whole socket", 85, [2, 1, 4, 2], "", 8, "0-7"),
    ("allocate across socket", 92, [2, 1, 4, 2], "", 12, "0-11"),
    ("allocate whole socket with partially-allocated socket", 99, [2, 1, 4, 2], "0-1", 8, "8-15"),
    ("allocate in the smallest idle socket", 107, [2, 2, 4, 2], "0-5,16-23", 6, "24-29"),
    ("allocate the most of CPUs on the same socket", 115, [2, 2, 4, 2], "0-5,16-23", 12, "6-15,24-25"),
    ("allocate from first socket", 123, [2, 2, 4, 2], "0-3,8-11", 4, "4-7"),
    ("allocate with less spread cpus", 131, [2, 2, 2, 2], "0,2,4,8,12", 4, "10-11,14-15"),
    ("allocate with the most spread cpus", 139, [2, 2, 2, 2], "0,2,4,8,10,12", 6, "5-7,13-15"),
    ("allocate with the most spread cpus on the smallest idle cpus socket", 147, [2, 2, 2, 2], "0,2,4,8-10,12", 6,
     "6-7,11,13-15"),
]
_full_least = [  # TestTakeFullPCPUsWithNUMALeastAllocated, :175-289
    ("allocate on non-NUMA node", 186, [1, 1, 4, 2], "", 2, "0-1"),
    ("with allocated cpus", 193, [1, 1, 4, 2], "0-1", 2, "2-3"),
    ("allocate whole socket", 201, [2, 1, 4, 2], "", 8, "0-7"),
    ("allocate across socket", 208, [2, 1, 4, 2], "", 12, "0-11"),
    ("allocate whole socket with partially-allocated socket", 215, [2, 1, 4, 2], "0-1", 8, "8-15"),
    ("allocate in the most idle socket", 223, [2, 2, 4, 2], "0-5,16-23", 6, "8-13"),
    ("allocate the most of CPUs on the same socket", 231, [2, 2, 4, 2], "0-5,16-23", 12, "6-15,24-25"),
    ("allocate from second socket", 239, [2, 2, 4, 2], "0-3,8-11", 4, "16-19"),
    ("allocate with less spread cpus", 247, [2, 2, 2, 2], "0,2,4,8,12", 4, "10-11,14-15"),
    ("allocate with the less spread cpus 2", 255, [2, 2, 2, 2], "0,2,4,8,10,12", 6, "1,3,6-7,14-15"),
    ("allocate with the most spread cpus on the most idle cpus socket 3", 263, [2, 2, 4, 2], "0,2,4,8-10,12", 6,
     "16-21"),
]
_spread_most = [  # TestTakeSpreadByPCPUs, :301-361
    ("allocate on non-NUMA node", 312, [1, 1, 4, 2], "", 4, "0,2,4,6"),
    ("allocate satisfied the partially-allocated socket", 319, [2, 1, 4, 2], "0,2", 4, "1,3,4,6"),
    ("allocate cpus on full-free socket", 327, [2, 1, 4, 2], "0-3", 4, "8,10,12,14"),
    ("allocate most of CPUs in the same socket and overlapped-cores", 335, [2, 1, 4, 2], "0,2", 6, "1,3-7"),
]
_spread_least = [  # TestTakeSpreadByPCPUsWithNUMALeastAllocated, :373-433
    ("allocate on non-NUMA node", 384, [1, 1, 4, 2], "", 4, "0,2,4,6"),
    ("allocate satisfied the partially-allocated socket", 391, [2, 1, 4, 2], "0,2", 4, "8,10,12,14"),
    ("allocate cpus on full-free socket", 399, [2, 1, 4, 2], "0-3", 4, "8,10,12,14"),
    ("allocate most of CPUs in the same socket and overlapped-cores", 407, [2, 1, 4, 2], "0,2", 6,
     "8-12,14"),
]
acc_cases = []
for n, l, t, a, k, w in _full_most:
    acc_cases.append(acc("FullPCPUs/" + n, l, t, k, w, allocated=a))
for n, l, t, a, k, w in _full_least:
    acc_cases.append(acc("FullPCPUs-least/" + n, l, t, k, w, allocated=a, strategy="LeastAllocated"))
for n, l, t, a, k, w in _spread_most:
    acc_cases.append(acc("Spread/" + n, l, t, k, w, allocated=a, policy="SpreadByPCPUs"))
for n, l, t, a, k, w in _spread_least:
    acc_cases.append(acc("Spread-least/" + n, l, t, k, w, allocated=a, policy="SpreadByPCPUs",
                         strategy="LeastAllocated"))
# TestTakeCPUsWithExclusivePolicy, :435-558: allocated CPUs carry PCPULevel unless stated, the pod's
# exclusive policy defaults to PCPULevel and its bind policy to SpreadByPCPUs (:531-540)
_excl = [
    ("allocate cpus on full-free socket with PCPULevel", 448, [2, 1, 4, 2], "0,2", "", "PCPULevel", "SpreadByPCPUs",
     4, "8,10,12,14"),
    ("allocate overlapped cpus with PCPULevel", 455, [2, 1, 4, 2], "", "", "PCPULevel", "SpreadByPCPUs", 10,
     "0-4,6,8,10,12,14"),
    ("allocate cpus on large-size partially-allocated socket with PCPULevel", 461, [2, 1, 8, 2], "0,2", "",
     "PCPULevel", "SpreadByPCPUs", 4, "4,6,8,10"),
    ("allocate cpus with none exclusive policy", 468, [2, 1, 8, 2], "0,2", "", "None", "SpreadByPCPUs", 4, "1,3,4,6"),
    ("allocate cpus on full-free socket with NUMANodeLevel", 476, [2, 1, 4, 2], "0,2", "NUMANodeLevel",
     "NUMANodeLevel", "SpreadByPCPUs", 4, "8,10,12,14"),
    ("allocate cpus on partially-allocated socket without NUMANodeLevel", 485, [2, 1, 4, 2], "0,2", "NUMANodeLevel",
     "None", "SpreadByPCPUs", 4, "1,3,4,6"),
    ("allocate cpus on full-free socket with NUMANodeLevel with PCPUs", 494, [2, 1, 4, 2], "0,2", "NUMANodeLevel",
     "NUMANodeLevel", "FullPCPUs", 4, "8-11"),
    ("allocate cpus on partially-allocated socket without NUMANodeLevel with PCPUs", 504, [2, 1, 4, 2], "0,2",
     "NUMANodeLevel", "None", "FullPCPUs", 4, "4-7"),
]
for n, l, t, a, ae, ex, pol, k, w in _excl:
    acc_cases.append(acc("Exclusive/" + n, l, t, k, w, allocated=a, policy=pol, excl=ex,
                         allocated_excl=ae or "PCPULevel"))
# TestTakePreferredCPUs, :758-777, the two calls without preferred CPUs
acc_cases.append(acc("Preferred/takeCPUs spread 2", 761, [2, 1, 16, 2], 2, "0,2", policy="SpreadByPCPUs"))
acc_cases.append(acc("Preferred/empty preferred on the rest", 769, [2, 1, 16, 2], 2, "1,3", allocated="0,2",
                     policy="SpreadByPCPUs"))
_SPREAD_ORDER = [0, 2, 4, 6, 8, 10, 12, 14, 16, 18, 20, 22, 24, 26, 28, 30,
                 1, 3, 5, 7, 9, 11, 13, 15, 17, 19, 21, 23, 25, 27, 29, 31]
spread_order_cases = [
    dict(name="TestCPUSpreadByPCPUs", source=f"{ACC_TEST}:291-299", topology=[2, 2, 4, 2], strategy="MostAllocated",
         want=_SPREAD_ORDER),
    dict(name="TestCPUSpreadByPCPUsWithNUMALeastAllocated", source=f"{ACC_TEST}:363-371", topology=[2, 2, 4, 2],
         strategy="LeastAllocated", want=_SPREAD_ORDER),
]

# ------------------------------------------------------------ scoring_test.go TestPlugin_Score
SCORE_TEST = "pkg/scheduler/plugins/nodenumaresource/scoring_test.go"


def nscore(name, line, want, topo=None, cpu_bind=True, policy="", need=0, labels=None, total_cpus=96):
    """One Score call: topology = buildCPUTopologyForTest(sockets, nodesPerSocket, coresPerNode, cpusPerCore)
    or None (no CPU topology) / "invalid" (&CPUTopology{}); the node's allocatable cpu is its CPU count
    x 1000 (96 CPUs without a topology), memory 512Gi; empty NodeAllocation; requests = cpu only."""
    return dict(name=name, source=f"{SCORE_TEST}:{line}", topology=topo, request_cpu_bind=cpu_bind,
                preferred_bind_policy=policy, need=need, node_labels=labels or {}, want=want,
                total_cpus=total_cpus)


LBL_STRATEGY = "node.koordinator.sh/numa-allocate-strategy"
LBL_BIND = "node.koordinator.sh/cpu-bind-policy"
numa_score_cases = [
    nscore("error with missing allocationState", 389, 0),
    nscore("error with invalid cpu topology", 398, 0, topo="invalid", total_cpus=0),
    nscore("succeed with skip", 408, 0, cpu_bind=False),
    nscore("score with full empty node FullPCPUs", 417, 25, [2, 1, 4, 2], policy="FullPCPUs", need=4),
    nscore("score with satisfied node FullPCPUs", 429, 50, [2, 1, 4, 2], policy="FullPCPUs", need=8),
    nscore("score with full empty node SpreadByPCPUs", 442, 25, [2, 1, 4, 2], policy="SpreadByPCPUs", need=4),
    nscore("score with exceed socket FullPCPUs", 454, 100, [2, 1, 4, 2], policy="FullPCPUs", need=16),
    nscore("score with satisfied socket FullPCPUs", 466, 50, [2, 2, 4, 2], policy="FullPCPUs", need=16),
    nscore("score with full empty socket SpreadByPCPUs", 478, 25, [2, 1, 4, 2], policy="SpreadByPCPUs", need=4),
    nscore("score with Node NUMA Allocate Strategy", 490, 12, [2, 1, 4, 2], policy="SpreadByPCPUs", need=2,
           labels={LBL_STRATEGY: "LeastAllocated"}),
    nscore("score with Node CPU Bind Policy", 505, 50, [2, 1, 4, 2], policy="SpreadByPCPUs", need=8,
           labels={LBL_BIND: "FullPCPUsOnly"}),
]


def dump(name, obj):
    with open(os.path.join(HERE, name), "w") as f:
        json.dump(obj, f, indent=1, sort_keys=True)
        f.write("\n")


if __name__ == "__main__":
    dump("loadaware_score.json", {"node": NODE_96, "cases": score_cases,
                                  "harness": f"{LA_TEST}:1754-1851"})
    dump("loadaware_filter.json", {"node": NODE_96, "cases": filter_cases + expired_cases,
                                   "harness": f"{LA_TEST}:804-910, :200-258"})
    dump("estimator.json", {"estimate_pod": estimate_cases, "estimate_node": estimate_node_cases,
                            "harness": f"{EST_TEST}:233-250, :314-329"})
    dump("cpu_accumulator.json", {"take_cpus": acc_cases, "spread_order": spread_order_cases,
                                  "harness": f"{ACC_TEST}:156-171 (takeCPUs, maxRefCount 1)",
                                  "not_transcribed": "TestTakeCPUsWithMaxRefCount / TestTakeCPUsSortByRefCount "
                                                     "(maxRefCount 2) and the preferred-CPU calls of "
                                                     "TestTakePreferredCPUs (Reservation): out of the engine's scope"})
    dump("numa_score.json", {"cases": numa_score_cases,
                             "harness": f"{SCORE_TEST}:520-594 (ScoringStrategy MostAllocated, resources cpu:1)",
                             "not_transcribed": "error with missing preFilterState (:384, a framework.Status error, "
                                                "not a score); TestNUMANodeScore (NUMA topology policies) and "
                                                "TestScoreWithAmplifiedCPUs (amplification): out of the engine's "
                                                "scope"})
    print("wrote golden fixtures")
