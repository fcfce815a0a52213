"""Turns the golden fixture JSON (tests/golden/*.json) into objects, snapshots
and pod records, the way the reference tests build their fakes
(load_aware_test.go:804-910, :1754-1851)."""
from __future__ import annotations

import json
import os

from koordinator_amd import k8s, marshal
from koordinator_amd.config import (LoadAwareSchedulingAggregatedArgs, LoadAwareSchedulingArgs, Profile,
                                    PLUGIN_LOADAWARE)

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NOW = 1_000_000.0


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def rlist(d):
    return {k: k8s.Quantity(v) for k, v in (d or {}).items()}


def make_pod(d):
    return k8s.Pod(namespace=d["ns"], name=d["name"], priority=d.get("priority"), labels=dict(d.get("labels") or {}),
                   owner_kinds=list(d.get("owner_kinds") or []),
                   containers=[k8s.Container(requests=rlist(c["requests"]), limits=rlist(c["limits"]))
                               for c in d.get("containers", [])])


def make_node_metric(d, node_name):
    if d is None:
        return None
    aggregated = [k8s.AggregatedUsage(a["duration_s"], {t: rlist(u) for t, u in a["usage"].items()})
                  for a in d.get("aggregated", [])]
    return k8s.NodeMetric(
        name=node_name,
        update_time=None if d["update_dt"] is None else NOW + d["update_dt"],
        report_interval_s=d.get("report_interval_s"),
        node_usage=rlist(d["node_usage"]) if d.get("node_usage") is not None else None,
        aggregated=aggregated,
        pods_metric=[k8s.PodMetric(p["ns"], p["name"], rlist(p["usage"])) for p in d.get("pods_metric", [])],
        has_node_metric=d.get("has_node_metric"),
    )


def make_args(d) -> LoadAwareSchedulingArgs:
    a = LoadAwareSchedulingArgs()
    for k, v in (d or {}).items():
        if k == "aggregated":
            a.aggregated = LoadAwareSchedulingAggregatedArgs(**v)
        else:
            setattr(a, k, v)
    return a


def la_profile(args_d) -> Profile:
    return Profile(filters=(PLUGIN_LOADAWARE,), scores={PLUGIN_LOADAWARE: 1}, loadaware=make_args(args_d))


def build_case(case, node_d, *, test_pod_key="pod"):
    """-> (profile, NodeTable(1 row), pod record array(1))"""
    node = k8s.Node(name=node_d["name"], allocatable=rlist(node_d["allocatable"]))
    if case.get("annotation") is not None:
        node.annotations[k8s.ANNOTATION_CUSTOM_USAGE_THRESHOLDS] = json.dumps(case["annotation"])
    profile = la_profile(case.get("args"))
    cluster = marshal.ClusterState(nodes=[node])
    nmd = make_node_metric(case.get("node_metric"), node.name)
    if nmd is not None:
        cluster.node_metrics[node.name] = nmd
    for p in case.get("pods", []):
        pp = make_pod(p)
        cluster.pods[pp.key] = pp
    tp = make_pod(case[test_pod_key])
    if case[test_pod_key]["name"]:
        cluster.pods[tp.key] = tp
    for a in case.get("assigned", []):
        ap = make_pod(a["pod"])
        ap.node_name = node.name
        cluster.pods[ap.key] = ap
        cluster.assigned.setdefault(node.name, []).append(marshal.AssignedPod(ap, NOW + a["dt"]))
    table = marshal.build_table(cluster, profile, NOW)
    rec = marshal.pod_records([tp], profile)
    return profile, table, rec


def score_cases():
    d = load("loadaware_score.json")
    return [(c["name"], c, d["node"]) for c in d["cases"]]


def filter_cases():
    d = load("loadaware_filter.json")
    return [(c["name"], c, c.get("node", d["node"])) for c in d["cases"]]


# ------------------------------------------------ NodeNUMAResource Score (scoring_test.go)
def numa_score_cases():
    return [(c["name"], c) for c in load("numa_score.json")["cases"]]


def build_numa_score_case(case):
    """-> (profile, NodeTable(1 row), pod record array(1)) for one TestPlugin_Score row
    (scoring_test.go:520-594: MostAllocated over cpu weight 1, allocatable cpu = #CPUs x 1000,
    memory 512Gi, an empty NodeAllocation, the test's preFilterState as the pod's NUMA state)."""
    from koordinator_amd import abi
    from koordinator_amd.config import PLUGIN_NUMA
    from koordinator_amd.numa import ClassTable, node_numa_flags, reference_test_topology
    from koordinator_amd.snapshot import NodeTable, pod_array
    prof = Profile(filters=(), scores={PLUGIN_NUMA: 1})
    prof.numa.scoring_type = "MostAllocated"
    prof.numa.resources = {k8s.CPU: 1}
    t = NodeTable.empty(1)
    if isinstance(case["topology"], list):
        topo = reference_test_topology(*case["topology"])
        ct = ClassTable()
        t["numa_class"][0] = ct.add(topo)
        t.numa_classes = ct.records()
        free = topo.all_mask()
        for w in range(abi.NUMA_WORDS):
            t[f"numa_free{w}"][0] = free[w]
        cpus = topo.num_cpus
    else:  # no CPU topology, or an invalid one (&CPUTopology{}: zero CPUs)
        t["numa_class"][0] = -1
        cpus = case["total_cpus"]
    t["alloc0"][0] = cpus * 1000
    t["alloc1"][0] = 512 * 2**30
    t["la_alloc_cpu_m"][0], t["la_alloc_mem"][0] = t["alloc0"][0], t["alloc1"][0]
    t["numa_flags"][0] = node_numa_flags(case["node_labels"], None, prof.numa.default_most_allocated)
    p = pod_array(1)
    if case["request_cpu_bind"]:
        need = case["need"]
        p["req"][0, abi.RES_CPU] = need * 1000
        p["nz_cpu_m"][0] = need * 1000
        p["flags"][0] = abi.POD_PROD | abi.POD_CPUSET | (abi.POD_HAS_REQ if need else 0)
        p["numa_cpus"][0] = need
        pol = {"": abi.CPUBIND_NONE, "FullPCPUs": abi.CPUBIND_FULL_PCPUS,
               "SpreadByPCPUs": abi.CPUBIND_SPREAD_BY_PCPUS}[case["preferred_bind_policy"]]
        p["numa_policy"][0] = abi.numa_policy(0, pol, 0)
    return prof, t, p


def numa_node_score_cases():
    return [(c["name"], c) for c in load("topology_policy_cases.json")["numa_node_score"]]


def build_numa_node_score_case(case):
    """-> (profile, NodeTable, pod record array(1)) for one TestNUMANodeScore row
    (scoring_test.go:302-352)."""
    import numpy as np
    from koordinator_amd import abi
    from koordinator_amd.config import PLUGIN_NUMA
    from koordinator_amd.numa import (ClassTable, LABEL_NUMA_TOPOLOGY_POLICY, node_numa_flags,
                                      reference_test_topology, zone_row)
    from koordinator_amd.snapshot import NodeTable, pod_array
    prof = Profile(filters=(PLUGIN_NUMA,), scores={PLUGIN_NUMA: 1})
    prof.numa.scoring_type = "MostAllocated"
    prof.numa.resources = {k8s.CPU: 1, k8s.MEMORY: 1}
    gi = 2 ** 30
    n = len(case["nodes"])
    t = NodeTable.empty(n)
    ct = ClassTable()
    topos = []
    for i, (name, cores, mem_gi, policy, count) in enumerate(case["nodes"]):
        t.names[i] = name
        alloc_m, mem = cores * 1000, mem_gi * gi
        t["alloc0"][i], t["alloc1"][i] = alloc_m, mem
        t["alloc_pods"][i] = 110
        t["la_alloc_cpu_m"][i], t["la_alloc_mem"][i] = alloc_m, mem
        topo = reference_test_topology(count, 1, cores // 2 // count, 2)
        topos.append(topo)
        t["numa_class"][i] = ct.add(topo)
        t["numa_flags"][i] = node_numa_flags({LABEL_NUMA_TOPOLOGY_POLICY: policy}, None,
                                             prof.numa.default_most_allocated)
        t["numa_zone_alloc"][i] = zone_row([(alloc_m // count, mem // count)] * count)
    t.numa_classes = ct.records()
    used_cpus = [set() for _ in range(n)]
    for node, cpu, mem_gi, lsr in case["existing"]:
        t["numa_zone_used"][node, 0, 0] += cpu * 1000
        t["numa_zone_used"][node, 1, 0] += mem_gi * gi
        if lsr:
            used_cpus[node] |= set(range(cpu))
    for i, topo in enumerate(topos):
        free = topo.mask([c for c in topo.cpu_of if c not in used_cpus[i]])
        for w in range(abi.NUMA_WORDS):
            t[f"numa_free{w}"][i] = free[w]
        t["numa_alloc_cnt"][i] = len(used_cpus[i])
    cpu, mem_gi, lsr = case["pod"]
    p = pod_array(1)
    p["req"][0, abi.RES_CPU] = cpu * 1000
    p["req"][0, abi.RES_MEM] = mem_gi * gi
    p["nz_cpu_m"][0], p["nz_mem"][0] = cpu * 1000, mem_gi * gi
    p["flags"][0] = abi.POD_HAS_REQ
    if lsr:  # AllowUseCPUSet: LSR + prod priority; default preferred policy FullPCPUs
        p["flags"][0] |= abi.POD_PROD | abi.POD_CPUSET
        p["numa_cpus"][0] = cpu
        p["numa_policy"][0] = abi.numa_policy(0, abi.CPUBIND_FULL_PCPUS, 0)
    return prof, t, p


def numa_plugin_cases(kind):
    return [(c["name"], c) for c in load("numa_plugin_cases.json")[kind]]


BIND = {"": 0, "FullPCPUs": 1, "SpreadByPCPUs": 2}


def build_numa_plugin_case(case):
    """-> (profile, NodeTable(1 row), pod(1), topology or None) for one
    TestPlugin_Filter / TestPlugin_Reserve row (plugin_test.go:740-811, :1060-1145)."""
    from koordinator_amd import abi
    from koordinator_amd.config import PLUGIN_NUMA
    from koordinator_amd.numa import ClassTable, node_numa_flags, reference_test_topology, zone_row
    from koordinator_amd.snapshot import NodeTable, pod_array
    prof = Profile(filters=(PLUGIN_NUMA,), scores={PLUGIN_NUMA: 1})
    t = NodeTable.empty(1)
    t["alloc0"][0], t["alloc1"][0] = 96000, 512 * 2**30
    t["alloc_pods"][0] = 110
    t["la_alloc_cpu_m"][0], t["la_alloc_mem"][0] = t["alloc0"][0], t["alloc1"][0]
    topo = None
    if isinstance(case["topology"], list):
        topo = reference_test_topology(*case["topology"])
        ct = ClassTable()
        t["numa_class"][0] = ct.add(topo)
        t.numa_classes = ct.records()
        alloc = set(case["allocated_cpus"])
        free = topo.mask([c for c in topo.cpu_of if c not in alloc])
        for w in range(abi.NUMA_WORDS):
            t[f"numa_free{w}"][0] = free[w]
        t["numa_alloc_cnt"][0] = len(alloc)
        per_node = topo.num_cpus // topo.num_nodes
        t["numa_zone_alloc"][0] = zone_row([(per_node * 1000, 32 * 2**30)] * topo.num_nodes)
    else:  # none, or &CPUTopology{} (invalid: the marshaller drops it)
        t["numa_class"][0] = -1
    t["numa_flags"][0] = node_numa_flags(case["labels"], case["kubelet_policy"], prof.numa.default_most_allocated)
    p = pod_array(1)
    if case["request_cpu_bind"]:
        need = case["need"]
        p["req"][0, abi.RES_CPU] = need * 1000
        p["nz_cpu_m"][0] = need * 1000
        p["flags"][0] = abi.POD_CPUSET | (abi.POD_HAS_REQ if need else 0)
        p["numa_cpus"][0] = need
        p["numa_policy"][0] = abi.numa_policy(BIND[case["required"]], BIND[case["preferred"]], 0)
    return prof, t, p, topo


def build_numa_score_node1_case(case, node=1):
    """-> (profile, NodeTable(1 row), pod(1)) for the node1 (ratio 1.0) or node2
    (ratio 2.0) column of one TestScoreWithAmplifiedCPUs row (scoring_test.go:797-851)."""
    from koordinator_amd import abi
    from koordinator_amd.config import PLUGIN_NUMA
    from koordinator_amd.numa import ClassTable, node_numa_flags, reference_test_topology
    from koordinator_amd.snapshot import NodeTable, pod_array
    gi = 2**30
    prof = Profile(filters=(PLUGIN_NUMA,), scores={PLUGIN_NUMA: 1})
    prof.numa.scoring_type = case["scoring"]
    t = NodeTable.empty(1)
    t["alloc0"][0], t["alloc1"][0] = (32000, 40 * gi) if node == 1 else (64000, 60 * gi)
    t["numa_amp_cpu"][0] = 1.0 if node == 1 else 2.0
    t["alloc_pods"][0] = 110
    t["la_alloc_cpu_m"][0], t["la_alloc_mem"][0] = t["alloc0"][0], t["alloc1"][0]
    if case["existing"]:
        t["requested0"][0], t["requested1"][0] = 20000, 4 * gi
        t["npods"][0] = 1
    if case["has_nrt"]:
        topo = reference_test_topology(2, 1, 8, 2)
        ct = ClassTable()
        t["numa_class"][0] = ct.add(topo)
        t.numa_classes = ct.records()
        held = set(range(20)) if case["existing"] and case["existing_cpuset"] else set()
        free = topo.mask([c for c in topo.cpu_of if c not in held])
        for w in range(abi.NUMA_WORDS):
            t[f"numa_free{w}"][0] = free[w]
        t["numa_alloc_cnt"][0] = len(held)
    t["numa_flags"][0] = node_numa_flags({}, None, prof.numa.default_most_allocated)
    p = pod_array(1)
    p["req"][0, abi.RES_CPU], p["req"][0, abi.RES_MEM] = 8000, 16 * gi
    p["nz_cpu_m"][0], p["nz_mem"][0] = 8000, 16 * gi
    p["flags"][0] = abi.POD_HAS_REQ | abi.POD_PROD
    if case["pod_cpuset"]:
        p["flags"][0] |= abi.POD_CPUSET
        p["numa_cpus"][0] = 8
        p["numa_policy"][0] = abi.numa_policy(0, abi.CPUBIND_FULL_PCPUS, 0)
    return prof, t, p


def build_numa_filter_amp_case(case):
    """-> (profile, NodeTable(1 row), pod(1)) for one TestFilterWithAmplifiedCPUs
    row (plugin_test.go:882-924)."""
    import math
    from koordinator_amd import abi
    from koordinator_amd.config import PLUGIN_NUMA
    from koordinator_amd.numa import ClassTable, node_numa_flags, reference_test_topology
    from koordinator_amd.snapshot import NodeTable, pod_array
    gi = 2**30
    prof = Profile(filters=(PLUGIN_NUMA,), scores={PLUGIN_NUMA: 1})
    ratio = case["ratio"]
    amp = lambda v: v if ratio <= 1 else int(math.ceil(v * ratio))
    t = NodeTable.empty(1)
    t["alloc0"][0], t["alloc1"][0], t["alloc_pods"][0] = amp(32) * 1000, 40 * gi, 110
    t["la_alloc_cpu_m"][0], t["la_alloc_mem"][0] = t["alloc0"][0], t["alloc1"][0]
    t["numa_amp_cpu"][0] = ratio
    ecpu, elsr = case["existing"]
    t["requested0"][0], t["npods"][0] = ecpu * 1000, 1
    if case["has_nrt"]:
        topo = reference_test_topology(2, 1, 8, 2)
        ct = ClassTable()
        t["numa_class"][0] = ct.add(topo)
        t.numa_classes = ct.records()
        held = set(range(ecpu)) if elsr else set()
        free = topo.mask([c for c in topo.cpu_of if c not in held])
        for w in range(abi.NUMA_WORDS):
            t[f"numa_free{w}"][0] = free[w]
        t["numa_alloc_cnt"][0] = len(held)
    t["numa_flags"][0] = node_numa_flags({}, None, prof.numa.default_most_allocated)
    p = pod_array(1)
    if case["pod"] is None:
        p["flags"][0] = abi.POD_NUMA_SKIP
        p["nz_cpu_m"][0], p["nz_mem"][0] = 100, 200 << 20
    else:
        cpu, lsr = case["pod"]
        p["req"][0, abi.RES_CPU] = cpu * 1000
        p["nz_cpu_m"][0], p["nz_mem"][0] = cpu * 1000, 200 << 20
        p["flags"][0] = abi.POD_HAS_REQ | abi.POD_PROD
        if lsr:
            p["flags"][0] |= abi.POD_CPUSET
            p["numa_cpus"][0] = cpu
            p["numa_policy"][0] = abi.numa_policy(0, abi.CPUBIND_FULL_PCPUS, 0)
    return prof, t, p


# ------------------------------------------------ Reservation (reservation/*_test.go)
def reservation_cases():
    return load("reservation_cases.json")


def resv_profile(fit_weight: int = 1):
    from koordinator_amd.config import PLUGIN_FIT, PLUGIN_RESERVATION, NodeResourcesFitArgs
    return Profile(filters=(PLUGIN_FIT, PLUGIN_RESERVATION), scores={PLUGIN_FIT: fit_weight, PLUGIN_RESERVATION: 5000},
                   fit=NodeResourcesFitArgs(resources={k8s.CPU: 1, k8s.MEMORY: 1}))


def resv_pod(req: dict, labels=None, name="pod"):
    return k8s.Pod(name=name, labels=dict(labels or {}), priority=9500,
                   containers=[k8s.Container(requests=rlist(req))] if req else [k8s.Container()])


def build_resv_nodes(nodes, reservations, profile, node_pods=None):
    """nodes: [(name, allocatable dict)]; reservations: reservation.Reservation
    objects (their reserve pods and assigned pods are NodeInfo pods)."""
    from koordinator_amd import reservation as rv
    cluster = marshal.ClusterState(nodes=[k8s.Node(name=n, allocatable=rlist(a)) for n, a in nodes])
    for name, pods in (node_pods or {}).items():
        cluster.node_pods.setdefault(name, []).extend(pods)
    for r in reservations:
        cluster.node_pods.setdefault(r.node_name, []).append(r.reserve_pod())
    table = marshal.build_table(cluster, profile, NOW)
    idx = rv.reservation_columns(table, {n: i for i, (n, _) in enumerate(nodes)}, reservations)
    return table, idx


def match_all_owner():
    """Owners = [{}]: matches every pod (reservation.go:403)."""
    from koordinator_amd import reservation as rv
    return [rv.ReservationOwner()]
