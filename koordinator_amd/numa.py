"""NodeNUMAResource host side: CPU topologies -> the engine's topology classes
(include/koordhip.h koordhip_numa_class), cpuset <-> position masks, and the
pod / node NUMA fields the Go shim marshals.

Reference: pkg/scheduler/plugins/nodenumaresource/cpu_topology.go:25-103
(CPUTopologyBuilder, CoreID = socket<<16 | core), topology_options.go:90-211
(NRT -> TopologyOptions), plugin.go:210-260 (PreFilter state),
apis/extension/numa_aware.go (annotations / labels).
"""
from __future__ import annotations

import json
from dataclasses import dataclass
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np

from . import abi


@dataclass(frozen=True)
class CPUInfo:
    cpu: int
    core: int
    node: int
    socket: int


class TopologyError(ValueError):
    pass


class Topology:
    """One CPU topology in the engine's core-major position order."""

    def __init__(self, infos: Sequence[CPUInfo], shift_core: bool = True):
        # CPUTopologyBuilder.AddCPUInfo (cpu_topology.go:44-70)
        details: Dict[int, CPUInfo] = {}
        tracker: Dict[int, Dict[int, set]] = {}
        num_sockets = num_nodes = num_cores = 0
        for i in infos:
            core = (i.socket << 16 | i.core) if shift_core else i.core
            details[i.cpu] = CPUInfo(i.cpu, core, i.node, i.socket)
            if i.socket not in tracker:
                num_sockets += 1
                tracker[i.socket] = {}
            if i.node not in tracker[i.socket]:
                num_nodes += 1
                tracker[i.socket][i.node] = set()
            if core not in tracker[i.socket][i.node]:
                num_cores += 1
                tracker[i.socket][i.node].add(core)
        self.details = details
        self.num_cpus, self.num_cores, self.num_nodes, self.num_sockets = len(details), num_cores, num_nodes, num_sockets
        if not self.valid:
            raise TopologyError("invalid CPU topology (IsValid, cpu_topology.go:77-79)")
        if self.num_cpus > abi.NUMA_MAX_CPUS:
            raise TopologyError(f"more than {abi.NUMA_MAX_CPUS} CPUs")
        by_core: Dict[int, List[int]] = {}
        for c, info in details.items():
            by_core.setdefault(info.core, []).append(c)
        cpc = self.num_cpus // self.num_cores
        if any(len(v) != cpc for v in by_core.values()) or len(by_core) * cpc != self.num_cpus:
            raise TopologyError("non-uniform CPUs per core")
        nodes = sorted({i.node for i in details.values()})
        sockets = sorted({i.socket for i in details.values()})
        if len(nodes) > abi.NUMA_MAX_NODES or len(sockets) > abi.NUMA_MAX_NODES:
            raise TopologyError("more than 8 NUMA nodes / sockets")
        for core, cpus in by_core.items():
            if len({details[c].node for c in cpus}) != 1 or len({details[c].socket for c in cpus}) != 1:
                raise TopologyError("a core spans NUMA nodes")
        self.cpus_per_core = cpc
        self.cpu_of: List[int] = []          # pos -> cpu id
        for core in sorted(by_core):
            self.cpu_of.extend(sorted(by_core[core]))
        self.pos_of = {c: p for p, c in enumerate(self.cpu_of)}
        node_rank = {n: r for r, n in enumerate(nodes)}
        sock_rank = {s: r for r, s in enumerate(sockets)}
        rec = np.zeros(1, abi.NUMA_CLASS_DTYPE)[0]
        rec["num_cpus"], rec["num_cores"] = self.num_cpus, self.num_cores
        rec["num_nodes"], rec["num_sockets"] = self.num_nodes, self.num_sockets
        rec["cpus_per_core"] = cpc
        for p, c in enumerate(self.cpu_of):
            rec["cpu_id"][p] = c
            rec["node_of"][p] = node_rank[details[c].node]
            rec["socket_of"][p] = sock_rank[details[c].socket]
        self.record = rec
        self.key = rec.tobytes()

    @property
    def valid(self) -> bool:
        return self.num_sockets != 0 and self.num_nodes != 0 and self.num_cores != 0 and self.num_cpus != 0

    def mask(self, cpus: Iterable[int]) -> np.ndarray:
        m = np.zeros(abi.NUMA_WORDS, np.uint64)
        for c in cpus:
            p = self.pos_of[c]
            m[p >> 6] |= np.uint64(1) << np.uint64(p & 63)
        return m

    def cpus(self, mask) -> List[int]:
        out = []
        for p in range(self.num_cpus):
            if (int(mask[p >> 6]) >> (p & 63)) & 1:
                out.append(self.cpu_of[p])
        return sorted(out)

    def all_mask(self) -> np.ndarray:
        return self.mask(self.cpu_of)


def reference_test_topology(num_sockets: int, nodes_per_socket: int, cores_per_node: int, cpus_per_core: int) -> Topology:
    """buildCPUTopologyForTest (cpu_accumulator_test.go:30-57): consecutive CPU
    ids per core, CoreID not socket-shifted."""
    infos = []
    node = core = cpu = 0
    for s in range(num_sockets):
        for _ in range(nodes_per_socket):
            for _ in range(cores_per_node):
                for _ in range(cpus_per_core):
                    infos.append(CPUInfo(cpu, core, node, s))
                    cpu += 1
                core += 1
            node += 1
    return Topology(infos, shift_core=False)


def linux_topology(sockets: int, nodes_per_socket: int, cores_per_node: int, threads: int = 2) -> Topology:
    """A Linux-style enumeration (as reported by koordlet's NRT cpu-topology
    annotation): hyperthread siblings are cpu and cpu + ncores."""
    ncores = sockets * nodes_per_socket * cores_per_node
    infos = []
    g = 0
    for s in range(sockets):
        for n in range(nodes_per_socket):
            for c in range(cores_per_node):
                for t in range(threads):
                    infos.append(CPUInfo(g + t * ncores, c + n * cores_per_node, s * nodes_per_socket + n, s))
                g += 1
    return Topology(infos, shift_core=True)


def parse_cpuset(s: str) -> List[int]:
    """cpuset.Parse ("0-3,8")."""
    out: List[int] = []
    s = s.strip()
    if not s:
        return out
    for part in s.split(","):
        if "-" in part:
            a, b = part.split("-")
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return sorted(set(out))


def format_cpuset(cpus: Iterable[int]) -> str:
    cs = sorted(set(cpus))
    parts, i = [], 0
    while i < len(cs):
        j = i
        while j + 1 < len(cs) and cs[j + 1] == cs[j] + 1:
            j += 1
        parts.append(str(cs[i]) if i == j else f"{cs[i]}-{cs[j]}")
        i = j + 1
    return ",".join(parts)


class ClassTable:
    """Deduplicated topology classes of a snapshot."""

    def __init__(self):
        self.classes: List[Topology] = []
        self._index: Dict[bytes, int] = {}

    def add(self, topo: Topology) -> int:
        i = self._index.get(topo.key)
        if i is None:
            i = len(self.classes)
            self._index[topo.key] = i
            self.classes.append(topo)
        return i

    def records(self) -> np.ndarray:
        out = np.zeros(len(self.classes), abi.NUMA_CLASS_DTYPE)
        for i, t in enumerate(self.classes):
            out[i] = t.record
        return out


# --------------------------------------------------------------- pod / node side
POLICY_CODES = {"": abi.CPUBIND_NONE, "Default": abi.CPUBIND_NONE, "FullPCPUs": abi.CPUBIND_FULL_PCPUS,
                "SpreadByPCPUs": abi.CPUBIND_SPREAD_BY_PCPUS}
EXCL_CODES = {"": abi.CPUEXCL_NONE, "None": abi.CPUEXCL_NONE, "PCPULevel": abi.CPUEXCL_PCPU,
              "NUMANodeLevel": abi.CPUEXCL_NUMA}
ANNOTATION_RESOURCE_SPEC = "scheduling.koordinator.sh/resource-spec"
LABEL_NODE_CPU_BIND_POLICY = "node.koordinator.sh/cpu-bind-policy"
LABEL_NODE_NUMA_ALLOCATE_STRATEGY = "node.koordinator.sh/numa-allocate-strategy"
LABEL_NUMA_TOPOLOGY_POLICY = "node.koordinator.sh/numa-topology-policy"


class PreFilterError(ValueError):
    pass


def prefilter_state(annotations: Dict[str, str], allow_cpuset: bool, cpu_request_milli: int, zero_request: bool,
                    default_bind_policy: str = "FullPCPUs") -> Tuple[int, int, int]:
    """NodeNUMAResource PreFilter (plugin.go:210-260) -> (pod flags, numa_cpus,
    numa_policy).  Raises PreFilterError for the reference's Error statuses."""
    if zero_request:
        return abi.POD_NUMA_SKIP, 0, 0
    spec = {}
    if ANNOTATION_RESOURCE_SPEC in annotations:
        try:
            spec = json.loads(annotations[ANNOTATION_RESOURCE_SPEC])
        except ValueError as e:  # GetResourceSpec error -> framework.Error (:211-214)
            raise PreFilterError(str(e))
    if not allow_cpuset:
        return 0, 0, 0
    policy = spec.get("preferredCPUBindPolicy", "") or ""
    if policy in ("", "Default"):
        policy = default_bind_policy
    required = spec.get("requiredCPUBindPolicy", "") or ""
    if required == "Default":
        required = default_bind_policy
    if required:
        policy = required
    if policy not in ("FullPCPUs", "SpreadByPCPUs"):
        return 0, 0, 0
    if cpu_request_milli % 1000 != 0:
        raise PreFilterError("the requested CPUs must be integer")  # :243-245
    if cpu_request_milli <= 0:
        return 0, 0, 0
    excl = spec.get("preferredCPUExclusivePolicy", "") or ""
    if excl not in EXCL_CODES:
        excl = ""
    pol = abi.numa_policy(POLICY_CODES.get(required, 0), POLICY_CODES[policy], EXCL_CODES[excl])
    return abi.POD_CPUSET, int(cpu_request_milli // 1000), pol


def node_numa_flags(labels: Dict[str, str], kubelet_policy: Optional[dict], default_most_allocated: bool) -> int:
    """GetNodeCPUBindPolicy (numa_aware.go:314-325) + GetNUMAAllocateStrategy
    (util.go:34-40)."""
    lab = labels.get(LABEL_NODE_CPU_BIND_POLICY, "")
    full_only = lab == "FullPCPUsOnly" or (
        kubelet_policy is not None and kubelet_policy.get("policy") == "static"
        and (kubelet_policy.get("options") or {}).get("full-pcpus-only") == "true")
    f = abi.NODE_CPUBIND_FULL_PCPUS_ONLY if full_only else (
        abi.NODE_CPUBIND_SPREAD_BY_PCPUS if lab == "SpreadByPCPUs" else abi.NODE_CPUBIND_NONE)
    strat = labels.get(LABEL_NODE_NUMA_ALLOCATE_STRATEGY, "")
    most = default_most_allocated if strat == "" else strat == "MostAllocated"
    if most:
        f |= abi.NODE_NUMA_MOST_ALLOCATED
    f |= numa_topology_policy(labels, kubelet_policy) << abi.NODE_NUMA_POLICY_SHIFT
    return f


NUMA_TOPOLOGY_POLICIES = {"": abi.NUMA_TOPO_NONE, "BestEffort": abi.NUMA_TOPO_BEST_EFFORT,
                          "Restricted": abi.NUMA_TOPO_RESTRICTED, "SingleNUMANode": abi.NUMA_TOPO_SINGLE_NUMA_NODE}


def numa_topology_policy(labels: Dict[str, str], nrt_policy: Optional[dict] = None) -> int:
    """getNUMATopologyPolicy (nodenumaresource/util.go:51-57): the node label
    node.koordinator.sh/numa-topology-policy, else the NRT's kubelet topology
    manager policy (convertToNUMATopologyPolicy, topology_options.go:213-225)."""
    lab = labels.get(LABEL_NUMA_TOPOLOGY_POLICY, "")
    if lab not in NUMA_TOPOLOGY_POLICIES:
        # createNUMATopologyPolicy (manager.go:112-123) has no policy for it: the
        # reference would dereference a nil Policy
        raise TopologyError(f"unknown NUMA topology policy {lab!r}")
    if lab:
        return NUMA_TOPOLOGY_POLICIES[lab]
    tm = (nrt_policy or {}).get("topologyManagerPolicy", "")
    return {"best-effort": abi.NUMA_TOPO_BEST_EFFORT, "restricted": abi.NUMA_TOPO_RESTRICTED,
            "single-numa-node": abi.NUMA_TOPO_SINGLE_NUMA_NODE}.get(tm, abi.NUMA_TOPO_NONE)


def zone_row(zones: Sequence[Tuple[int, int]]) -> np.ndarray:
    """NRT zones node-0..node-(M-1) -> the numa_zone_alloc row [2][NUMA_MAX_NODES]
    (cpu milli, memory bytes per zone)."""
    if len(zones) > abi.NUMA_MAX_NODES:
        raise TopologyError("more than 8 NUMA zones")
    row = np.zeros((2, abi.NUMA_MAX_NODES), np.int64)
    for k, (cpu_m, mem) in enumerate(zones):
        row[0, k], row[1, k] = cpu_m, mem
    return row


ANNOTATION_AMPLIFICATION_RATIO = "node.koordinator.sh/resource-amplification-ratio"


def cpu_amplification_ratio(annotations: Dict[str, str]) -> float:
    """GetNodeResourceAmplificationRatio(annotations, cpu)
    (apis/extension/node_resource_amplification.go:56-76) -> the numa_amp_cpu
    column value: the ratio, 1.0 when unset (the reference's -1 means "none"
    too: every use checks ratio <= 1).  A malformed annotation is an error
    (the reference's Filter then fails UnschedulableAndUnresolvable)."""
    import json
    raw = annotations.get(ANNOTATION_AMPLIFICATION_RATIO)
    if raw is None:
        return 1.0
    try:
        ratios = json.loads(raw)
        v = float(ratios.get("cpu", -1))
    except (ValueError, TypeError, AttributeError) as e:
        raise TopologyError(f"invalid {ANNOTATION_AMPLIFICATION_RATIO}: {e}")
    return v if v > 1.0 else 1.0
