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


# --------------------------------------------------------------- NodeResourceTopology objects
ANNOTATION_CPU_TOPOLOGY = "node.koordinator.sh/cpu-topology"                  # apis/extension/numa_aware.go:40
ANNOTATION_POD_CPU_ALLOCS = "node.koordinator.sh/pod-cpu-allocs"              # :42
ANNOTATION_KUBELET_CPU_MANAGER_POLICY = "kubelet.koordinator.sh/cpu-manager-policy"  # :149
ANNOTATION_NODE_RESERVATION = "node.koordinator.sh/reservation"               # node_reservation.go:28
ANNOTATION_SYSTEM_QOS_RESOURCE = "node.koordinator.sh/system-qos-resource"     # system_qos.go:24
ANNOTATION_RESOURCE_STATUS = "scheduling.koordinator.sh/resource-status"      # numa_aware.go:34

# nrtv1alpha1.TopologyManagerPolicy values -> convertToNUMATopologyPolicy (topology_options.go:213-225)
NRT_POLICIES = {"BestEffort": abi.NUMA_TOPO_BEST_EFFORT, "Restricted": abi.NUMA_TOPO_RESTRICTED,
                "SingleNUMANodePodLevel": abi.NUMA_TOPO_SINGLE_NUMA_NODE}


@dataclass
class Zone:
    """nrtv1alpha1.Zone: name "node-<id>", type "Node", resources name -> allocatable."""
    name: str
    type: str = "Node"
    resources: Optional[Dict[str, int]] = None      # cpu in milli, memory in bytes


@dataclass
class NodeResourceTopology:
    """The NRT object koordlet reports (one per node, same name)."""
    name: str
    annotations: Optional[Dict[str, str]] = None
    topology_policies: Optional[List[str]] = None
    zones: Optional[List[Zone]] = None


@dataclass
class TopologyOptions:
    """NewTopologyOptions (topology_options.go:90-158) as the engine needs it."""
    topology: Optional[Topology]
    reserved: List[int]
    kubelet_policy: Optional[dict]
    policy: int
    zones: List[Tuple[int, Dict[str, int]]]        # (NUMA node id, resources), ascending id
    amp_cpu: float


def _json_or_none(annotations: Dict[str, str], key: str):
    raw = annotations.get(key)
    if not raw:
        return None
    try:
        return json.loads(raw)
    except ValueError:
        return None                               # the reference logs the error and goes on without it


def topology_options(nrt: NodeResourceTopology) -> TopologyOptions:
    """NewTopologyOptions: CPU topology from the cpu-topology annotation,
    reserved CPUs = kubelet-managed pod allocs + kubelet reserved + node
    reservation + exclusive system-QoS CPUs, the NRT's topology policy, the
    "node-<id>" zones and the amplification ratios."""
    ann = nrt.annotations or {}
    topo = None
    ct = _json_or_none(ann, ANNOTATION_CPU_TOPOLOGY)
    infos = [CPUInfo(int(d["id"]), int(d.get("core", 0)), int(d.get("node", 0)), int(d.get("socket", 0)))
             for d in ((ct or {}).get("detail") or [])]
    if infos:
        try:
            topo = Topology(infos, shift_core=True)
        except TopologyError:
            topo = None                            # IsValid false / unsupported shape: no topology
    reserved = set()
    for a in (_json_or_none(ann, ANNOTATION_POD_CPU_ALLOCS) or []):   # getPodAllocsCPUSet :160-175
        if a.get("managedByKubelet") and a.get("uid") and a.get("cpuset"):
            try:
                reserved.update(parse_cpuset(a["cpuset"]))
            except ValueError:
                pass
    kp = _json_or_none(ann, ANNOTATION_KUBELET_CPU_MANAGER_POLICY)
    if kp and kp.get("reservedCPUs"):
        try:
            reserved.update(parse_cpuset(kp["reservedCPUs"]))
        except ValueError:
            pass
    nr = _json_or_none(ann, ANNOTATION_NODE_RESERVATION)            # GetReservedCPUs
    if nr and nr.get("reservedCPUs"):
        try:
            reserved.update(parse_cpuset(nr["reservedCPUs"]))
        except ValueError:
            pass
    sq = _json_or_none(ann, ANNOTATION_SYSTEM_QOS_RESOURCE)
    if sq and sq.get("cpusetExclusive", True) and sq.get("cpuset"):
        try:
            reserved.update(parse_cpuset(sq["cpuset"]))
        except ValueError:
            pass
    policy = abi.NUMA_TOPO_NONE
    for p in nrt.topology_policies or []:
        if p in NRT_POLICIES:
            policy = NRT_POLICIES[p]
            break
    zones = []
    for z in nrt.zones or []:                                        # extractNUMANodeResources :183-211
        if z.type != "Node":
            continue
        parts = z.name.split("node-")
        if len(parts) != 2 or not parts[1].isdigit():
            continue
        zones.append((int(parts[1]), dict(z.resources or {})))
    zones.sort(key=lambda x: x[0])
    return TopologyOptions(topo, sorted(reserved), kp, policy, zones, cpu_amplification_ratio(ann))


class NodeAllocation:
    """NodeAllocation (node_allocation.go:32-177) of one node: pod allocations
    by UID, per-CPU ref count + exclusive policy, per-NUMA-node allocated
    resources."""

    def __init__(self):
        self.pods: Dict[str, Tuple[List[int], str, List[Tuple[int, Dict[str, int]]]]] = {}
        self.cpus: Dict[int, List] = {}            # cpu -> [refcount, exclusive policy]
        self.resources: Dict[int, Dict[str, int]] = {}

    def add(self, uid: str, cpus: List[int], excl: str, numa_res: List[Tuple[int, Dict[str, int]]]):
        if uid in self.pods:                        # addPodAllocation :74-100
            return
        self.pods[uid] = (cpus, excl, numa_res)
        for c in cpus:
            info = self.cpus.setdefault(c, [0, ""])
            info[1] = excl
            info[0] += 1
        for node, res in numa_res:
            acc = self.resources.setdefault(node, {})
            for k, v in res.items():
                acc[k] = acc.get(k, 0) + v

    def release(self, uid: str):                   # release :102-131
        req = self.pods.pop(uid, None)
        if req is None:
            return
        cpus, _, numa_res = req
        for c in cpus:
            info = self.cpus.get(c)
            if info is None:
                continue
            info[0] -= 1
            if info[0] == 0:
                del self.cpus[c]
        for node, res in numa_res:
            acc = self.resources.get(node)
            if acc is not None:
                for k, v in res.items():              # SubtractWithNonNegativeResult
                    acc[k] = max(0, acc.get(k, 0) - v)

    def update(self, uid: str, cpus: List[int], excl: str, numa_res):
        self.release(uid)
        self.add(uid, cpus, excl, numa_res)


def available_cpus(topo: Topology, alloc: Optional[NodeAllocation], reserved: Iterable[int] = (),
                   preferred: Iterable[int] = ()) -> List[int]:
    """NodeAllocation.getAvailableCPUs with maxRefCount 1 (node_allocation.go:133-153):
    every CPU minus those still allocated once the preferred CPUs' RefCount
    dropped by one, minus the node's reserved CPUs."""
    held = {c: info[0] for c, info in (alloc.cpus.items() if alloc is not None else [])}
    for c in preferred:
        if c in held:
            held[c] -= 1
    res = set(reserved)
    return sorted(c for c in topo.cpu_of if held.get(c, 0) < 1 and c not in res)


def pod_allocation(annotations: Dict[str, str]):
    """podEventHandler.updatePod's parse (pod_eventhandler.go:94-131): (cpus,
    exclusive policy, NUMA node resources), or None when the pod holds
    neither a cpuset nor NUMA node resources (or an annotation is malformed)."""
    try:
        st = json.loads(annotations[ANNOTATION_RESOURCE_STATUS]) if annotations.get(ANNOTATION_RESOURCE_STATUS) else {}
        sp = json.loads(annotations[ANNOTATION_RESOURCE_SPEC]) if annotations.get(ANNOTATION_RESOURCE_SPEC) else {}
        cpus = parse_cpuset(st.get("cpuset", "") or "")
    except (ValueError, TypeError):
        return None
    nres = []
    for x in st.get("numaNodeResources") or []:
        res = {}
        for k, v in (x.get("resources") or {}).items():
            res[k] = int(v)
        nres.append((int(x.get("node", 0)), res))
    if not nres and not cpus:
        return None
    return cpus, sp.get("preferredCPUExclusivePolicy", "") or "", nres


def numa_row(table, i: int, opts: Optional[TopologyOptions], alloc: Optional[NodeAllocation], classes: ClassTable,
             labels: Dict[str, str], default_most_allocated: bool, frozen: bool = False):
    """Row i of the NodeNUMAResource columns from the node's TopologyOptions and
    NodeAllocation.  frozen: the class table is fixed (a row update); a
    topology it does not hold raises TopologyError (the caller reloads)."""
    for w in range(abi.NUMA_WORDS):
        table[f"numa_free{w}"][i] = 0
        table[f"numa_excl_pcpu{w}"][i] = 0
        table[f"numa_excl_numa{w}"][i] = 0
    table["numa_alloc_cnt"][i] = 0
    table["numa_zone_alloc"][i] = 0
    table["numa_zone_used"][i] = 0
    table["numa_amp_cpu"][i] = 1.0
    topo = opts.topology if opts is not None else None
    if topo is None:
        table["numa_class"][i] = -1
        table["numa_flags"][i] = node_numa_flags(labels, None, default_most_allocated) & ~(3 << abi.NODE_NUMA_POLICY_SHIFT)
        return
    if frozen and topo.key not in classes._index:
        raise TopologyError("a topology class the loaded snapshot does not hold (reload)")
    table["numa_class"][i] = classes.add(topo)
    cpus = (alloc.cpus if alloc is not None else {})
    allocated = [c for c in cpus if c in topo.pos_of]
    free = available_cpus(topo, alloc, opts.reserved)
    fm = topo.mask(free)
    pm = topo.mask([c for c in allocated if cpus[c][1] == "PCPULevel"])
    nm = topo.mask([c for c in allocated if cpus[c][1] == "NUMANodeLevel"])
    for w in range(abi.NUMA_WORDS):
        table[f"numa_free{w}"][i] = fm[w]
        table[f"numa_excl_pcpu{w}"][i] = pm[w]
        table[f"numa_excl_numa{w}"][i] = nm[w]
    table["numa_alloc_cnt"][i] = len(cpus)
    flags = node_numa_flags(labels, opts.kubelet_policy, default_most_allocated) & ~(3 << abi.NODE_NUMA_POLICY_SHIFT)
    pol = numa_topology_policy(labels) or opts.policy                       # getNUMATopologyPolicy: the label wins
    flags |= pol << abi.NODE_NUMA_POLICY_SHIFT
    table["numa_flags"][i] = flags
    if opts.zones and pol:  # zone rows are read only on topology-policy nodes
        node_rank = {n: r for r, n in enumerate(sorted({topo.details[c].node for c in topo.cpu_of}))}
        for nid, res in opts.zones:
            r = node_rank.get(nid)
            if r is None:
                continue
            table["numa_zone_alloc"][i, 0, r] = res.get("cpu", 0)
            table["numa_zone_alloc"][i, 1, r] = res.get("memory", 0)
            used = (alloc.resources.get(nid, {}) if alloc is not None else {})
            table["numa_zone_used"][i, 0, r] = used.get("cpu", 0)
            table["numa_zone_used"][i, 1, r] = used.get("memory", 0)
    table["numa_amp_cpu"][i] = opts.amp_cpu
