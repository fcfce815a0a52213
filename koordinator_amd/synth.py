"""Seeded synthetic clusters and pod streams.

One generator, shared by the HIP engine and the oracle: it emits the SoA node
table and koordhip_pod records directly (vectorised, so 200k-node snapshots
build in well under a second).  All randomness is splitmix64 with the seed
0x6B6F6F7264 ("koord") by default, so every run of every config sees the same
bytes.  `cluster_objects` / `pod_objects` rebuild the same rows as Kubernetes
objects for the marshaller cross-check (tests/test_synth.py).

Units: cpu milli-cores, memory bytes, batch-cpu Value() (milli-core count).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Tuple

import numpy as np

from . import abi, k8s
from .config import Profile
from .snapshot import slot_col, NodeTable, pod_array

SEED = 0x6B6F6F7264
GI = 1 << 30
MI = 1 << 20
_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(seed: int, n: int, stream: int) -> np.ndarray:
    """n splitmix64 outputs of the sequence seeded by (seed, stream)."""
    with np.errstate(over="ignore"):
        base = np.uint64((seed ^ (stream * 0x9E3779B97F4A7C15)) & 0xFFFFFFFFFFFFFFFF)
        z = base + (np.arange(1, n + 1, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15))
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def uniform(seed: int, n: int, stream: int) -> np.ndarray:
    """U[0,1) doubles from the top 53 bits."""
    return (splitmix64(seed, n, stream) >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def choice(seed: int, n: int, stream: int, values) -> np.ndarray:
    v = np.asarray(values)
    idx = (splitmix64(seed, n, stream) % np.uint64(len(v))).astype(np.int64)
    return v[idx]


@dataclass
class ClusterSpec:
    n_nodes: int
    seed: int = SEED
    metric_missing_frac: float = 0.02
    pods_allocatable: int = 110


def make_cluster(spec: ClusterSpec, profile: Profile) -> NodeTable:
    """Node shapes / NodeMetric / Requested per SURVEY.md §8(d)."""
    n, s = spec.n_nodes, spec.seed
    la = profile.resolved().loadaware
    t = NodeTable.empty(n)
    cpu = choice(s, n, 1, [32, 64, 96, 128]).astype(np.int64) * 1000
    mem = choice(s, n, 2, [128, 256, 512, 1024]).astype(np.int64) * GI
    bcpu = np.floor(cpu * (0.2 + 0.4 * uniform(s, n, 3))).astype(np.int64)
    bmem = np.floor(mem * (0.2 + 0.4 * uniform(s, n, 4))).astype(np.int64)
    t["alloc0"][:] = cpu
    t["alloc1"][:] = mem
    t["alloc2"][:] = 0
    t["alloc3"][:] = bcpu
    t["alloc4"][:] = bmem
    t["alloc_pods"][:] = spec.pods_allocatable
    rc = np.floor(cpu * 0.5 * uniform(s, n, 5)).astype(np.int64)
    rm = np.floor(mem * 0.5 * uniform(s, n, 6)).astype(np.int64)
    t["requested0"][:] = rc
    t["requested1"][:] = rm
    t["requested3"][:] = np.floor(bcpu * 0.5 * uniform(s, n, 7)).astype(np.int64)
    t["requested4"][:] = np.floor(bmem * 0.5 * uniform(s, n, 8)).astype(np.int64)
    t["nz_cpu_m"][:] = rc
    t["nz_mem"][:] = rm
    t["npods"][:] = (splitmix64(s, n, 9) % np.uint64(41)).astype(np.int32)
    # NodeMetric: usage cpu U[0,0.8]*alloc, mem U[0.1,0.9]*alloc, never expired, 2% missing
    ucpu = np.floor(cpu * 0.8 * uniform(s, n, 10)).astype(np.int64)
    umem = np.floor(mem * (0.1 + 0.8 * uniform(s, n, 11))).astype(np.int64)
    has = uniform(s, n, 12) >= spec.metric_missing_frac
    t["la_alloc_cpu_m"][:] = cpu
    t["la_alloc_mem"][:] = mem
    t["la_used_cpu_m"][:] = np.where(has, ucpu, 0)
    t["la_used_mem"][:] = np.where(has, umem, 0)
    t["la_used_prod_cpu_m"][:] = 0
    t["la_used_prod_mem"][:] = 0
    t["laf_used_m0"][:] = np.where(has, ucpu, 0)          # cpu MilliValue
    t["laf_used_m1"][:] = np.where(has, umem * 1000, 0)   # memory MilliValue
    t["laf_total_m0"][:] = cpu
    t["laf_total_m1"][:] = mem * 1000
    t["laf_thr0"][:] = np.where(has, la.usage_thresholds.get(k8s.CPU, 0), 0)
    t["laf_thr1"][:] = np.where(has, la.usage_thresholds.get(k8s.MEMORY, 0), 0)
    flags = np.where(has, abi.LA_HAS_METRIC | abi.LA_FILTER_USAGE, 0)
    if la.prod_usage_thresholds:
        flags = flags | np.where(has, abi.LA_PROD_MODE, 0)
        t["laf_prod_thr0"][:] = np.where(has, la.prod_usage_thresholds.get(k8s.CPU, 0), 0)
        t["laf_prod_thr1"][:] = np.where(has, la.prod_usage_thresholds.get(k8s.MEMORY, 0), 0)
    t["la_flags"][:] = flags.astype(np.uint8)
    return t


# ------------------------------------------------------------------ NUMA (config 3)
# node cpu -> 2-socket topology (sockets, NUMA nodes per socket, cores per node, threads)
NUMA_SHAPES = {32000: (2, 1, 8, 2), 64000: (2, 1, 16, 2), 96000: (2, 1, 24, 2), 128000: (2, 2, 16, 2)}


@dataclass
class NumaSpec:
    no_topology_frac: float = 0.02     # nodes without a (valid) NodeResourceTopology
    max_prealloc_frac: float = 0.5     # cores already held by cpuset pods: U[0, max] of the cores
    excl_frac: float = 0.2             # share of pre-allocated cores held with an exclusive policy
    reserved_frac: float = 0.3         # nodes with kubelet-reserved CPUs (the first core)
    full_only_frac: float = 0.05       # node label cpu-bind-policy=FullPCPUsOnly
    spread_frac: float = 0.05          # node label cpu-bind-policy=SpreadByPCPUs
    most_allocated_frac: float = 0.3   # node label numa-allocate-strategy=MostAllocated
    linux_numbering: bool = True
    policy_frac: float = 0.0           # nodes with a NUMA topology policy (BestEffort / Restricted / SingleNUMANode)
    amp_frac: float = 0.0              # nodes with a CPU amplification ratio (1.25 / 1.5 / 2.0), no topology policy
    zone_used_frac: float = 0.6        # policy nodes: zone usage of non-cpuset pods, U[0, max] of the zone
    nodes_per_socket: int = 0          # NUMA nodes per socket (4: 2-socket NPS4 hosts, 8 NUMA zones); 0 = NUMA_SHAPES


def add_numa(t: NodeTable, spec: NumaSpec, profile: Profile, seed: int = SEED) -> NodeTable:
    """NodeNUMAResource columns for a synthetic cluster: a 2-socket topology
    matching each node's cpu, pre-allocated cpusets (some exclusive), reserved
    CPUs, node bind-policy / allocate-strategy labels."""
    from . import numa as nm
    n, s = t.n, seed + 7
    classes = nm.ClassTable()
    cls_of = {}
    for cpu, shape in NUMA_SHAPES.items():
        if spec.nodes_per_socket:
            sk, nps0, cpn0, th = shape
            per_socket = nps0 * cpn0
            if per_socket % spec.nodes_per_socket:
                raise ValueError(f"{per_socket} cores per socket do not split into {spec.nodes_per_socket} NUMA nodes")
            shape = (sk, spec.nodes_per_socket, per_socket // spec.nodes_per_socket, th)
        topo = nm.linux_topology(*shape) if spec.linux_numbering else nm.reference_test_topology(*shape)
        cls_of[cpu] = (classes.add(topo), topo)
    t.numa_classes = classes.records()
    no_topo = uniform(s, n, 40) < spec.no_topology_frac
    frac = uniform(s, n, 41) * spec.max_prealloc_frac
    reserved = uniform(s, n, 42) < spec.reserved_frac
    u_pol = uniform(s, n, 43)
    most = uniform(s, n, 44) < spec.most_allocated_frac
    default_most = profile.numa.default_most_allocated
    rnd = splitmix64(s, n * 4, 45)
    for i in range(n):
        cpu = int(t["alloc0"][i])
        if no_topo[i] or cpu not in cls_of:
            t["numa_class"][i] = -1
            continue
        ci, topo = cls_of[cpu]
        t["numa_class"][i] = ci
        ncores = topo.num_cores
        cpc = topo.cpus_per_core
        rng = np.random.default_rng(int(rnd[i * 4]))
        k = int(frac[i] * ncores)
        taken = rng.choice(ncores, size=k, replace=False) if k else np.zeros(0, np.int64)
        free = np.zeros(abi.NUMA_WORDS, np.uint64)
        ep = np.zeros(abi.NUMA_WORDS, np.uint64)
        en = np.zeros(abi.NUMA_WORDS, np.uint64)
        all_pos = np.arange(topo.num_cpus)
        used = np.zeros(topo.num_cpus, bool)
        for c in taken:
            used[c * cpc:(c + 1) * cpc] = True
            r = rng.random()
            if r < spec.excl_frac / 2:
                for p in range(c * cpc, (c + 1) * cpc):
                    ep[p >> 6] |= np.uint64(1) << np.uint64(p & 63)
            elif r < spec.excl_frac:
                for p in range(c * cpc, (c + 1) * cpc):
                    en[p >> 6] |= np.uint64(1) << np.uint64(p & 63)
        res = np.zeros(topo.num_cpus, bool)
        if reserved[i]:
            res[0:cpc] = True           # kubelet reserved: the first core
        for p in all_pos[~used & ~res]:
            free[p >> 6] |= np.uint64(1) << np.uint64(int(p) & 63)
        for w in range(abi.NUMA_WORDS):
            t[f"numa_free{w}"][i] = free[w]
            t[f"numa_excl_pcpu{w}"][i] = ep[w]
            t[f"numa_excl_numa{w}"][i] = en[w]
        t["numa_alloc_cnt"][i] = int(used.sum())
        f = 0
        if u_pol[i] < spec.full_only_frac:
            f = abi.NODE_CPUBIND_FULL_PCPUS_ONLY
        elif u_pol[i] < spec.full_only_frac + spec.spread_frac:
            f = abi.NODE_CPUBIND_SPREAD_BY_PCPUS
        if (most[i] if spec.most_allocated_frac > 0 else default_most):
            f |= abi.NODE_NUMA_MOST_ALLOCATED
        if spec.policy_frac and rng.random() < spec.policy_frac:
            # NRT zones node-0..: the zone's CPUs and an even memory share; used =
            # its cpuset CPUs + other pods' requests (sometimes past allocatable)
            f |= int(rng.integers(1, 4)) << abi.NODE_NUMA_POLICY_SHIFT
            nn = topo.num_nodes
            node_of = topo.record["node_of"][:topo.num_cpus]
            for k in range(nn):
                in_k = node_of == k
                t["numa_zone_alloc"][i, 0, k] = int(in_k.sum()) * 1000
                t["numa_zone_alloc"][i, 1, k] = int(t["alloc1"][i]) // nn
                extra = rng.random() * spec.zone_used_frac * 1.1
                t["numa_zone_used"][i, 0, k] = int((used & in_k).sum()) * 1000 + int(extra * in_k.sum() * 1000) // 100 * 100
                t["numa_zone_used"][i, 1, k] = int(extra * t["numa_zone_alloc"][i, 1, k]) // MI * MI
        if spec.amp_frac and not (f >> abi.NODE_NUMA_POLICY_SHIFT) and rng.random() < spec.amp_frac:
            # the node's allocatable cpu is the amplified figure (koord-manager's NodeResource)
            ratio = float(rng.choice([1.25, 1.5, 2.0]))
            t["numa_amp_cpu"][i] = ratio
            t["alloc0"][i] = int(np.ceil(t["alloc0"][i] * ratio))
            t["la_alloc_cpu_m"][i] = t["alloc0"][i]
            t["laf_total_m0"][i] = t["alloc0"][i]
        t["numa_flags"][i] = f
    return t


# ------------------------------------------------------------------ Reservation (config 5)
RESV_CPU = [4000, 8000, 16000]
RESV_MEM = [8 * GI, 16 * GI, 32 * GI]


@dataclass
class ResvSpec:
    node_frac: float = 0.10          # nodes holding an Available reservation
    groups: int = 8                  # distinct owner specs (e.g. one label selector per workload)
    allocate_once_frac: float = 0.5  # Spec.AllocateOnce (else reusable until full)
    aligned_frac: float = 0.15
    restricted_frac: float = 0.15
    unschedulable_frac: float = 0.02
    ordered_frac: float = 0.05       # reservation-order label, values 1..100
    cpu_only_frac: float = 0.05      # ResourceNames = {cpu}
    assigned_frac: float = 0.3       # already holding 1-3 pods
    slots: int = 1                   # reservations per node at most (koordhip_node_soa.resv_slots)
    multi_frac: float = 0.0          # P(a node holding q reservations holds a (q+1)-th), q < slots


def add_reservations(t: NodeTable, spec: ResvSpec, seed: int = SEED) -> NodeTable:
    """resv_* columns (the layout reservation.reservation_columns builds from
    objects) plus the reserve pods' and assigned pods' share of each node's
    Requested / NonZeroRequested / pod count.  Slot 0 draws from the streams
    of the one-per-node layout (so slots = 1 reproduces it); slot q >= 1 is
    filled on a multi_frac share of the nodes whose slot q - 1 is."""
    n, s = t.n, seed + 11
    t.set_resv_slots(max(t.resv_slots, spec.slots))
    prev = uniform(s, n, 60) < spec.node_frac
    slots = []
    for q in range(spec.slots):
        o = 0 if q == 0 else 1000 + 20 * q    # stream offset of slot q
        has = prev if q == 0 else prev & (uniform(s, n, o + 0) < spec.multi_frac)
        g = (splitmix64(s, n, 61 + o) % np.uint64(max(1, spec.groups))).astype(np.int64)
        rc = choice(s, n, 62 + o, RESV_CPU).astype(np.int64)
        cpu_only = uniform(s, n, 63 + o) < spec.cpu_only_frac
        rm = np.where(cpu_only, 0, choice(s, n, 64 + o, RESV_MEM).astype(np.int64))
        once = uniform(s, n, 65 + o) < spec.allocate_once_frac
        up = uniform(s, n, 66 + o)
        pol = np.where(up < spec.aligned_frac, abi.RESV_POLICY_ALIGNED,
                       np.where(up < spec.aligned_frac + spec.restricted_frac, abi.RESV_POLICY_RESTRICTED,
                                abi.RESV_POLICY_DEFAULT))
        unsched = uniform(s, n, 67 + o) < spec.unschedulable_frac
        ordered = uniform(s, n, 68 + o) < spec.ordered_frac
        order = (splitmix64(s, n, 69 + o) % np.uint64(100)).astype(np.int64) + 1
        assigned = np.where(uniform(s, n, 70 + o) < spec.assigned_frac,
                            (splitmix64(s, n, 71 + o) % np.uint64(3)).astype(np.int64) + 1, 0)
        fa = uniform(s, n, 72 + o)
        dc = np.where(assigned > 0, np.floor(rc * fa).astype(np.int64) // 100 * 100, 0)
        dm = np.where(assigned > 0, np.floor(rm * fa).astype(np.int64) // MI * MI, 0)
        f = (abi.RESV_PRESENT | abi.RESV_KEY_CPU | np.where(cpu_only, 0, abi.RESV_KEY_MEM)
             | np.where(once, abi.RESV_ALLOCATE_ONCE, 0) | np.where(unsched, abi.RESV_UNSCHEDULABLE, 0)
             | np.where(ordered, abi.RESV_ORDERED, 0) | (pol << abi.RESV_POLICY_SHIFT) | (g << abi.RESV_GROUP_SHIFT))
        col = lambda c: t[slot_col(c, q)]
        col("resv_flags")[:] = np.where(has, f, 0).astype(np.uint32)
        col("resv_alloc0")[:] = np.where(has, rc, 0)
        col("resv_alloc1")[:] = np.where(has, rm, 0)
        nzm = np.where(cpu_only, 200 * MI, rm)         # the reserve pod lists no memory: GetNonzeroRequests default
        col("resv_nz0")[:] = np.where(has, rc, 0)
        col("resv_nz1")[:] = np.where(has, nzm, 0)
        col("resv_allocated0")[:] = np.where(has, dc, 0)
        col("resv_allocated1")[:] = np.where(has, dm, 0)
        col("resv_assigned")[:] = np.where(has, assigned, 0).astype(np.int32)
        # the reserve pod and the pods it holds are NodeInfo pods
        t["requested0"][:] += np.where(has, rc + dc, 0)
        t["requested1"][:] += np.where(has, rm + dm, 0)
        t["nz_cpu_m"][:] += np.where(has, rc + dc, 0)
        t["nz_mem"][:] += np.where(has, nzm + dm, 0)
        t["npods"][:] += np.where(has, 1 + assigned, 0).astype(np.int32)
        slots.append((has & ordered, order))
        prev = has
    vals = np.unique(np.concatenate([order[m] for m, order in slots]))
    for q, (m, order) in enumerate(slots):
        t[slot_col("resv_order_rank", q)][:] = np.where(m, np.searchsorted(vals, order), 0).astype(np.int32)
    return t


def add_reserved_cpus(t: NodeTable, frac: float = 0.6, partial_frac: float = 0.4, excl_frac: float = 0.3,
                      seed: int = SEED, policy_nodes: bool = False) -> NodeTable:
    """Give a `frac` share of the reservations on NUMA nodes (a CPU topology; a
    topology policy only with `policy_nodes`) a cpuset: ~Allocatable cpu / 1000
    CPUs of the node's free ones, whole free cores first (the reserve pod's
    allocation in NodeAllocation, some with an exclusive policy; on a policy
    node its CPUs' zones also hold their count x 1000 of cpu in
    NodeAllocation.allocatedResources); on a `partial_frac` share of those with
    assigned pods some of the CPUs went to the assigned pods (still allocated,
    no longer reserved: RestoreReservation, nodenumaresource/reservation.go:84-104).
    Call after add_numa and add_reservations."""
    n, s = t.n, seed + 17
    rnd = splitmix64(s, n, 80)
    for i in range(n):
        cls = int(t["numa_class"][i])
        policy = (int(t["numa_flags"][i]) >> abi.NODE_NUMA_POLICY_SHIFT) & 3
        if cls < 0 or (policy and not policy_nodes):
            continue
        rng = np.random.default_rng(int(rnd[i]))
        rec = t.numa_classes[cls]
        ncpu, cpc = int(rec["num_cpus"]), int(rec["cpus_per_core"])
        for q in range(t.resv_slots):
            if not (int(t[slot_col("resv_flags", q)][i]) & abi.RESV_PRESENT) or rng.random() >= frac:
                continue
            free = [int(t[f"numa_free{w}"][i]) for w in range(abi.NUMA_WORDS)]
            isfree = lambda p: (free[p >> 6] >> (p & 63)) & 1
            want = max(1, int(t[slot_col("resv_alloc0", q)][i]) // 1000)
            start = int(rng.integers(0, ncpu // cpc))
            order = [(start + k) % (ncpu // cpc) for k in range(ncpu // cpc)]
            full = [c for c in order if all(isfree(c * cpc + x) for x in range(cpc))]
            pick = [c * cpc + x for c in full for x in range(cpc)][:want]
            if len(pick) < want:
                pick += [p for p in range(ncpu) if isfree(p) and p not in pick][:want - len(pick)]
            if not pick:
                continue
            r = rng.random()
            ex = "PCPULevel" if r < excl_frac / 2 else ("NUMANodeLevel" if r < excl_frac else "")
            m = [0] * abi.NUMA_WORDS
            for p in pick:
                m[p >> 6] |= 1 << (p & 63)
            for w in range(abi.NUMA_WORDS):
                t[f"numa_free{w}"][i] = np.uint64(free[w] & ~m[w] & 0xFFFFFFFFFFFFFFFF)
                if ex == "PCPULevel":
                    t[f"numa_excl_pcpu{w}"][i] |= np.uint64(m[w])
                elif ex == "NUMANodeLevel":
                    t[f"numa_excl_numa{w}"][i] |= np.uint64(m[w])
            t["numa_alloc_cnt"][i] += len(pick)
            if policy:
                node_of = rec["node_of"]
                for p in pick:
                    t["numa_zone_used"][i, 0, int(node_of[p])] += 1000
            if int(t[slot_col("resv_assigned", q)][i]) > 0 and rng.random() < partial_frac and len(pick) > 1:
                gone = rng.choice(len(pick), size=int(rng.integers(1, len(pick) // 2 + 1)), replace=False)
                for g in gone:
                    p = pick[int(g)]
                    m[p >> 6] &= ~(1 << (p & 63))
            for w in range(abi.NUMA_WORDS):
                t[slot_col(f"resv_cpus{w}", q)][i] = np.uint64(m[w])
    return t


@dataclass
class StaticSpec:
    """Node labels / taints / cordons and pod nodeSelector / required node
    affinity / tolerations for the upstream static filters."""
    tainted_frac: float = 0.15        # dedicated=<team>:NoSchedule
    noexec_frac: float = 0.03         # maintenance:NoExecute
    prefer_frac: float = 0.10         # soft=yes:PreferNoSchedule (Filter ignores it)
    spot_frac: float = 0.15           # spot=true:PreferNoSchedule (a second soft taint)
    unschedulable_frac: float = 0.02  # spec.unschedulable (cordoned)
    constrained_frac: float = 0.5     # pods with a non-empty static spec


ZONES = ["zone-a", "zone-b", "zone-c", "zone-d"]
TEAMS = ["team-1", "team-2"]


def static_nodes(n: int, spec: StaticSpec, seed: int = SEED):
    """NodeStatic records: zone / disktype / cpu-gen labels, taints, cordons."""
    from .nodefilters import NO_EXECUTE, NO_SCHEDULE, PREFER_NO_SCHEDULE, NodeStatic, Taint
    s = seed + 31
    zone = splitmix64(s, n, 90) % np.uint64(len(ZONES))
    ssd = uniform(s, n, 91) < 0.5
    gen = (splitmix64(s, n, 92) % np.uint64(4)).astype(np.int64) + 2
    tainted = uniform(s, n, 93) < spec.tainted_frac
    team = splitmix64(s, n, 94) % np.uint64(len(TEAMS))
    noexec = uniform(s, n, 95) < spec.noexec_frac
    prefer = uniform(s, n, 96) < spec.prefer_frac
    cordon = uniform(s, n, 97) < spec.unschedulable_frac
    spot = uniform(s, n, 100) < spec.spot_frac
    out = []
    for i in range(n):
        labels = {"topology.kubernetes.io/zone": ZONES[int(zone[i])], "cpu-gen": str(int(gen[i]))}
        if ssd[i]:
            labels["disktype"] = "ssd"
        taints = []
        if tainted[i]:
            taints.append(Taint("dedicated", TEAMS[int(team[i])], NO_SCHEDULE))
        if noexec[i]:
            taints.append(Taint("maintenance", "", NO_EXECUTE))
        if prefer[i]:
            taints.append(Taint("soft", "yes", PREFER_NO_SCHEDULE))
        if spot[i]:
            taints.append(Taint("spot", "true", PREFER_NO_SCHEDULE))
        out.append(NodeStatic(labels=labels, taints=taints, unschedulable=bool(cordon[i]), name=f"node-{i}"))
    return out


def static_templates():
    """Pod static specs the stream draws from (template 0: unconstrained)."""
    from .nodefilters import PodStatic, Toleration
    from .reservation import NodeSelectorRequirement as R, NodeSelectorTerm as T
    zone = "topology.kubernetes.io/zone"
    return [
        PodStatic(),
        PodStatic(node_selector={zone: "zone-a"}),
        PodStatic(node_selector={"disktype": "ssd"}),
        PodStatic(required_terms=[T([R(zone, "In", ["zone-b", "zone-c"])])]),
        PodStatic(required_terms=[T([R(zone, "NotIn", ["zone-a"]), R("disktype", "Exists")])]),
        PodStatic(required_terms=[T([R("cpu-gen", "Gt", ["3"])]), T([R("disktype", "DoesNotExist")])]),
        PodStatic(tolerations=[Toleration("dedicated", "Equal", "team-1", "NoSchedule")]),
        PodStatic(tolerations=[Toleration("dedicated", "Exists")]),
        PodStatic(node_selector={zone: "zone-d"}, tolerations=[Toleration(operator="Exists")]),
        PodStatic(tolerations=[Toleration("node.kubernetes.io/unschedulable", "Exists", "", "NoSchedule"),
                               Toleration("maintenance", "Exists", "", "NoExecute")]),
        PodStatic(required_terms=[T([R("cpu-gen", "Lt", ["4"])], [R("metadata.name", "NotIn", ["node-0"])])]),
        PodStatic(required_terms=[]),  # an empty term list matches no node
        # preferred terms (NodeAffinity Score) / PreferNoSchedule tolerations (TaintToleration Score)
        PodStatic(preferred_terms=[(10, T([R(zone, "In", ["zone-a"])])), (5, T([R("disktype", "Exists")]))]),
        PodStatic(preferred_terms=[(1, T([R("cpu-gen", "Gt", ["3"])])),
                                   (50, T([], [R("metadata.name", "In", ["node-1", "node-2", "node-3"])]))],
                  tolerations=[Toleration("soft", "Equal", "yes", "PreferNoSchedule")]),
        PodStatic(node_selector={"disktype": "ssd"},
                  preferred_terms=[(100, T([R(zone, "NotIn", ["zone-b"])])), (0, T([R("cpu-gen", "Exists")])),
                                   (7, T())]),
        PodStatic(tolerations=[Toleration("spot", "Exists", "", "NoSchedule")]),   # not a PreferNoSchedule one
        PodStatic(tolerations=[Toleration("spot", "Exists")],
                  preferred_terms=[(3, T([R("cpu-gen", "Lt", ["4"])])), (3, T([R("disktype", "DoesNotExist")]))]),
    ]


def add_static(t: NodeTable, pods: np.ndarray, spec: StaticSpec, profile: Profile, seed: int = SEED):
    """Static classes for the pods (pods['static_class']), the static_allow
    column for the profile's enabled static filters and, on a table with the
    sequential cycle's columns, the NodeAffinity / TaintToleration raw Scores
    (static_score).  Returns (node specs, pod class specs) for tests."""
    from .config import STATIC_FILTERS
    from .nodefilters import StaticClasses, static_allow, static_scores
    nodes = static_nodes(t.n, spec, seed)
    tmpl = static_templates()
    n, s = len(pods), seed + 37
    constrained = uniform(s, n, 98) < spec.constrained_frac
    pick = (splitmix64(s, n, 99) % np.uint64(len(tmpl) - 1)).astype(np.int64) + 1
    cls = StaticClasses()
    cls.classify(tmpl[0])
    ids = [cls.classify(tmpl[int(pick[j])]) if constrained[j] else 0 for j in range(n)]
    pods["static_class"][:] = np.asarray(ids, dtype=np.int32)
    t["static_allow"][:] = static_allow(nodes, cls, [f for f in profile.filters if f in STATIC_FILTERS])
    if t.has_ext:
        t["static_score"][:] = static_scores(nodes, cls)
    return nodes, cls


@dataclass
class StreamSpec:
    n_pods: int
    be_frac: float = 0.0
    seed: int = SEED
    cpuset_frac: float = 0.0   # share of LS pods that are LSR/LSE cpuset pods (NodeNUMAResource)
    resv_match_frac: float = 0.0  # pods matching one reservation owner group (Reservation)
    resv_groups: int = 8
    resv_affinity_frac: float = 0.0  # pods with a required reservation affinity (match: a subset of their group)


LS_CPU = [250, 500, 1000, 2000, 4000]
LS_MEM = [256 * MI, 512 * MI, 1 * GI, 2 * GI, 4 * GI, 8 * GI]
BE_CPU = [500, 1000, 2000, 4000]
BE_MEM = [512 * MI, 1 * GI, 2 * GI, 4 * GI, 8 * GI]


def _round_half_away(x: np.ndarray) -> np.ndarray:
    f = np.floor(x)
    return (f + ((x - f) >= 0.5)).astype(np.int64)


def make_pods(spec: StreamSpec, profile: Profile) -> np.ndarray:
    """LS: prod, Burstable, 50% with limit = 2x request; BE: koord.sh/qosClass=BE,
    priority 5000, batch-cpu/batch-memory with limit = request."""
    n, s = spec.n_pods, spec.seed + 1
    la = profile.resolved().loadaware
    fc = la.estimated_scaling_factors.get(k8s.CPU, 85)
    fm = la.estimated_scaling_factors.get(k8s.MEMORY, 70)
    pods = pod_array(n)
    be = uniform(s, n, 20) < spec.be_frac
    burst = uniform(s, n, 21) < 0.5
    ls_cpu = choice(s, n, 22, LS_CPU).astype(np.int64)
    ls_mem = choice(s, n, 23, LS_MEM).astype(np.int64)
    be_cpu = choice(s, n, 24, BE_CPU).astype(np.int64)
    be_mem = choice(s, n, 25, BE_MEM).astype(np.int64)
    # LS (prod): requests cpu/mem; limit = 2x request when bursting else = request
    lim_mult = np.where(burst, 2, 1)
    ls_est_cpu = np.where(burst, ls_cpu * 2, _round_half_away(ls_cpu.astype(np.float64) * fc / 100))
    ls_est_cpu = np.minimum(ls_est_cpu, ls_cpu * lim_mult)
    ls_est_mem = np.where(burst, ls_mem * 2, _round_half_away(ls_mem.astype(np.float64) * fm / 100))
    ls_est_mem = np.minimum(ls_est_mem, ls_mem * lim_mult)
    be_est_cpu = np.minimum(_round_half_away(be_cpu.astype(np.float64) * fc / 100), be_cpu)
    be_est_mem = np.minimum(_round_half_away(be_mem.astype(np.float64) * fm / 100), be_mem)
    req = pods["req"]
    req[:, abi.RES_CPU] = np.where(be, 0, ls_cpu)
    req[:, abi.RES_MEM] = np.where(be, 0, ls_mem)
    req[:, abi.RES_BCPU] = np.where(be, be_cpu, 0)
    req[:, abi.RES_BMEM] = np.where(be, be_mem, 0)
    # BE pods request no cpu/memory -> non-zero defaults 100m / 200MiB
    pods["nz_cpu_m"] = np.where(be, 100, ls_cpu)
    pods["nz_mem"] = np.where(be, 200 * MI, ls_mem)
    pods["est_cpu"] = np.where(be, be_est_cpu, ls_est_cpu)
    pods["est_mem"] = np.where(be, be_est_mem, ls_est_mem)
    pods["flags"] = np.where(be, abi.POD_HAS_REQ | abi.POD_REQ_BCPU | abi.POD_REQ_BMEM,
                             abi.POD_PROD | abi.POD_HAS_REQ | abi.POD_KEY_CPU | abi.POD_KEY_MEM).astype(np.uint32)
    if spec.cpuset_frac > 0:
        _make_cpuset_pods(pods, be, spec, fc, fm)
    if spec.resv_match_frac > 0:
        m = uniform(s, n, 50) < spec.resv_match_frac
        g = (splitmix64(s, n, 51) % np.uint64(max(1, spec.resv_groups))).astype(np.uint64)
        pods["resv_match"] = np.where(m, np.uint64(1) << g, np.uint64(0))
        if spec.resv_affinity_frac > 0:
            # a required reservation affinity: KOORDHIP_POD_RESV_AFFINITY, and a
            # second owner group standing for "the group's reservations whose
            # labels the affinity selects" (or none: unschedulable everywhere)
            a = uniform(s, n, 52) < spec.resv_affinity_frac
            g2 = (splitmix64(s, n, 53) % np.uint64(max(1, spec.resv_groups))).astype(np.uint64)
            keep = uniform(s, n, 54) < 0.8
            pods["flags"] |= np.where(a, abi.POD_RESV_AFFINITY, 0).astype(pods["flags"].dtype)
            pods["resv_match"] = np.where(a, np.where(keep, np.uint64(1) << g2, np.uint64(0)), pods["resv_match"])
    return pods


CPUSET_CPUS = [1, 2, 4, 8, 16]
# (required, preferred, exclusive) mixes of LSR/LSE resource-spec annotations
CPUSET_POLICIES = [
    (abi.CPUBIND_NONE, abi.CPUBIND_FULL_PCPUS, abi.CPUEXCL_NONE),          # default policy (FullPCPUs)
    (abi.CPUBIND_NONE, abi.CPUBIND_FULL_PCPUS, abi.CPUEXCL_NONE),
    (abi.CPUBIND_NONE, abi.CPUBIND_SPREAD_BY_PCPUS, abi.CPUEXCL_NONE),
    (abi.CPUBIND_FULL_PCPUS, abi.CPUBIND_FULL_PCPUS, abi.CPUEXCL_NONE),
    (abi.CPUBIND_SPREAD_BY_PCPUS, abi.CPUBIND_SPREAD_BY_PCPUS, abi.CPUEXCL_NONE),
    (abi.CPUBIND_NONE, abi.CPUBIND_SPREAD_BY_PCPUS, abi.CPUEXCL_PCPU),
    (abi.CPUBIND_FULL_PCPUS, abi.CPUBIND_FULL_PCPUS, abi.CPUEXCL_NUMA),
    (abi.CPUBIND_SPREAD_BY_PCPUS, abi.CPUBIND_SPREAD_BY_PCPUS, abi.CPUEXCL_PCPU),
]


def _make_cpuset_pods(pods, be, spec: StreamSpec, fc: int, fm: int):
    """LSR/LSE prod pods with integral cpu (Guaranteed: limit = request)."""
    n, s = spec.n_pods, spec.seed + 1
    cs = (~be) & (uniform(s, n, 30) < spec.cpuset_frac)
    ncpu = choice(s, n, 31, CPUSET_CPUS).astype(np.int64)
    pol = (splitmix64(s, n, 32) % np.uint64(len(CPUSET_POLICIES))).astype(np.int64)
    mem = choice(s, n, 33, LS_MEM).astype(np.int64)
    req = pods["req"]
    req[cs, abi.RES_CPU] = ncpu[cs] * 1000
    req[cs, abi.RES_MEM] = mem[cs]
    pods["nz_cpu_m"][cs] = ncpu[cs] * 1000
    pods["nz_mem"][cs] = mem[cs]
    pods["est_cpu"][cs] = np.minimum(_round_half_away((ncpu[cs] * 1000).astype(np.float64) * fc / 100),
                                     ncpu[cs] * 1000)
    pods["est_mem"][cs] = np.minimum(_round_half_away(mem[cs].astype(np.float64) * fm / 100), mem[cs])
    pods["flags"][cs] |= np.uint32(abi.POD_CPUSET)
    pods["numa_cpus"][cs] = ncpu[cs].astype(np.int32)
    codes = np.array([abi.numa_policy(*x) for x in CPUSET_POLICIES], np.uint32)
    pods["numa_policy"][cs] = codes[pol[cs]]


def pod_objects(spec: StreamSpec, limit: int = None) -> List[k8s.Pod]:
    """The same stream as Kubernetes objects (for the marshaller cross-check)."""
    n, s = spec.n_pods, spec.seed + 1
    be = uniform(s, n, 20) < spec.be_frac
    burst = uniform(s, n, 21) < 0.5
    ls_cpu = choice(s, n, 22, LS_CPU)
    ls_mem = choice(s, n, 23, LS_MEM)
    be_cpu = choice(s, n, 24, BE_CPU)
    be_mem = choice(s, n, 25, BE_MEM)
    out = []
    for i in range(n if limit is None else min(n, limit)):
        if be[i]:
            r = {k8s.BATCH_CPU: k8s.Q(int(be_cpu[i])), k8s.BATCH_MEMORY: k8s.Q(int(be_mem[i]))}
            out.append(k8s.Pod(name=f"be-{i}", labels={k8s.LABEL_POD_QOS: k8s.QOS_BE}, priority=5000,
                               containers=[k8s.Container(requests=dict(r), limits=dict(r))]))
        else:
            m = 2 if burst[i] else 1
            r = {k8s.CPU: k8s.Q(f"{int(ls_cpu[i])}m"), k8s.MEMORY: k8s.Q(int(ls_mem[i]))}
            lim = {k8s.CPU: k8s.Q(f"{int(ls_cpu[i]) * m}m"), k8s.MEMORY: k8s.Q(int(ls_mem[i]) * m)}
            out.append(k8s.Pod(name=f"ls-{i}", priority=9500, containers=[k8s.Container(requests=r, limits=lim)]))
    return out


@dataclass
class DevSpec:
    """DeviceShare cluster: a share of the nodes hold GPUs (one model per
    node: 4 or 8 GPUs of 16 / 32 / 80 GiB, gpu-core = gpu-memory-ratio = 100
    each, a few unhealthy) and some RDMA NICs; already-running device pods
    hold part of them (deviceUsed).  Node allocatable carries the device
    scalars (koordlet reports them): nvidia.com/gpu = GPU count, gpu-core /
    gpu-memory-ratio = 100 per GPU, gpu-memory, rdma = 100 per NIC."""
    gpu_frac: float = 0.3
    rdma_frac: float = 0.5        # of the GPU nodes
    unhealthy_frac: float = 0.03  # of the GPUs
    used_frac: float = 0.4        # of the GPUs, partly used by running pods
    no_entry_frac: float = 0.2    # of the non-GPU nodes: no Device CR (no nodeDevice entry)


def add_devices(t: NodeTable, spec: DevSpec, seed: int = SEED) -> NodeTable:
    """The DeviceShare columns (dev_*) and the extended scalars' allocatable /
    requested (xalloc / xrequested) of a synthetic cluster."""
    from .deviceshare import XRES_INDEX, NVIDIA_GPU, KOORD_GPU, GPU_CORE, GPU_MEMORY, GPU_MEMORY_RATIO, RDMA
    n, sd = t.n, seed + 7
    t.enable_ext(dev_slots=8)
    gpu = uniform(sd, n, 1) < spec.gpu_frac
    ngpu = np.where(uniform(sd, n, 2) < 0.5, 4, 8)
    mem = choice(sd, n, 3, [16 * GI, 32 * GI, 80 * GI]).astype(np.int64)
    rdma = gpu & (uniform(sd, n, 4) < spec.rdma_frac)
    entry = gpu | (uniform(sd, n, 5) >= spec.no_entry_frac)
    t["dev_present"][:] = entry.astype(np.uint8)
    G = abi.DEV_GPU
    for s in range(8):
        on = gpu & (s < ngpu)
        t["dev_minor"][on, G, s] = s
        healthy = on & (uniform(sd, n, 10 + s) >= spec.unhealthy_frac)
        t["dev_total"][healthy, G, s, 0] = 100
        t["dev_total"][healthy, G, s, 1] = 100
        t["dev_total"][healthy, G, s, 2] = mem[healthy]
        # running pods hold a share of some GPUs: 25 / 50 / 100 % of core / ratio / memory
        part = healthy & (uniform(sd, n, 30 + s) < spec.used_frac)
        share = choice(sd, n, 40 + s, [25, 50, 100]).astype(np.int64)
        t["dev_used"][part, G, s, 0] = share[part]
        t["dev_used"][part, G, s, 1] = share[part]
        t["dev_used"][part, G, s, 2] = mem[part] * share[part] // 100
    for s in range(2):
        on = rdma
        t["dev_minor"][on, abi.DEV_RDMA, s] = s
        t["dev_total"][on, abi.DEV_RDMA, s, 0] = 100
    xa, xr = t["xalloc"], t["xrequested"]
    used = t["dev_used"][:, G]
    # the slo-controller syncs the healthy GPUs' resources into the node's
    # allocatable, koordinator.sh/gpu = their gpu-core sum
    # (noderesource/device_resource_calculator.go:84-100)
    tot = t["dev_total"][:, G]
    xa[gpu, XRES_INDEX[NVIDIA_GPU]] = ngpu[gpu]
    xa[:, XRES_INDEX[KOORD_GPU]] = tot[:, :, 0].sum(axis=1)
    xa[:, XRES_INDEX[GPU_CORE]] = tot[:, :, 0].sum(axis=1)
    xa[:, XRES_INDEX[GPU_MEMORY_RATIO]] = tot[:, :, 1].sum(axis=1)
    xa[:, XRES_INDEX[GPU_MEMORY]] = tot[:, :, 2].sum(axis=1)
    xa[rdma, XRES_INDEX[RDMA]] = 200
    xr[:, XRES_INDEX[GPU_CORE]] = used[:, :, 0].sum(axis=1)
    xr[:, XRES_INDEX[GPU_MEMORY_RATIO]] = used[:, :, 1].sum(axis=1)
    xr[:, XRES_INDEX[GPU_MEMORY]] = used[:, :, 2].sum(axis=1)
    return t


@dataclass
class DevResvSpec:
    """Reservations holding devices (after add_reservations and add_devices):
    on a GPU node with an Available reservation in slot 0, with probability
    `frac` the reservation's reserve pod holds one or two of its GPUs (25, 50 or
    100 % of each) and its assigned pods a share of that (0, 1/4 or 1/2); the
    reservation's AllocatePolicy is drawn from `policy` (Default, Aligned,
    Restricted)."""
    frac: float = 0.8
    policy: tuple = (0.5, 0.25, 0.25)
    # the reserve pod requests its GPUs in the koordinator.sh/gpu-core +
    # gpu-memory-ratio form: those scalars are the reservation's extended
    # Allocatable (resv_xalloc), its assigned pods' share its Allocated
    # (resv_xallocated), and both sit in the node's Requested (xrequested)
    scalars: bool = True


def add_device_reservations(t: NodeTable, spec: DevResvSpec = DevResvSpec(), seed: int = SEED) -> NodeTable:
    """The resv_dev_* columns: both allocations join dev_used, as in the
    nodeDevice cache (the reserve pod and its assigned pods are pods of the node)."""
    from .deviceshare import GPU_CORE, GPU_MEMORY_RATIO, XRES_INDEX
    G = abi.DEV_GPU
    rng = np.random.default_rng(seed + 1000)
    t.enable_resv_dev()
    pol = rng.choice(3, size=t.n, p=list(spec.policy))
    for i in range(t.n):
        if not (t["resv_flags"][i] & abi.RESV_PRESENT) or not t["dev_present"][i]:
            continue
        gpus = [s for s in range(t.dev_slots) if t["dev_minor"][i, G, s] >= 0 and t["dev_total"][i, G, s].any()]
        if not gpus or rng.random() >= spec.frac:
            continue
        for s in rng.choice(gpus, size=min(len(gpus), int(rng.integers(1, 3))), replace=False):
            tot = t["dev_total"][i, G, s]
            frac = int(rng.choice([25, 50, 100]))
            a = np.array([tot[0] * frac // 100, frac, tot[2] * frac // 100], np.int64)
            a = np.minimum(a, np.maximum(tot - t["dev_used"][i, G, s], 0))
            d = np.minimum(a * int(rng.choice([0, 0, 1, 2])) // 4, a)
            if not a.any():
                continue
            t["resv_dev"][i, 0, G, s] = a
            t["resv_dev"][i, 1, G, s] = d
            t["dev_used"][i, G, s] += a + d
        if t["resv_dev"][i, 0].any():
            t["resv_dev_slot"][i] = 0
            if spec.scalars:
                A, D = t["resv_dev"][i, 0, G], t["resv_dev"][i, 1, G]
                for k, name in ((0, GPU_CORE), (1, GPU_MEMORY_RATIO)):
                    j = XRES_INDEX[name]
                    t["resv_xalloc"][i, j] = int(A[:, k].sum())
                    t["resv_xallocated"][i, j] = int(D[:, k].sum())
                    t["xrequested"][i, j] += int(A[:, k].sum()) + int(D[:, k].sum())
            f = int(t["resv_flags"][i]) & ~(3 << abi.RESV_POLICY_SHIFT)
            t["resv_flags"][i] = f | (int(pol[i]) << abi.RESV_POLICY_SHIFT)
    return t


@dataclass
class DevStreamSpec:
    """Device pods of a stream (their koordhip_pod_ext records): a share of the
    pods request GPUs in the reference's request forms -- koordinator.sh/gpu
    (a percentage of one GPU, or 200 = two GPUs), nvidia.com/gpu (whole
    GPUs), gpu-core + gpu-memory-ratio, gpu-memory alone -- some with RDMA."""
    frac: float = 0.2
    rdma_frac: float = 0.2
    seed: int = SEED


def make_device_ext(n: int, spec: DevStreamSpec) -> np.ndarray:
    from .deviceshare import XRES_INDEX, NVIDIA_GPU, KOORD_GPU, GPU_CORE, GPU_MEMORY, GPU_MEMORY_RATIO, RDMA
    sd = spec.seed + 9
    ext = abi.pod_ext_array(n)
    dev = uniform(sd, n, 1) < spec.frac
    form = choice(sd, n, 2, [0, 1, 2, 3]).astype(np.int64)
    pct = choice(sd, n, 3, [25, 50, 100, 200]).astype(np.int64)
    whole = choice(sd, n, 4, [1, 1, 2, 4]).astype(np.int64)
    gmem = choice(sd, n, 5, [4 * GI, 8 * GI, 16 * GI]).astype(np.int64)
    rd = dev & (uniform(sd, n, 6) < spec.rdma_frac)
    for j in np.flatnonzero(dev):
        x = ext[j]
        x["flags"] = abi.PODX_DEVICE
        g = x["dev_req"][abi.DEV_GPU]
        f = int(form[j])
        if f == 0:      # koordinator.sh/gpu: core = ratio = the percentage
            g[0] = g[1] = pct[j]
            xr = {KOORD_GPU: int(pct[j])}
        elif f == 1:    # nvidia.com/gpu: whole GPUs
            g[0] = g[1] = 100 * whole[j]
            xr = {NVIDIA_GPU: int(whole[j])}
        elif f == 2:    # gpu-core + gpu-memory-ratio
            g[0] = pct[j] if pct[j] <= 100 else 100
            g[1] = pct[j]
            xr = {GPU_CORE: int(g[0]), GPU_MEMORY_RATIO: int(g[1])}
        else:           # gpu-memory alone
            g[2] = gmem[j]
            xr = {GPU_MEMORY: int(gmem[j])}
        if rd[j]:
            x["dev_req"][abi.DEV_RDMA, 0] = 100
            xr[RDMA] = 100
        for name, v in xr.items():
            x["xreq"][XRES_INDEX[name]] = v
            x["xmask"] |= 1 << XRES_INDEX[name]
    return ext


@dataclass
class SpreadSpec:
    """PodTopologySpread: zone / rack / hostname keys (a few nodes without a zone
    or rack label), three apps with running pods, and pods of five spread
    classes (hard zone; soft zone + hostname; hard hostname + soft rack; rack
    affinity-restricted hard + soft zone; hard zone + hostname)."""
    zones: int = 6
    racks: int = 24
    no_zone_frac: float = 0.03
    no_rack_frac: float = 0.05
    running_frac: float = 0.4     # nodes holding running pods of an app
    pod_frac: float = 0.6         # pods with constraints
    seed: int = SEED


# the constraint table: (app, key) -- keys 0 zone, 1 rack, 2 hostname
SPREAD_CONS = [(0, 0), (1, 0), (2, 0), (0, 1), (1, 1), (2, 1), (0, 2), (1, 2)]
# per class: (hard key mask, soft key mask, [(key, hard, max_skew)])
SPREAD_CLASSES = [
    (0b001, 0b000, [(0, True, 1)]),
    (0b000, 0b101, [(0, False, 1), (2, False, 2)]),
    (0b100, 0b010, [(2, True, 2), (1, False, 1)]),
    (0b010, 0b001, [(1, True, 3), (0, False, 2)]),
    (0b101, 0b000, [(0, True, 2), (2, True, 1)]),
]


def add_spread(t: NodeTable, ext: np.ndarray, spec: SpreadSpec) -> NodeTable:
    """The pts_* columns of a synthetic cluster and the pts_* fields of the
    pods' koordhip_pod_ext records (class 3's required affinity: the nodes of
    even zones)."""
    from .snapshot import PtsMeta
    n, sd = t.n, spec.seed + 13
    t.enable_pts(PtsMeta(keys=3, hostname=0b100, ndom=[spec.zones, spec.racks, 0, 0],
                         cons_key=[k for _, k in SPREAD_CONS], classes=len(SPREAD_CLASSES)))
    zone = (splitmix64(sd, n, 1) % np.uint64(spec.zones)).astype(np.int32)
    rack = (splitmix64(sd, n, 2) % np.uint64(spec.racks)).astype(np.int32)
    zone[uniform(sd, n, 3) < spec.no_zone_frac] = -1
    rack[uniform(sd, n, 4) < spec.no_rack_frac] = -1
    dom = t["pts_dom"]
    dom[:, 0], dom[:, 1], dom[:, 2] = zone, rack, np.arange(n, dtype=np.int32)
    running = np.zeros((n, 3), np.int32)
    for a in range(3):
        on = uniform(sd, n, 10 + a) < spec.running_frac
        running[:, a] = np.where(on, (splitmix64(sd, n, 20 + a) % np.uint64(4)).astype(np.int32) + 1, 0)
    for c, (a, _) in enumerate(SPREAD_CONS):
        t["pts_cnt"][:, c] = running[:, a]
    has = lambda mask: np.all([dom[:, k] >= 0 for k in range(3) if (mask >> k) & 1] or [np.ones(n, bool)], axis=0)
    elig = np.zeros(n, np.uint16)
    for s_, (hard, soft, _) in enumerate(SPREAD_CLASSES):
        aff = (zone >= 0) & (zone % 2 == 0) if s_ == 3 else np.ones(n, bool)
        elig |= np.where(aff & has(hard), 1 << (2 * s_), 0).astype(np.uint16)
        elig |= np.where(aff & has(soft), 1 << (2 * s_ + 1), 0).astype(np.uint16)
    t["pts_elig"][:] = elig
    m = len(ext)
    sp = spec.seed + 17
    on = uniform(sp, m, 1) < spec.pod_frac
    app = (splitmix64(sp, m, 2) % np.uint64(3)).astype(np.int64)
    cls = (splitmix64(sp, m, 3) % np.uint64(len(SPREAD_CLASSES))).astype(np.int64)
    cls = np.where(app == 2, np.where(cls % 2 == 0, 0, 3), cls)   # app 2 has no hostname constraint
    for j in np.flatnonzero(on):
        a, s_ = int(app[j]), int(cls[j])
        x = ext[j]
        items = SPREAD_CLASSES[s_][2]
        x["pts_n"] = len(items)
        x["pts_class"] = s_
        x["pts_match"] = sum(1 << c for c, (ca, _) in enumerate(SPREAD_CONS) if ca == a)
        for q, (k, hard, skew) in enumerate(items):
            x["pts_c"][q] = SPREAD_CONS.index((a, k))
            x["pts_fl"][q] = (abi.PTS_HARD if hard else 0) | abi.PTS_SELF
            x["pts_skew"][q] = skew
    return t


# Benchmark / parity configurations (BASELINE.json "configs")
CONFIGS = {
    1: dict(nodes=500, pods=1000, be_frac=0.0),
    2: dict(nodes=5000, pods=10000, be_frac=0.0),
    3: dict(nodes=5000, pods=10000, be_frac=0.2, cpuset_frac=0.5, numa=True),
    4: dict(nodes=50000, pods=100000, be_frac=0.3),
    5: dict(nodes=200000, pods=100000, be_frac=0.3, numa=True, reservation=True, resv_match_frac=0.2),
}


def config_workload(cfg_id: int, profile: Profile, n_nodes: int = None, n_pods: int = None) -> Tuple[NodeTable, np.ndarray]:
    c = CONFIGS[cfg_id]
    table = make_cluster(ClusterSpec(n_nodes or c["nodes"]), profile)
    if c.get("numa"):
        add_numa(table, NumaSpec(), profile)
    if c.get("reservation"):
        add_reservations(table, ResvSpec())
    pods = make_pods(StreamSpec(n_pods or c["pods"], be_frac=c["be_frac"], cpuset_frac=c.get("cpuset_frac", 0.0),
                                resv_match_frac=c.get("resv_match_frac", 0.0)), profile)
    return table, pods


@dataclass
class IpaSpec:
    """InterPodAffinity: zone / hostname topology (the PodTopologySpread keys
    when the table has them), four apps with running pods, and pending pods of
    those apps with the common term shapes -- app 0 spreads one pod per host
    (required anti-affinity to itself), app 1 prefers zones running app 2
    (weight 50), app 2 needs a zone running app 3 (required affinity; the
    running app 2 pods carry it, so app 3 pods score hardPodAffinityWeight 1
    there), app 3 avoids its own hosts (preferred anti-affinity, weight 30,
    which its running pods carry too)."""
    zones: int = 6
    no_zone_frac: float = 0.03
    running_frac: float = 0.3     # nodes holding running pods of an app
    pod_frac: float = 0.6         # pending pods of one of the apps
    seed: int = SEED


# the count entries: (kind, app, key) with key 0 zone, 1 hostname
IPA_ENTRIES = [("M", 0, 0), ("M", 0, 1), ("M", 1, 0), ("M", 1, 1), ("M", 2, 0), ("M", 2, 1), ("M", 3, 0), ("M", 3, 1),
               ("C-anti", 0, 1), ("C-pref", 3, 1), ("C-aff", 2, 0)]


def add_ipa(t: NodeTable, ext: np.ndarray, spec: IpaSpec) -> NodeTable:
    """The ipa_* column and the pods' ipa_* fields (hand-encoded tables of the
    shapes IpaSpec describes; test_ipa_objects.py checks the object path)."""
    from .snapshot import IpaMeta, PtsMeta
    n, sd = t.n, spec.seed + 23
    if t.has_pts:   # the spread workload's keys: zone 0, hostname = the hostname bit
        zk, hk = 0, int(t.pts.hostname).bit_length() - 1
    else:
        t.enable_pts(PtsMeta(keys=2, hostname=0b10, ndom=[spec.zones, 0, 0, 0], cons_key=[], classes=0))
        zone = (splitmix64(sd, n, 1) % np.uint64(spec.zones)).astype(np.int32)
        zone[uniform(sd, n, 3) < spec.no_zone_frac] = -1
        t["pts_dom"][:, 0] = zone
        t["pts_dom"][:, 1] = np.arange(n, dtype=np.int32)
        zk, hk = 0, 1
    key = {0: zk, 1: hk}
    t.enable_ipa(IpaMeta(ent_key=[key[k] for _, _, k in IPA_ENTRIES]))
    running = np.zeros((n, 4), np.int32)
    for a in range(4):
        on = uniform(sd, n, 10 + a) < spec.running_frac
        running[:, a] = np.where(on, (splitmix64(sd, n, 20 + a) % np.uint64(3)).astype(np.int32) + 1, 0)
    cnt = t["ipa_cnt"]
    for e, (kind, a, _) in enumerate(IPA_ENTRIES):
        cnt[:, e] = running[:, a]       # M: the app's pods; C: the app's pods carry the term
    m = len(ext)
    sp = spec.seed + 29
    on = uniform(sp, m, 1) < spec.pod_frac
    app = (splitmix64(sp, m, 2) % np.uint64(4)).astype(np.int64)
    for j in np.flatnonzero(on):
        x = ext[j]
        a = int(app[j])
        x["ipa_inc"] = (1 << (2 * a)) | (1 << (2 * a + 1))
        if a == 0:
            x["ipa_inc"] |= 1 << 8
            x["ipa_anti"] = (1 << 1) | (1 << 8)
        elif a == 1:
            x["ipa_w"][4] = 50
        elif a == 2:
            x["ipa_inc"] |= 1 << 10
            x["ipa_aff"] = 1 << 6
        else:
            x["ipa_inc"] |= 1 << 9
            x["ipa_w"][7] = -30
            x["ipa_w"][9] = -30
            x["ipa_w"][10] = 1
        x["ipa_score"] = sum(1 << e for e in range(abi.IPA_ENTRIES) if x["ipa_w"][e] != 0)
    return t
