"""The event-driven marshaller (koordinator_amd/informer.py): podAssignCache
semantics pinned by the reference's pod_assign_cache_test.go tables, and
randomized event streams whose incremental row deltas equal a from-scratch
build_table of the same ClusterState after every flush."""
import copy

import numpy as np
import pytest

from koordinator_amd import k8s
from koordinator_amd.config import shipped_profile
from koordinator_amd.informer import Informer, PodAssignCache
from koordinator_amd.marshal import build_table
from koordinator_amd.snapshot import ALL_COLS

NOW = 1_000_000.0


def _pod(uid="123456789", node="test-node", phase="Running", ns="default", name="test"):
    return k8s.Pod(namespace=ns, name=name, uid=uid, node_name=node, phase=phase)


def _cache(c: PodAssignCache):
    return {n: sorted(m) for n, m in c.items.items()}


# pod_assign_cache_test.go:35-107 TestPodAssignCache_OnAdd
@pytest.mark.parametrize("pod,want", [
    (k8s.Pod(), {}),                                               # update pending pod (:42-45)
    (_pod(uid="", phase="Failed"), {}),                            # update terminated pod (:46-57)
    (_pod(), {"test-node": ["123456789"]}),                        # update scheduled running pod (:58-93)
], ids=["pending", "terminated", "running"])
def test_assign_cache_on_add(pod, want):
    c = PodAssignCache()
    c.on_add(pod, NOW)
    assert _cache(c) == want
    for n, m in c.items.items():
        assert all(info.timestamp == NOW for info in m.values())


# pod_assign_cache_test.go:109-212 TestPodAssignCache_OnUpdate
@pytest.mark.parametrize("start,pod,want", [
    (None, k8s.Pod(), {}),                                          # update pending pod (:116-120)
    ({"test-node": [_pod()]}, _pod(phase="Failed"), {}),            # update terminated pod (:121-159)
    (None, _pod(), {"test-node": ["123456789"]}),                   # update scheduled running pod (:160-195)
], ids=["pending", "terminated", "running"])
def test_assign_cache_on_update(start, pod, want):
    c = PodAssignCache()
    for n, pods in (start or {}).items():
        for p in pods:
            c.assign(n, p, NOW)
    c.on_update(None, pod, NOW)
    assert _cache(c) == want


def test_assign_cache_on_delete():
    """pod_assign_cache_test.go:214-250: deleting the node's last pod drops the node."""
    c = PodAssignCache()
    c.assign("test-node", _pod(), NOW)
    c.on_delete(_pod(phase="Failed"))
    assert _cache(c) == {}


# ------------------------------------------------------------------ random event streams
GI = 1 << 30


def _rand_pod(rng, i, nodes):
    prio = [None, 9500, 5500, 3500][rng.integers(0, 4)]
    cpu = int(rng.choice([100, 250, 500, 1000, 2000]))
    mem = int(rng.choice([128, 256, 1024, 2048])) << 20
    req = {k8s.CPU: k8s.Q(f"{cpu}m"), k8s.MEMORY: k8s.Q(mem)}
    if prio == 5500:  # batch resources
        req = {k8s.BATCH_CPU: k8s.Q(cpu), k8s.BATCH_MEMORY: k8s.Q(mem)}
    node = nodes[rng.integers(0, len(nodes))].name if rng.random() < 0.8 else ""
    return k8s.Pod(namespace="ns", name=f"p{i}", uid=f"u{i}", priority=prio, node_name=node,
                   containers=[k8s.Container(requests=req, limits=dict(req))])


def _rand_metric(rng, node, pods, now):
    on = [p for p in pods if p.node_name == node.name]
    pm = [k8s.PodMetric(p.namespace, p.name, {k8s.CPU: k8s.Q(f"{int(rng.integers(10, 900))}m"),
                                               k8s.MEMORY: k8s.Q(int(rng.integers(1, 500)) << 20)})
          for p in on if rng.random() < 0.7]
    return k8s.NodeMetric(name=node.name, update_time=now - float(rng.integers(0, 400)), report_interval_s=60,
                          node_usage={k8s.CPU: k8s.Q(f"{int(rng.integers(0, 30000))}m"),
                                      k8s.MEMORY: k8s.Q(int(rng.integers(0, 60)) * GI)},
                          pods_metric=pm)


class _TableEngine:
    """Stands in for the device: applies update_nodes rows to a NodeTable."""

    def __init__(self, table):
        self.table = table.copy()

    def update_nodes(self, idx, rows):
        for c in ALL_COLS:
            self.table.cols[c][idx] = rows.cols[c]


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_incremental_rows_equal_rebuild(seed):
    rng = np.random.default_rng(seed)
    prof = shipped_profile()
    nodes = [k8s.Node(name=f"n{i}", allocatable={k8s.CPU: k8s.Q(32), k8s.MEMORY: k8s.Q(64 * GI), k8s.PODS: k8s.Q(110),
                                                 k8s.BATCH_CPU: k8s.Q(20000), k8s.BATCH_MEMORY: k8s.Q(40 * GI)})
             for i in range(12)]
    inf = Informer(prof, nodes, NOW)
    pods = [_rand_pod(rng, i, nodes) for i in range(40)]
    now = NOW
    for p in pods:
        inf.on_pod_add(p, now)
    for n in nodes:
        if rng.random() < 0.8:
            inf.on_node_metric(_rand_metric(rng, n, pods, now))
    eng = _TableEngine(inf.table(now))
    live = {p.uid: p for p in pods}
    nxt = len(pods)
    for step in range(25):
        now += float(rng.integers(1, 120))
        for _ in range(int(rng.integers(1, 8))):
            op = rng.random()
            if op < 0.3:                                   # new pod (pending or bound)
                p = _rand_pod(rng, nxt, nodes)
                nxt += 1
                live[p.uid] = p
                inf.on_pod_add(p, now)
            elif op < 0.5 and live:                        # bind / move / finish a pod
                p = copy.deepcopy(live[list(live)[int(rng.integers(0, len(live)))]])
                r = rng.random()
                if r < 0.4:
                    p.node_name = nodes[int(rng.integers(0, len(nodes)))].name
                elif r < 0.7:
                    p.phase = "Succeeded"
                else:
                    p.labels = {"x": str(step)}
                live[p.uid] = p
                inf.on_pod_update(None, p, now)
            elif op < 0.65 and live:                       # delete a pod
                p = live.pop(list(live)[int(rng.integers(0, len(live)))])
                inf.on_pod_delete(p)
            elif op < 0.85:                                # NodeMetric report
                n = nodes[int(rng.integers(0, len(nodes)))]
                inf.on_node_metric(_rand_metric(rng, n, list(live.values()), now))
            elif op < 0.92:                                # NodeMetric gone
                inf.on_node_metric_delete(nodes[int(rng.integers(0, len(nodes)))].name)
            else:                                          # node allocatable change
                i = int(rng.integers(0, len(nodes)))
                n = copy.deepcopy(nodes[i])
                n.allocatable[k8s.CPU] = k8s.Q(int(rng.choice([16, 32, 48])))
                nodes[i] = n
                inf.on_node_update(None, n)
        res = inf.flush(eng, now)
        assert not res.needs_reload
        want = build_table(inf.cluster, prof, now)
        for c in ALL_COLS:
            assert np.array_equal(eng.table.cols[c], want.cols[c]), (step, c)


def test_node_set_change_needs_reload():
    prof = shipped_profile()
    nodes = [k8s.Node(name=f"n{i}", allocatable={k8s.CPU: k8s.Q(8), k8s.MEMORY: k8s.Q(GI), k8s.PODS: k8s.Q(10)})
             for i in range(3)]
    inf = Informer(prof, nodes, NOW)
    inf.table(NOW)
    inf.on_node_add(k8s.Node(name="n3", allocatable={k8s.CPU: k8s.Q(8)}))
    assert inf.flush(_TableEngine(inf.table(NOW)), NOW).needs_reload is False  # table() rebuilt it
    inf.on_node_delete(nodes[0])
    assert inf.delta(NOW)[2].needs_reload
    t = inf.table(NOW)
    assert t.names == ["n1", "n2", "n3"]


@pytest.mark.gpu
def test_gpu_informer_deltas_then_stream():
    """Informer deltas through koordhip_update_nodes, then a greedy stream: the
    device state and placements equal a fresh snapshot of the same objects."""
    import torch  # noqa: F401
    import oracle
    from koordinator_amd.config import to_c_config
    from koordinator_amd.engine import PlacementEngine
    from koordinator_amd import synth
    rng = np.random.default_rng(9)
    prof = shipped_profile()
    nodes = [k8s.Node(name=f"n{i}", allocatable={k8s.CPU: k8s.Q(32), k8s.MEMORY: k8s.Q(64 * GI), k8s.PODS: k8s.Q(110),
                                                 k8s.BATCH_CPU: k8s.Q(20000), k8s.BATCH_MEMORY: k8s.Q(40 * GI)})
             for i in range(200)]
    inf = Informer(prof, nodes, NOW)
    pods = [_rand_pod(rng, i, nodes) for i in range(600)]
    for p in pods:
        inf.on_pod_add(p, NOW)
    for n in nodes:
        inf.on_node_metric(_rand_metric(rng, n, pods, NOW))
    stream = synth.make_pods(synth.StreamSpec(400, be_frac=0.3), prof)
    with PlacementEngine(prof, device=0) as e:
        e.load_snapshot(inf.table(NOW))
        now = NOW + 30
        for p in pods[::7]:
            q = copy.deepcopy(p)
            q.phase = "Succeeded"
            inf.on_pod_update(None, q, now)
        for n in nodes[::5]:
            inf.on_node_metric(_rand_metric(rng, n, pods, now))
        res = inf.flush(e, now)
        assert res.rows > 0 and not res.needs_reload
        got = e.place_stream(stream)
        st = e.read_nodes()
    fresh = build_table(inf.cluster, prof, now)
    o = oracle.Oracle(to_c_config(prof), fresh)
    ref = o.place_stream(stream)
    assert np.array_equal(got, ref)
    rs = o.state()
    for k in ("requested", "npods", "la_used"):
        assert np.array_equal(st[k], rs[k]), k


def _rand_resv(rng, i, nodes):
    from koordinator_amd import reservation as rv
    cpu = int(rng.choice([1000, 2000, 4000]))
    mem = int(rng.choice([1, 2, 4])) * GI
    order = str(int(rng.choice([1, 2, 3]))) if rng.random() < 0.3 else None
    return rv.Reservation(
        name=f"r{i}", node_name=nodes[int(rng.integers(0, len(nodes)))].name, uid=f"ru{i}",
        labels={rv.LABEL_RESERVATION_ORDER: order} if order else {},
        owners=[rv.ReservationOwner(label_selector=rv.LabelSelector(match_labels={"app": f"a{int(rng.integers(0, 3))}"}))],
        allocatable={k8s.CPU: k8s.Q(f"{cpu}m"), k8s.MEMORY: k8s.Q(mem)},
        allocated={k8s.CPU: k8s.Q(f"{int(rng.integers(0, 2)) * 500}m")}, assigned=int(rng.integers(0, 2)),
        allocate_once=bool(rng.random() < 0.5))


@pytest.mark.parametrize("seed", [4, 5])
def test_reservation_events_rows_equal_rebuild(seed):
    """Reservation add / update / delete events (reservation/cache.go:117-252):
    the incremental resv_* rows equal reservation_columns over the same
    reservations, and a reload keeps the owner groups and the NUMA columns."""
    from koordinator_amd import reservation as rv
    rng = np.random.default_rng(seed)
    prof = shipped_profile(numa=True, reservation=True)
    nodes = [k8s.Node(name=f"n{i}", allocatable={k8s.CPU: k8s.Q(32), k8s.MEMORY: k8s.Q(64 * GI), k8s.PODS: k8s.Q(110)})
             for i in range(16)]
    inf = Informer(prof, nodes, NOW)
    live = {}
    for i in range(5):   # distinct nodes to start with (at most one Available reservation per node)
        r = _rand_resv(rng, i, nodes)
        r.node_name = nodes[i].name
        r.labels = {rv.LABEL_RESERVATION_ORDER: str(1 + i % 3)}
        live[r.name] = r
        inf.on_reservation(r)
    eng = _TableEngine(inf.table(NOW))
    nxt = 5
    for step in range(30):
        op = rng.random()
        if op < 0.4:
            r = _rand_resv(rng, nxt, nodes)
            nxt += 1
        elif op < 0.75 and live:
            r = copy.deepcopy(live[list(live)[int(rng.integers(0, len(live)))]])
            r.allocated = {k8s.CPU: k8s.Q(f"{int(rng.integers(0, 4)) * 250}m")}
            r.assigned = int(rng.integers(0, 3))
            if rng.random() < 0.3:
                r.node_name = nodes[int(rng.integers(0, len(nodes)))].name
            if rng.random() < 0.2:
                r.phase = "Succeeded"
        else:
            if live:
                inf.on_reservation_delete(live.pop(list(live)[int(rng.integers(0, len(live)))]).name)
            r = None
        if r is not None:
            busy = {x.node_name for x in live.values() if x.name != r.name and x.is_available()}
            if r.is_available() and r.node_name in busy:
                continue                                  # a second Available reservation on a node: unsupported
            live[r.name] = r
            inf.on_reservation(r)
        res = inf.flush(eng, NOW)
        if res.needs_reload:                              # a reservation order the snapshot has no rank for
            eng = _TableEngine(inf.table(NOW))
        want = build_table(inf.cluster, prof, NOW)
        rv.reservation_columns(want, {n.name: i for i, n in enumerate(nodes)}, list(live.values()),
                               rv.ReservationIndex(groups=list(inf.resv_index.groups),
                                                   group_of=dict(inf.resv_index.group_of)))
        for c in ("resv_flags", "resv_alloc0", "resv_alloc1", "resv_nz0", "resv_nz1", "resv_allocated0",
                  "resv_allocated1", "resv_assigned"):
            assert np.array_equal(eng.table.cols[c], want.cols[c]), (step, c)
        # order ranks: the same relative order of the order labels
        ordered = (want.cols["resv_flags"] & 8) != 0
        assert np.array_equal((eng.table.cols["resv_flags"] & 8) != 0, ordered)
        a, b = eng.table.cols["resv_order_rank"][ordered], want.cols["resv_order_rank"][ordered]
        assert np.array_equal(np.argsort(a, kind="stable"), np.argsort(b, kind="stable"))


def test_reload_keeps_reservations_and_numa_by_name():
    """a node add / delete reload must keep every reservation (and
    the NUMA columns) of the nodes that stay."""
    from koordinator_amd import reservation as rv
    prof = shipped_profile(numa=True, reservation=True)
    nodes = [k8s.Node(name=f"n{i}", allocatable={k8s.CPU: k8s.Q(16), k8s.MEMORY: k8s.Q(32 * GI), k8s.PODS: k8s.Q(110)})
             for i in range(4)]
    inf = Informer(prof, nodes, NOW)
    inf.on_reservation(rv.Reservation(name="r", node_name="n2", owners=[rv.ReservationOwner(
        label_selector=rv.LabelSelector(match_labels={"app": "x"}))], allocatable={k8s.CPU: k8s.Q(2), k8s.MEMORY: k8s.Q(GI)}))
    t = inf.table(NOW)
    t.cols["numa_class"][2] = 7                            # stands for NUMA columns loaded from an NRT
    inf.on_node_delete(nodes[0])
    t2 = inf.table(NOW)
    assert t2.names == ["n1", "n2", "n3"]
    assert t2.cols["resv_flags"][1] & 1 and t2.cols["resv_alloc0"][1] == 2000
    assert t2.cols["resv_flags"][0] == 0 and t2.cols["resv_flags"][2] == 0
    assert t2.cols["numa_class"][1] == 7


# ------------------------------------------------ NodeResourceTopology + NUMA pod events
def _nrt(rng, name, sockets=2, nps=1, cores=8, policy=None):
    import json as _j
    from koordinator_amd import numa as nm
    topo = nm.linux_topology(sockets, nps, cores, 2)
    detail = [{"id": c, "core": topo.details[c].core & 0xFFFF, "socket": topo.details[c].socket,
               "node": topo.details[c].node} for c in topo.cpu_of]
    ann = {nm.ANNOTATION_CPU_TOPOLOGY: _j.dumps({"detail": detail})}
    if rng.random() < 0.5:
        ann[nm.ANNOTATION_KUBELET_CPU_MANAGER_POLICY] = _j.dumps({"policy": "static", "reservedCPUs": "0-1"})
    nn = sockets * nps
    zones = [nm.Zone(f"node-{k}", resources={"cpu": cores * 2 * 1000, "memory": 16 * GI}) for k in range(nn)]
    return nm.NodeResourceTopology(name=name, annotations=ann, zones=zones,
                                   topology_policies=[policy] if policy else ["None"])


def _numa_pod(rng, i, node, topo_cpus):
    import json as _j
    from koordinator_amd import numa as nm
    k = int(rng.integers(1, 5)) * 2
    start = int(rng.integers(0, max(1, len(topo_cpus) - k)))
    cpus = topo_cpus[start:start + k]
    status = {"cpuset": nm.format_cpuset(cpus),
              "numaNodeResources": [{"node": int(rng.integers(0, 2)), "resources": {"cpu": k * 1000, "memory": GI}}]}
    spec = {"preferredCPUBindPolicy": "FullPCPUs",
            "preferredCPUExclusivePolicy": str(rng.choice(["", "PCPULevel", "NUMANodeLevel"]))}
    return k8s.Pod(namespace="ns", name=f"np{i}", uid=f"nu{i}", node_name=node, priority=9500,
                   annotations={nm.ANNOTATION_RESOURCE_STATUS: _j.dumps(status), nm.ANNOTATION_RESOURCE_SPEC: _j.dumps(spec)},
                   containers=[k8s.Container(requests={k8s.CPU: k8s.Q(k), k8s.MEMORY: k8s.Q(GI)})])


NUMA_COLS = ([f"numa_free{w}" for w in range(4)] + [f"numa_excl_pcpu{w}" for w in range(4)]
             + [f"numa_excl_numa{w}" for w in range(4)] + ["numa_alloc_cnt", "numa_class", "numa_flags",
                                                         "numa_zone_alloc", "numa_zone_used", "numa_amp_cpu"])


@pytest.mark.parametrize("seed", [6, 7, 8])
def test_numa_events_rows_equal_rebuild(seed):
    """NRT add / update / delete and NUMA pod bind / finish / delete events
    (topology_eventhandler.go:62-113, pod_eventhandler.go:94-144): after every
    flush the device-row image equals a from-scratch table() of the same state."""
    from koordinator_amd import numa as nm
    rng = np.random.default_rng(seed)
    prof = shipped_profile(numa=True)
    nodes = [k8s.Node(name=f"n{i}", allocatable={k8s.CPU: k8s.Q(32), k8s.MEMORY: k8s.Q(64 * GI), k8s.PODS: k8s.Q(110)},
                      labels={nm.LABEL_NUMA_TOPOLOGY_POLICY: "BestEffort"} if i % 5 == 0 else {})
             for i in range(10)]
    inf = Informer(prof, nodes, NOW)
    shapes = [(2, 1, 8), (2, 2, 4)]
    for i, n in enumerate(nodes[:8]):
        inf.on_nrt(_nrt(rng, n.name, *shapes[i % 2], policy=["Restricted", None][i % 2]))
    eng = _TableEngine(inf.table(NOW))
    live, nxt = {}, 0
    cpus_of = {n: list(range(32)) for n in (x.name for x in nodes)}
    for step in range(40):
        op = rng.random()
        if op < 0.45:
            n = nodes[int(rng.integers(0, len(nodes)))].name
            p = _numa_pod(rng, nxt, n, cpus_of[n])
            nxt += 1
            live[p.uid] = p
            inf.on_pod_add(p, NOW)
        elif op < 0.6 and live:
            p = copy.deepcopy(live[list(live)[int(rng.integers(0, len(live)))]])
            p.phase = "Succeeded"
            live.pop(p.uid)
            inf.on_pod_update(None, p, NOW)
        elif op < 0.75 and live:
            inf.on_pod_delete(live.pop(list(live)[int(rng.integers(0, len(live)))]))
        elif op < 0.9:
            i = int(rng.integers(0, len(nodes)))
            inf.on_nrt(_nrt(rng, nodes[i].name, *shapes[int(rng.integers(0, 2))],
                            policy=[None, "BestEffort", "SingleNUMANodePodLevel"][int(rng.integers(0, 3))]))
        else:
            inf.on_nrt_delete(nodes[int(rng.integers(0, len(nodes)))].name)
        res = inf.flush(eng, NOW)
        if res.needs_reload:
            eng = _TableEngine(inf.table(NOW))
        classes = inf._classes
        want = inf.table(NOW)
        # the rebuild may number classes differently: compare the class records
        for c in NUMA_COLS:
            if c == "numa_class":
                a, b = eng.table.cols[c], want.cols[c]
                assert np.array_equal(a < 0, b < 0), step
                ra = [classes.records()[x].tobytes() for x in a[a >= 0]]
                rb = [want.numa_classes[x].tobytes() for x in b[b >= 0]]
                assert ra == rb, step
            else:
                assert np.array_equal(eng.table.cols[c], want.cols[c]), (step, c)
        eng = _TableEngine(want)
        inf.attach(want, NOW)
    assert inf._alloc and any(a.cpus for a in inf._alloc.values())


def test_numa_pod_before_its_nrt_is_dropped():
    """resourceManager.Update (resource_manager.go:328-339) ignores an allocation
    while the node has no CPU topology: the event order matters."""
    from koordinator_amd import numa as nm
    rng = np.random.default_rng(1)
    prof = shipped_profile(numa=True)
    nodes = [k8s.Node(name="n0", allocatable={k8s.CPU: k8s.Q(32), k8s.MEMORY: k8s.Q(64 * GI), k8s.PODS: k8s.Q(110)})]
    inf = Informer(prof, nodes, NOW)
    inf.on_pod_add(_numa_pod(rng, 0, "n0", list(range(32))), NOW)
    inf.on_nrt(_nrt(rng, "n0"))
    t = inf.table(NOW)
    assert t["numa_class"][0] == 0 and t["numa_alloc_cnt"][0] == 0
    inf.on_pod_add(_numa_pod(rng, 1, "n0", list(range(32))), NOW)
    assert inf.table(NOW)["numa_alloc_cnt"][0] > 0


@pytest.mark.gpu
def test_gpu_numa_events_then_stream():
    """§8(f)#2: a burst of NRT and NUMA pod events pushed through
    koordhip_update_nodes, then a greedy stream with cpuset pods: placements,
    cpusets and the NUMA state equal the oracle's on a fresh snapshot."""
    import torch  # noqa: F401
    import oracle
    from koordinator_amd import numa as nm, synth
    from koordinator_amd.config import to_c_config
    from koordinator_amd.engine import PlacementEngine
    rng = np.random.default_rng(12)
    prof = shipped_profile(numa=True)
    nodes = [k8s.Node(name=f"n{i}", allocatable={k8s.CPU: k8s.Q(32), k8s.MEMORY: k8s.Q(64 * GI), k8s.PODS: k8s.Q(110)})
             for i in range(120)]
    inf = Informer(prof, nodes, NOW)
    for i, n in enumerate(nodes):
        if i % 10:
            inf.on_nrt(_nrt(rng, n.name, *[(2, 1, 8), (2, 2, 4)][i % 2], policy=[None, "BestEffort", "Restricted"][i % 3]))
    for j in range(150):
        n = nodes[int(rng.integers(0, len(nodes)))].name
        inf.on_pod_add(_numa_pod(rng, j, n, list(range(32))), NOW)
    stream = synth.make_pods(synth.StreamSpec(300, be_frac=0.2, cpuset_frac=0.5), prof)
    with PlacementEngine(prof, device=0) as e:
        e.load_snapshot(inf.table(NOW))
        for j in range(150, 230):                  # the burst: new NUMA pods, finished pods, NRT updates
            n = nodes[int(rng.integers(0, len(nodes)))].name
            inf.on_pod_add(_numa_pod(rng, j, n, list(range(32))), NOW)
        for j in range(0, 150, 4):
            p = copy.deepcopy(inf._pods_by_uid[f"nu{j}"])
            p.phase = "Succeeded"
            inf.on_pod_update(None, p, NOW)
        for i in range(1, 120, 7):
            inf.on_nrt(_nrt(rng, nodes[i].name, *[(2, 1, 8), (2, 2, 4)][i % 2], policy="SingleNUMANodePodLevel"))
        res = inf.flush(e, NOW)
        assert res.rows > 0 and not res.needs_reload
        got = e.place_stream(stream)
        cs = e.fetch_cpusets(len(stream))
        nst = e.read_numa()
    fresh = inf.table(NOW)
    o = oracle.Oracle(to_c_config(prof), fresh)
    ref, rcs = o.place_stream(stream, cpusets=True)
    assert np.array_equal(got, ref), int(np.flatnonzero(got != ref)[0])
    assert np.array_equal(cs, rcs)
    for k, v in o.numa_state().items():
        assert np.array_equal(nst[k], v), k


def test_reservation_cpuset_events_rows_equal_rebuild():
    """A reservation holding a cpuset: its reserve pod's CPUs are a NodeAllocation
    entry (ReservationToPodEventHandler, nodenumaresource/pod_eventhandler.go:
    40-50), its reserved CPUs (less the assigned pods', reservation.go:84-104)
    the slot's resv_cpus; deleting it frees them.  Each flush equals a rebuild."""
    from koordinator_amd import numa as nm
    from koordinator_amd import reservation as rv
    rng = np.random.default_rng(3)
    prof = shipped_profile(numa=True, reservation=True)
    nodes = [k8s.Node(name=f"n{i}", allocatable={k8s.CPU: k8s.Q(32), k8s.MEMORY: k8s.Q(64 * GI), k8s.PODS: k8s.Q(110)})
             for i in range(3)]
    inf = Informer(prof, nodes, NOW)
    for n in nodes:
        inf.on_nrt(_nrt(rng, n.name))
    t0 = inf.table(NOW)
    cnt0 = int(t0["numa_alloc_cnt"][1])
    eng = _TableEngine(t0)
    r = rv.Reservation("r0", "n1", uid="ru0", allocatable={k8s.CPU: k8s.Q(4)}, owners=[rv.ReservationOwner()],
                       cpus=[4, 5, 6, 7], assigned_cpus=[4, 5])
    inf.on_reservation(r)
    # the snapshot was loaded without resv_cpus columns -> a reload,
    # not rows the engine would refuse (the image keeps its rows, still dirty)
    before = {c: eng.table.cols[c].copy() for c in NUMA_COLS[:13]}
    assert inf.flush(eng, NOW).needs_reload
    assert all(np.array_equal(eng.table.cols[c], before[c]) for c in before)
    assert inf.pending() == {"n1"}
    want = inf.table(NOW)
    eng = _TableEngine(want)
    inf.attach(want, NOW)
    r2 = copy.deepcopy(r)
    r2.assigned_cpus = [4]
    inf.on_reservation(r2)                     # now the columns exist: a plain row delta
    res = inf.flush(eng, NOW)
    assert not res.needs_reload and res.rows == 1
    want = inf.table(NOW)
    for c in NUMA_COLS[:13] + [f"resv_cpus{w}" for w in range(4)]:
        assert np.array_equal(eng.table.cols[c], want.cols[c]), c
    inf.on_reservation(r)
    assert not inf.flush(eng, NOW).needs_reload
    want = inf.table(NOW)
    topo = nm.linux_topology(2, 1, 8, 2)
    held = topo.mask([4, 5, 6, 7])
    assert not any(int(want[f"numa_free{w}"][1]) & int(held[w]) for w in range(4))
    assert [int(want[f"resv_cpus{w}"][1]) for w in range(4)] == [int(x) for x in topo.mask([6, 7])]
    inf.attach(want, NOW)
    eng = _TableEngine(want)
    inf.on_reservation_delete("r0")
    inf.flush(eng, NOW)
    assert int(eng.table["numa_alloc_cnt"][1]) == cnt0
    assert not any(int(eng.table[f"resv_cpus{w}"][1]) for w in range(4))


def test_reserve_pod_through_the_informer():
    """A pending Reservation is scheduled as its reserve pod (NewReservePod):
    the informer's pod records mark it (KOORDHIP_POD_RESERVE, its allocate
    policy, no reservation match) and its ext record pins its node; the oracle
    places it only on that node and no later pod of the batch matches it (it is
    not Available yet).  Once the Reservation is Available on that node, a
    reload's owner groups let a matching pod nominate it."""
    import oracle
    from koordinator_amd import abi
    from koordinator_amd import reservation as rv
    from koordinator_amd.config import to_c_config
    prof = shipped_profile(reservation=True)
    nodes = [k8s.Node(name=f"n{i}", allocatable={k8s.CPU: k8s.Q(32), k8s.MEMORY: k8s.Q(64 * GI), k8s.PODS: k8s.Q(110)})
             for i in range(8)]
    inf = Informer(prof, nodes, NOW)
    owner = rv.ReservationOwner(label_selector=rv.LabelSelector(match_labels={"app": "web"}))
    r = rv.Reservation("r-web", phase="Pending", owners=[owner], spec_node_name="n5",
                       allocatable={k8s.CPU: k8s.Q(4), k8s.MEMORY: k8s.Q(8 * GI)},
                       allocate_policy=rv.POLICY_ALIGNED)
    inf.on_reservation(r)
    t = inf.table(NOW)
    rp = rv.new_reserve_pod(r)
    web = k8s.Pod(name="web-0", labels={"app": "web"},
                  containers=[k8s.Container(requests={k8s.CPU: k8s.Q(1), k8s.MEMORY: k8s.Q(GI)})])
    recs = inf.pod_records([rp, web])
    ext = inf.pod_ext_records([rp, web])
    assert recs["flags"][0] & abi.POD_RESERVE and recs["resv_match"][0] == 0
    assert ext["reserve_node"][0] == 6 and ext["reserve_node"][1] == 0
    o = oracle.Oracle(to_c_config(prof), t)
    got = o.place_stream_ext(recs, ext)
    assert got[0] == 5
    assert o.resv_state()["assigned"].sum() == 0          # nothing matched the pending reservation
    # the reservation is Available on n5 now: after a reload the web pod matches it
    r2 = copy.deepcopy(r)
    r2.phase, r2.node_name = "Available", "n5"
    inf.on_reservation(r2)
    t2 = inf.table(NOW)
    recs2 = inf.pod_records([web])
    assert recs2["resv_match"][0] != 0
    o2 = oracle.Oracle(to_c_config(prof), t2)
    assert o2.place_stream(recs2)[0] == 5                 # the reservation's node wins (weight 5000)


def test_operating_mode_pod_is_a_reservation():
    """A bound pod in the reservation operating mode is also an Available
    reservation on its node (pod_eventhandler.go:104-124, cache.go:139-168,
    NewReservationInfoFromPod): its requests are the slot's Allocatable, its
    reservation-owners annotation the owners, AllocateOnce and Aligned always;
    Ready gates it, a current owner takes it out of matching, deleting the pod
    removes the slot.  A matching pod nominates it and fits through the
    restore where a non-matching one does not (oracle)."""
    import json as _json
    import oracle
    from koordinator_amd import abi
    from koordinator_amd import reservation as rv
    from koordinator_amd.config import to_c_config
    prof = shipped_profile(reservation=True)
    nodes = [k8s.Node(name=f"n{i}", allocatable={k8s.CPU: k8s.Q(8), k8s.MEMORY: k8s.Q(16 * GI), k8s.PODS: k8s.Q(110)})
             for i in range(4)]
    inf = Informer(prof, nodes, NOW)
    # every node but n2 is full; n2 holds the operating pod (6 cpu / 12 Gi) and a 1-cpu pod
    for i in (0, 1, 3):
        inf.on_pod_add(k8s.Pod(name=f"filler-{i}", uid=f"f{i}", node_name=f"n{i}", containers=[
            k8s.Container(requests={k8s.CPU: k8s.Q(8), k8s.MEMORY: k8s.Q(16 * GI)})]), NOW)
    owners = [{"labelSelector": {"matchLabels": {"app": "web"}}}]
    op = k8s.Pod(name="op-0", uid="op0", node_name="n2",
                 labels={rv.LABEL_POD_OPERATING_MODE: "Reservation"},
                 annotations={rv.ANNOTATION_RESERVATION_OWNERS: _json.dumps(owners)},
                 containers=[k8s.Container(requests={k8s.CPU: k8s.Q(6), k8s.MEMORY: k8s.Q(12 * GI)})])
    inf.on_pod_add(op, NOW)
    inf.on_pod_add(k8s.Pod(name="other", uid="o1", node_name="n2", containers=[
        k8s.Container(requests={k8s.CPU: k8s.Q(1), k8s.MEMORY: k8s.Q(GI)})]), NOW)
    t = inf.table(NOW)
    f = int(t["resv_flags"][2])
    assert f & abi.RESV_PRESENT and f & abi.RESV_ALLOCATE_ONCE
    assert (f >> abi.RESV_POLICY_SHIFT) & 3 == abi.RESV_POLICY_ALIGNED
    assert int(t["resv_alloc0"][2]) == 6000 and int(t["resv_alloc1"][2]) == 12 * GI
    assert int(t["resv_assigned"][2]) == 0 and not any(int(t["resv_flags"][i]) for i in (0, 1, 3))
    web = k8s.Pod(name="web-0", labels={"app": "web"},
                  containers=[k8s.Container(requests={k8s.CPU: k8s.Q(4), k8s.MEMORY: k8s.Q(4 * GI)})])
    db = k8s.Pod(name="db-0", labels={"app": "db"},
                 containers=[k8s.Container(requests={k8s.CPU: k8s.Q(4), k8s.MEMORY: k8s.Q(4 * GI)})])
    recs = inf.pod_records([web, db])
    assert recs["resv_match"][0] != 0 and recs["resv_match"][1] == 0
    got = oracle.Oracle(to_c_config(prof), t).place_stream(recs)
    assert got[0] == 2 and got[1] < 0       # only the owner fits, into the operating pod's reservation
    # a current owner: AllocateOnce with an assigned pod -> no longer matchable
    op2 = copy.deepcopy(op)
    op2.annotations[rv.ANNOTATION_RESERVATION_CURRENT_OWNER] = _json.dumps({"name": "web-9", "namespace": "default"})
    inf.on_pod_update(op, op2, NOW)
    t2 = inf.table(NOW)
    assert int(t2["resv_assigned"][2]) == 1
    assert oracle.Oracle(to_c_config(prof), t2).place_stream(inf.pod_records([web]))[0] < 0
    # not Ready: not Available; deleted: no slot
    op3 = copy.deepcopy(op)
    op3.ready = False
    inf.on_pod_update(op2, op3, NOW)
    assert not int(inf.table(NOW)["resv_flags"][2])
    inf.on_pod_update(op3, op, NOW)
    assert int(inf.table(NOW)["resv_flags"][2]) & abi.RESV_PRESENT
    inf.on_pod_delete(op)
    assert not int(inf.table(NOW)["resv_flags"][2])


def test_operating_mode_pod_cpuset_is_the_slot_reserved_cpus():
    """an operating-mode pod holding a cpuset (its
    resource-status allocation) is a reservation whose reserved CPUs are that
    cpuset, less the CPUs of the pods it admitted (its current owners'
    allocations) -- nodenumaresource/reservation.go:76-113 -- so a matching
    cpuset pod takes them first."""
    import json as _json
    from koordinator_amd import numa as nm
    from koordinator_amd import reservation as rv
    rng = np.random.default_rng(5)
    prof = shipped_profile(numa=True, reservation=True)
    nodes = [k8s.Node(name=f"n{i}", allocatable={k8s.CPU: k8s.Q(32), k8s.MEMORY: k8s.Q(64 * GI), k8s.PODS: k8s.Q(110)})
             for i in range(3)]
    inf = Informer(prof, nodes, NOW)
    for n in nodes:
        inf.on_nrt(_nrt(rng, n.name))
    owners = [{"labelSelector": {"matchLabels": {"app": "web"}}}]
    op = k8s.Pod(name="op-0", uid="op0", node_name="n1",
                 labels={rv.LABEL_POD_OPERATING_MODE: "Reservation"},
                 annotations={rv.ANNOTATION_RESERVATION_OWNERS: _json.dumps(owners),
                              nm.ANNOTATION_RESOURCE_STATUS: _json.dumps({"cpuset": "4-7"})},
                 containers=[k8s.Container(requests={k8s.CPU: k8s.Q(4), k8s.MEMORY: k8s.Q(4 * GI)})])
    inf.on_pod_add(op, NOW)
    t = inf.table(NOW)
    topo = nm.linux_topology(2, 1, 8, 2)
    assert int(t["resv_flags"][1]) and [int(t[f"resv_cpus{w}"][1]) for w in range(4)] == \
        [int(x) for x in topo.mask([4, 5, 6, 7])]
    # a current owner holding CPUs 4-5 of them: the slot keeps 6-7
    web = k8s.Pod(name="web-1", uid="w1", node_name="n1", labels={"app": "web"},
                  annotations={nm.ANNOTATION_RESOURCE_STATUS: _json.dumps({"cpuset": "4-5"})},
                  containers=[k8s.Container(requests={k8s.CPU: k8s.Q(2), k8s.MEMORY: k8s.Q(GI)})])
    inf.on_pod_add(web, NOW)
    op2 = copy.deepcopy(op)
    op2.annotations[rv.ANNOTATION_RESERVATION_CURRENT_OWNER] = _json.dumps({"name": "web-1", "namespace": "default"})
    inf.on_pod_update(op, op2, NOW)
    t2 = inf.table(NOW)
    assert [int(t2[f"resv_cpus{w}"][1]) for w in range(4)] == [int(x) for x in topo.mask([6, 7])]


def test_operating_mode_pods_outside_the_envelope_stay_plain_pods():
    """a bound operating-mode pod whose requests the engine
    cannot hold as a reservation slot (ephemeral-storage, or nvidia.com/gpu
    without DeviceShare's device columns) stays a plain NodeInfo pod, counted in
    `outside_envelope` -- table() and delta() do not raise; more than
    RESV_SLOTS_MAX operating pods on one node likewise (the extra ones stay
    plain).  Its owners parsed on the first add stay and its current owners
    accumulate (cache.go:139-161); a terminated pod leaves the cache."""
    import json as _json
    from koordinator_amd import abi
    from koordinator_amd import reservation as rv
    prof = shipped_profile(reservation=True)
    nodes = [k8s.Node(name=f"n{i}", allocatable={k8s.CPU: k8s.Q(64), k8s.MEMORY: k8s.Q(128 * GI), k8s.PODS: k8s.Q(110),
                                                 k8s.EPHEMERAL: k8s.Q(100 * GI)}) for i in range(2)]
    inf = Informer(prof, nodes, NOW)
    op = lambda name, req, ann=None: k8s.Pod(name=name, uid=name, node_name="n0",
                                             labels={rv.LABEL_POD_OPERATING_MODE: "Reservation"},
                                             annotations=dict(ann or {}),
                                             containers=[k8s.Container(requests=req)])
    gpu = op("op-gpu", {k8s.CPU: k8s.Q(1), "nvidia.com/gpu": k8s.Q(1)})
    eph = op("op-eph", {k8s.CPU: k8s.Q(1), k8s.EPHEMERAL: k8s.Q(GI)})
    inf.on_pod_add(gpu, NOW)
    inf.on_pod_add(eph, NOW)
    t = inf.table(NOW)                              # no raise
    assert not int(t["resv_flags"][0]) & abi.RESV_PRESENT
    assert set(inf.outside_envelope) == {gpu.key, eph.key}
    assert int(t["npods"][0]) == 2                  # still NodeInfo pods
    # nine supported operating pods on one node: eight slots, the ninth plain
    owners = _json.dumps([{"labelSelector": {"matchLabels": {"app": "web"}}}])
    for k in range(9):
        inf.on_pod_add(op(f"op-{k}", {k8s.CPU: k8s.Q(1), k8s.MEMORY: k8s.Q(GI)},
                          {rv.ANNOTATION_RESERVATION_OWNERS: owners}), NOW)
    t = inf.table(NOW)
    assert t.resv_slots == abi.RESV_SLOTS_MAX and len(inf.outside_envelope) == 3
    res = inf.flush(_TableEngine(t), NOW)           # a delta does not raise either
    assert not res.needs_reload
    # sticky owners: an edit of the owners annotation does not change the groups the slot matches
    p0 = next(p for p in inf.cluster.node_pods["n0"] if p.name == "op-0")
    edited = copy.deepcopy(p0)
    edited.annotations[rv.ANNOTATION_RESERVATION_OWNERS] = _json.dumps([{"labelSelector": {"matchLabels": {"app": "db"}}}])
    edited.annotations[rv.ANNOTATION_RESERVATION_CURRENT_OWNER] = _json.dumps({"name": "web-1", "namespace": "default"})
    inf.on_pod_update(p0, edited, NOW)
    r = inf.reservations[rv.operating_reservation_name(edited)]
    assert r.owners[0].label_selector.match_labels == {"app": "web"} and r.assigned == 1
    cleared = copy.deepcopy(edited)
    del cleared.annotations[rv.ANNOTATION_RESERVATION_CURRENT_OWNER]
    inf.on_pod_update(edited, cleared, NOW)         # AddAssignedPod is cumulative: still assigned
    assert inf.reservations[rv.operating_reservation_name(cleared)].assigned == 1
    done = copy.deepcopy(cleared)
    done.phase = "Succeeded"
    inf.on_pod_update(cleared, done, NOW)           # terminated: out of the cache
    assert rv.operating_reservation_name(done) not in inf.reservations
