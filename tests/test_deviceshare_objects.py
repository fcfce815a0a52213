"""DeviceShare from Kubernetes objects: Device CRs, node allocatable device
scalars and the running pods' device-allocated annotations marshalled into the
sequential cycle's columns (marshal.ext_row / deviceshare.device_rows), pod ext
records from pod requests, and the oracle's cycle over that snapshot; marked
gpu, libkoordhip.so on the same snapshot equals the oracle."""
import json

import numpy as np
import pytest

import oracle
from koordinator_amd import abi, deviceshare as ds, k8s
from koordinator_amd.config import shipped_profile, to_c_config, with_deviceshare, with_normalized_scores
from koordinator_amd.marshal import ClusterState, MarshalError, build_table, pod_records, static_classes_for
from koordinator_amd.nodefilters import PREFER_NO_SCHEDULE, Taint, Toleration
from koordinator_amd.reservation import NodeSelectorRequirement as R, NodeSelectorTerm as T

GI = 1 << 30
Q = k8s.Q


def _gpu(minor, mem=16 * GI, health=True):
    return ds.DeviceInfo("gpu", minor, health, {ds.GPU_CORE: Q(100), ds.GPU_MEMORY_RATIO: Q(100), ds.GPU_MEMORY: Q(mem)})


def _rdma(minor):
    return ds.DeviceInfo("rdma", minor, True, {ds.RDMA: Q(100)})


def _node(name, ngpu=0, mem=16 * GI, rdma=0, labels=None, taints=()):
    a = {k8s.CPU: Q(32), k8s.MEMORY: Q(128 * GI), k8s.PODS: Q(110)}
    if ngpu:
        # the slo-controller's sync of the Device CR (device_resource_calculator.go:84-100)
        a.update({ds.NVIDIA_GPU: Q(ngpu), ds.GPU_CORE: Q(100 * ngpu), ds.GPU_MEMORY_RATIO: Q(100 * ngpu),
                  ds.GPU_MEMORY: Q(mem * ngpu), ds.KOORD_GPU: Q(100 * ngpu)})
    if rdma:
        a[ds.RDMA] = Q(100 * rdma)
    n = k8s.Node(name=name, allocatable=a, labels=dict(labels or {}))
    n.taints = list(taints)
    return n


def _pod(name, req, node="", alloc=None, pref=None, tols=()):
    r = {k8s.CPU: Q("1"), k8s.MEMORY: Q(2 * GI)}
    r.update({k: Q(v) for k, v in req.items()})
    ann = {ds.ANNOTATION_DEVICE_ALLOCATED: json.dumps(alloc)} if alloc else {}
    return k8s.Pod(name=name, uid=name, node_name=node, annotations=ann, priority=9500,
                   containers=[k8s.Container(requests=dict(r), limits=dict(r))],
                   preferred_node_affinity=list(pref or []), tolerations=list(tols))


def cluster():
    nodes = [_node("g0", 4, rdma=2, labels={"zone": "a"}), _node("g1", 2, mem=80 * GI, labels={"zone": "b"}),
             _node("c0", labels={"zone": "a"}, taints=[Taint("spot", "true", PREFER_NO_SCHEDULE)]), _node("c1")]
    devices = {"g0": ds.Device("g0", [_gpu(3), _gpu(0), _gpu(1), _gpu(2), _rdma(0), _rdma(1)]),
               "g1": ds.Device("g1", [_gpu(0, 80 * GI), _gpu(1, 80 * GI, health=False)]),
               "c0": ds.Device("c0", [])}
    running = _pod("r0", {ds.KOORD_GPU: 50}, node="g0",
                   alloc={"gpu": [{"minor": 1, "resources": {ds.GPU_CORE: "50", ds.GPU_MEMORY_RATIO: "50",
                                                             ds.GPU_MEMORY: "8Gi"}}]})
    return ClusterState(nodes=nodes, devices=devices, node_pods={"g0": [running]}, pods={running.key: running})


def stream():
    pref = [(10, T([R("zone", "In", ["b"])]))]
    return [_pod("p0", {ds.NVIDIA_GPU: 1}), _pod("p1", {ds.KOORD_GPU: 50}, pref=pref),
            _pod("p2", {}), _pod("p3", {ds.GPU_MEMORY: 8 * GI, ds.RDMA: 100}),
            _pod("p4", {ds.NVIDIA_GPU: 2}), _pod("p5", {}, tols=[Toleration("spot", "Exists")]),
            _pod("p6", {ds.NVIDIA_GPU: 4}), _pod("p7", {ds.KOORD_GPU: 100}, pref=pref)]


def _profile():
    return with_normalized_scores(with_deviceshare(shipped_profile()), affinity=1, taint=1)


def test_device_columns_from_objects():
    prof = _profile()
    c = cluster()
    sc = static_classes_for(stream(), prof)
    t = build_table(c, prof, 0.0, sc)
    assert t.has_ext and t.dev_slots == 4
    assert t["dev_present"].tolist() == [1, 1, 1, 0]
    G = abi.DEV_GPU
    assert t["dev_minor"][0, G].tolist() == [0, 1, 2, 3]                  # ascending minors
    assert t["dev_used"][0, G, 1].tolist() == [50, 50, 8 * GI]            # the running pod's allocation
    assert t["dev_total"][1, G, 1].tolist() == [0, 0, 0]                  # unhealthy: no resources
    assert t["dev_minor"][0, abi.DEV_RDMA, :2].tolist() == [0, 1]
    xi = ds.XRES_INDEX
    assert t["xalloc"][0, xi[ds.NVIDIA_GPU]] == 4 and t["xalloc"][0, xi[ds.RDMA]] == 200
    assert t["xrequested"][0, xi[ds.KOORD_GPU]] == 50 and t["xrequested"][1].sum() == 0
    # static_score: zone-b preference on g1, the spot taint on c0
    p1 = pod_records(stream(), prof, static_classes=sc)
    cls = int(p1["static_class"][1])
    assert t["static_score"][:, 0, cls].tolist() == [0, 10, 0, 0]
    assert t["static_score"][:, 1, int(p1["static_class"][0])].tolist() == [0, 0, 1, 0]
    assert t["static_score"][:, 1, int(p1["static_class"][5])].tolist() == [0, 0, 0, 0]


def test_pod_ext_records_from_objects():
    x = ds.pod_ext_records(stream())
    dev = (x["flags"] & abi.PODX_DEVICE) != 0
    assert dev.tolist() == [True, True, False, True, True, False, True, True]
    assert x["dev_req"][0, abi.DEV_GPU].tolist() == [100, 100, -1]
    assert x["dev_req"][3, abi.DEV_GPU].tolist() == [-1, -1, 8 * GI] or x["dev_req"][3, abi.DEV_GPU, 2] == 8 * GI
    assert x["dev_req"][3, abi.DEV_RDMA, 0] == 100


def test_device_pod_needs_deviceshare_profile():
    with pytest.raises(MarshalError):
        pod_records([_pod("g", {ds.NVIDIA_GPU: 1})], shipped_profile())


def _oracle_run(prof, t, pods, ext):
    o = oracle.Oracle(to_c_config(prof), t)
    out, dv = o.place_stream_ext(pods, ext, devices=True)
    return o, out, dv


def test_oracle_cycle_on_objects():
    prof = _profile()
    c = cluster()
    objs = stream()
    sc = static_classes_for(objs, prof)
    t = build_table(c, prof, 0.0, sc)
    pods = pod_records(objs, prof, static_classes=sc)
    ext = ds.pod_ext_records(objs)
    o, out, dv = _oracle_run(prof, t, pods, ext)
    # device pods land on GPU nodes with their devices; p4 (2 whole GPUs) and
    # p6 (4) find no node: g0 has one free GPU left after p0 / p3 (the running
    # pod holds half of minor 1) and g1 has one healthy GPU
    for j in (0, 1, 3, 7):
        assert out[j] in (0, 1), j
        assert dv[j, abi.DEV_GPU] != 0
    assert out[4] == -1 and out[6] == -1
    assert out[1] == 1                                    # the zone-b preference (NodeAffinity Score)
    assert out[3] == 0 and dv[3, abi.DEV_RDMA] != 0       # RDMA only on g0
    assert out[2] >= 0 and out[5] >= 0
    used = o.dev_state()["dev_used"]
    assert used[0, abi.DEV_GPU, :, 0].tolist() == [100, 50, 0, 100]   # p0, running, p3 (memory only), p7
    assert used[1, abi.DEV_GPU, :, 0].tolist() == [50, 0, 0, 0]       # p1
    assert used[0, abi.DEV_GPU, 2, 2] == 8 * GI and used[0, abi.DEV_GPU, 2, 1] == 50   # fillGPUTotalMem


@pytest.mark.gpu
def test_engine_cycle_on_objects():
    import torch  # noqa: F401
    from koordinator_amd.engine import PlacementEngine
    prof = _profile()
    objs = stream()
    sc = static_classes_for(objs, prof)
    t = build_table(cluster(), prof, 0.0, sc)
    pods = pod_records(objs, prof, static_classes=sc)
    ext = ds.pod_ext_records(objs)
    o, ref, rdv = _oracle_run(prof, t, pods, ext)
    with PlacementEngine(prof, device=0) as e:
        e.load_snapshot(t)
        got = e.place_stream_ext(pods, ext)
        gdv = e.fetch_devices(len(pods))
        gst = e.read_devices()
    assert np.array_equal(got, ref)
    assert np.array_equal(gdv, rdv)
    assert np.array_equal(gst["dev_used"], o.dev_state()["dev_used"])


class _TableEngine:
    """update_nodes into a host table (the informer's delta target)."""

    def __init__(self, table):
        self.table = table.copy()

    def update_nodes(self, idx, rows):
        for c in rows.cols:
            self.table.cols[c][idx] = rows.cols[c]


def test_informer_device_events_rows_equal_rebuild():
    """Device CR add / update / delete and device pods binding / finishing:
    the flushed rows equal a rebuilt snapshot, column by column."""
    import copy
    from koordinator_amd.informer import Informer
    prof = _profile()
    c = cluster()
    inf = Informer(prof, c.nodes, 0.0)
    for name, d in c.devices.items():
        inf.on_device(d)
    for p in c.node_pods["g0"]:
        inf.on_pod_add(p, 0.0)
    inf.register_pods(stream())
    eng = _TableEngine(inf.table(0.0))
    alloc = lambda m, pct: {"gpu": [{"minor": m, "resources": {ds.GPU_CORE: str(pct), ds.GPU_MEMORY_RATIO: str(pct),
                                                              ds.GPU_MEMORY: f"{pct * 16 // 100}Gi"}}]}
    steps = [
        lambda: inf.on_pod_add(_pod("b0", {ds.NVIDIA_GPU: 1}, node="g0", alloc=alloc(3, 100)), 1.0),
        lambda: inf.on_device(ds.Device("c1", [_gpu(0), _gpu(1)])),               # a new Device CR
        lambda: inf.on_pod_add(_pod("b1", {ds.KOORD_GPU: 25}, node="c1", alloc=alloc(1, 25)), 2.0),
        lambda: inf.on_device(ds.Device("g1", [_gpu(0, 80 * GI), _gpu(1, 80 * GI)])),   # minor 1 healthy again
        lambda: inf.on_pod_delete(c.node_pods["g0"][0]),                          # the running pod finished
        lambda: inf.on_device_delete("c0"),
    ]
    for k, step in enumerate(steps):
        step()
        res = inf.flush(eng, 3.0 + k)
        assert not res.needs_reload, k
        want = build_table(inf.cluster, prof, 3.0 + k, inf.static_classes)
        for col in want.cols:
            assert np.array_equal(eng.table.cols[col], want.cols[col]), (k, col)
    # more devices of one type than the snapshot's dev_slots: reload
    inf.on_device(ds.Device("c1", [_gpu(m) for m in range(6)]))
    assert inf.delta(9.0)[2].needs_reload
    assert inf.table(9.0).dev_slots == 6
