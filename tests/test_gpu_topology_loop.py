"""The scheduling loop end to end from objects with PodTopologySpread,
InterPodAffinity and DeviceShare in the profile: the informer registers each
batch of pending pods (reloading the snapshot when the batch brings new
constraints, terms or topology values), the engine places the batch, the
placed pods are bound back through the informer and the next batch is flushed
as row deltas (koordhip_update_nodes of the pts_* / ipa_* / dev_* rows).
Every batch's placements, and the spread / affinity counts after it, equal
the oracle's on the informer's image of the device state."""
import copy
import json

import numpy as np
import pytest

import oracle
from koordinator_amd import abi, deviceshare as ds, k8s
from koordinator_amd import interpodaffinity as ia
from koordinator_amd import topologyspread as ts
from koordinator_amd.config import shipped_profile, to_c_config, with_deviceshare, with_interpod_affinity, \
    with_topology_spread
from koordinator_amd.informer import Informer

pytestmark = pytest.mark.gpu

GI = 1 << 30
Q = k8s.Q
ZONE = "topology.kubernetes.io/zone"
RACK = "example.com/rack"


def _nodes(n, rng):
    out = []
    for i in range(n):
        lb = {ts.HOSTNAME: f"n{i}"}
        if rng.random() < 0.95:
            lb[ZONE] = f"z{i % 4}"
        if rng.random() < 0.9:
            lb[RACK] = f"r{i % 7}"
        a = {k8s.CPU: Q(32), k8s.MEMORY: Q(128 * GI), k8s.PODS: Q(40)}
        if i % 5 == 0:
            a.update({ds.NVIDIA_GPU: Q(4), ds.GPU_CORE: Q(400), ds.GPU_MEMORY_RATIO: Q(400),
                      ds.GPU_MEMORY: Q(64 * GI), ds.KOORD_GPU: Q(400)})
        out.append(k8s.Node(name=f"n{i}", allocatable=a, labels=lb))
    return out


def _device(name):
    return ds.Device(name, [ds.DeviceInfo("gpu", m, True, {ds.GPU_CORE: Q(100), ds.GPU_MEMORY_RATIO: Q(100),
                                                           ds.GPU_MEMORY: Q(16 * GI)}) for m in range(4)])


APPS = ["web", "db", "cache", "batch"]


def _pod(j, rng):
    app = APPS[j % 4]
    sel = ts.LabelSelector.of({"app": app})
    kw = {}
    if app == "web":
        kw["topology_spread_constraints"] = [ts.TopologySpreadConstraint(1, ZONE, ts.DO_NOT_SCHEDULE, sel),
                                             ts.TopologySpreadConstraint(2, ts.HOSTNAME, ts.SCHEDULE_ANYWAY, sel)]
        kw["pod_anti_affinity_required"] = [ia.PodAffinityTerm(sel, ts.HOSTNAME)]
    elif app == "db":
        kw["pod_affinity_preferred"] = [ia.WeightedPodAffinityTerm(40, ia.PodAffinityTerm(
            ts.LabelSelector.of({"app": "cache"}), ZONE))]
        kw["topology_spread_constraints"] = [ts.TopologySpreadConstraint(1, RACK, ts.SCHEDULE_ANYWAY, sel)]
    elif app == "cache":
        kw["pod_anti_affinity_preferred"] = [ia.WeightedPodAffinityTerm(20, ia.PodAffinityTerm(sel, RACK))]
    req = {k8s.CPU: Q("500m"), k8s.MEMORY: Q(GI)}
    if app == "batch" and rng.random() < 0.5:
        req[ds.KOORD_GPU] = Q(50)
    return k8s.Pod(name=f"p{j}", uid=f"p{j}", labels={"app": app}, priority=9500,
                   containers=[k8s.Container(requests=dict(req), limits=dict(req))], **kw)


def test_scheduling_loop_with_topology_plugins():
    import torch  # noqa: F401
    from koordinator_amd.engine import PlacementEngine
    rng = np.random.default_rng(29)
    prof = with_interpod_affinity(with_topology_spread(with_deviceshare(shipped_profile())))
    nodes = _nodes(60, rng)
    inf = Informer(prof, nodes, 0.0)
    for nd in nodes[::5]:
        inf.on_device(_device(nd.name))
    for j in range(30):   # running pods of the apps
        p = _pod(1000 + j, rng)
        p.node_name = nodes[int(rng.integers(0, 60))].name
        inf.on_pod_add(p, 0.0)
    cfg = to_c_config(prof)
    reloads = deltas = 0
    with PlacementEngine(prof, device=0) as e:
        loaded = False
        for b in range(5):
            now = 10.0 * (b + 1)
            batch = [_pod(b * 24 + j, rng) for j in range(24)]
            if inf.register_pods(batch) or not loaded:
                e.load_snapshot(inf.table(now))
                loaded = True
                reloads += 1
            else:
                res = inf.flush(e, now)
                if res.needs_reload:
                    e.load_snapshot(inf.table(now))
                    reloads += 1
                else:
                    deltas += res.rows > 0
            pods = inf.pod_records(batch)
            ext = inf.pod_ext_records(batch)
            o = oracle.Oracle(cfg, inf._table)
            ref = o.place_stream_ext(pods, ext)
            got = e.place_stream_ext(pods, ext)
            assert np.array_equal(got, ref), (b, np.flatnonzero(got != ref)[:5])
            assert np.array_equal(e.read_pts(), o.pts_counts()), b
            assert np.array_equal(e.read_ipa(), o.ipa_counts()), b
            assert (got >= 0).sum() > 12, b
            devs = e.fetch_devices(len(batch))
            # bind: the placed pods run (with their device allocations) from now on
            for p, nd, dv in zip(batch, got, devs):
                if nd < 0:
                    continue
                q = copy.deepcopy(p)
                q.node_name = nodes[int(nd)].name
                if dv[abi.DEV_GPU]:
                    minors = [m for s, m in enumerate(inf._table["dev_minor"][int(nd), abi.DEV_GPU])
                              if (int(dv[abi.DEV_GPU]) >> s) & 1]
                    q.annotations = {ds.ANNOTATION_DEVICE_ALLOCATED: json.dumps(
                        {"gpu": [{"minor": int(m), "resources": {ds.GPU_CORE: "50", ds.GPU_MEMORY_RATIO: "50",
                                                                 ds.GPU_MEMORY: "8Gi"}} for m in minors]})}
                inf.on_pod_add(q, now + 1.0)
    assert reloads >= 1 and deltas >= 1
