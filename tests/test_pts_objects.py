"""PodTopologySpread from Kubernetes objects: nodes' topology labels, running
pods and the pending pods' topologySpreadConstraints marshalled into the pts_*
columns (marshal.pts_row / topologyspread) and pod ext records, the oracle's
cycle over that snapshot (spread rules checked step by step), informer deltas
equal to a rebuild; marked gpu, libkoordhip.so on the same snapshot equals the
oracle.  Upstream semantics are not vendored: parity with upstream is
unpinned (see test_pts_oracle.py)."""
import numpy as np
import pytest

import oracle
from koordinator_amd import abi, k8s
from koordinator_amd import topologyspread as ts
from koordinator_amd.config import shipped_profile, to_c_config, with_topology_spread
from koordinator_amd.marshal import ClusterState, MarshalError, build_table, pod_ext_records, pod_records

GI = 1 << 30
Q = k8s.Q
WEB = ts.LabelSelector.of({"app": "web"})
DB = ts.LabelSelector.of({"app": "db"})
ZONE = "topology.kubernetes.io/zone"


def _node(name, zone=None, extra=None):
    lb = {ts.HOSTNAME: name}
    if zone:
        lb[ZONE] = zone
    lb.update(extra or {})
    return k8s.Node(name=name, allocatable={k8s.CPU: Q(16), k8s.MEMORY: Q(64 * GI), k8s.PODS: Q(110)}, labels=lb)


def _pod(name, app, cons=(), node="", ns="default", selector=None):
    r = {k8s.CPU: Q("1"), k8s.MEMORY: Q(GI)}
    return k8s.Pod(name=name, uid=name, namespace=ns, node_name=node, labels={"app": app}, priority=9500,
                   containers=[k8s.Container(requests=dict(r), limits=dict(r))], node_selector=dict(selector or {}),
                   topology_spread_constraints=list(cons))


def _web(name, skew=1):
    return _pod(name, "web", [ts.TopologySpreadConstraint(skew, ZONE, ts.DO_NOT_SCHEDULE, WEB),
                              ts.TopologySpreadConstraint(1, ts.HOSTNAME, ts.SCHEDULE_ANYWAY, WEB)])


def _db(name):
    return _pod(name, "db", [ts.TopologySpreadConstraint(1, ZONE, ts.SCHEDULE_ANYWAY, DB)])


def cluster():
    nodes = [_node("a", "z1"), _node("b", "z1"), _node("c", "z1"), _node("d", "z2"), _node("e", "z2"), _node("f")]
    running = [_pod("r0", "web", node="a"), _pod("r1", "web", node="a"), _pod("r2", "web", node="b"),
               _pod("r3", "db", node="d"), _pod("r4", "web", node="d", ns="other")]
    c = ClusterState(nodes=nodes, pods={p.key: p for p in running})
    for p in running:
        c.node_pods.setdefault(p.node_name, []).append(p)
    return c


def stream():
    return [_web(f"w{j}") for j in range(6)] + [_db("d0"), _db("d1"), _pod("plain", "x")]


def _profile(**kw):
    return with_topology_spread(shipped_profile(), **kw)


def _snapshot(prof=None):
    prof = prof or _profile()
    objs = stream()
    c = cluster()
    c.spread = ts.registry_for(objs)
    t = build_table(c, prof, 0.0)
    return c, t, objs, pod_records(objs, prof), pod_ext_records(objs, prof, c.spread)


def test_spread_columns_from_objects():
    c, t, objs, pods, ext = _snapshot()
    reg = c.spread
    assert t.has_pts and reg.keys == [ZONE, ts.HOSTNAME]
    assert t.pts.hostname == 0b10 and t.pts.ndom[:2] == [2, 0] and t.pts.classes == 2
    assert t["pts_dom"][:, 0].tolist() == [0, 0, 0, 1, 1, -1]
    assert t["pts_dom"][:, 1].tolist() == list(range(6))
    # constraints: (web, zone) (web, hostname) (db, zone), namespace default
    assert [k for _, _, k in reg.cons] == [0, 1, 0]
    assert t["pts_cnt"][:, 0].tolist() == [2, 1, 0, 0, 0, 0]          # r4 is in another namespace
    assert t["pts_cnt"][:, 1].tolist() == [2, 1, 0, 0, 0, 0]
    assert t["pts_cnt"][:, 2].tolist() == [0, 0, 0, 1, 0, 0]
    # class 0 (web: hard zone, soft hostname), class 1 (db: soft zone)
    assert t["pts_elig"].tolist() == [0b1111] * 5 + [0b0110]
    assert ext["pts_n"].tolist() == [2] * 6 + [1, 1, 0]
    assert ext["pts_match"].tolist() == [0b011] * 6 + [0b100] * 2 + [0]
    assert ext["pts_fl"][0, :2].tolist() == [abi.PTS_HARD | abi.PTS_SELF, abi.PTS_SELF]
    assert ext["pts_class"][6] == 1


def test_pod_ext_records_need_the_registry():
    with pytest.raises(MarshalError):
        pod_ext_records(stream(), _profile())
    c, t, objs, pods, ext = _snapshot()
    late = _pod("late", "web", [ts.TopologySpreadConstraint(1, "rack", ts.DO_NOT_SCHEDULE, WEB)])
    with pytest.raises(MarshalError):
        pod_ext_records([late], _profile(), c.spread)


def test_oracle_cycle_on_objects_keeps_the_skew():
    """Each web pod lands in a zone whose count + 1 - min <= 1 at that step
    (zones z1 = 3 / z2 = 0 at start, so the first three go to z2), never on
    the zoneless node f; db pods spread softly; the counts advance."""
    c, t, objs, pods, ext = _snapshot()
    o = oracle.Oracle(to_c_config(_profile()), t)
    out = o.place_stream_ext(pods, ext)
    zone = {0: "z1", 1: "z1", 2: "z1", 3: "z2", 4: "z2"}
    cnt = {"z1": 3, "z2": 0}
    for j in range(6):
        assert out[j] in zone, (j, out[j])
        z = zone[int(out[j])]
        assert cnt[z] + 1 - min(cnt.values()) <= 1, (j, cnt)
        cnt[z] += 1
    assert [zone[int(i)] for i in out[:3]] == ["z2"] * 3
    assert out[6] >= 0 and out[7] >= 0 and out[8] >= 0
    got = o.pts_counts()
    assert got[:, 0].sum() == 3 + 6 and got[:, 2].sum() == 1 + 2
    assert got[:, 1].tolist() == got[:, 0].tolist()


def test_filter_only_profile_and_hard_fail():
    """maxSkew 1 with every z2 node full of pods: the web pods fit only until
    the skew bound stops them."""
    prof = _profile(weight=0)
    c, t, objs, pods, ext = _snapshot(prof)
    t["alloc_pods"][3:5] = t["npods"][3:5]           # z2 full: z1 = 3 stays ahead by more than 1
    o = oracle.Oracle(to_c_config(prof), t)
    out = o.place_stream_ext(pods, ext)
    assert (out[:6] == -1).all()
    assert (out[6:] >= 0).all()


@pytest.mark.gpu
def test_engine_cycle_on_objects():
    import torch  # noqa: F401
    from koordinator_amd.engine import PlacementEngine
    prof = _profile()
    c, t, objs, pods, ext = _snapshot(prof)
    o = oracle.Oracle(to_c_config(prof), t)
    ref = o.place_stream_ext(pods, ext)
    with PlacementEngine(prof, device=0) as e:
        e.load_snapshot(t)
        got = e.place_stream_ext(pods, ext)
        cnt = e.read_pts()
    assert np.array_equal(got, ref)
    assert np.array_equal(cnt, o.pts_counts())


class _TableEngine:
    def __init__(self, table):
        self.table = table.copy()

    def update_nodes(self, idx, rows):
        for col in rows.cols:
            self.table.cols[col][idx] = rows.cols[col]


def test_informer_spread_events_rows_equal_rebuild():
    """Pods binding / finishing and nodes relabelled within the known zones:
    the flushed rows equal a rebuilt snapshot; a new zone value or a pod with
    constraints the snapshot lacks asks for a reload."""
    from koordinator_amd.informer import Informer
    prof = _profile()
    c = cluster()
    inf = Informer(prof, c.nodes, 0.0)
    for p in c.pods.values():
        inf.on_pod_add(p, 0.0)
    assert inf.register_pods(stream()) in (True, False)
    eng = _TableEngine(inf.table(0.0))
    assert eng.table.has_pts
    assert not inf.register_pods(stream())
    steps = [
        lambda: inf.on_pod_add(_pod("b0", "web", node="e"), 1.0),
        lambda: inf.on_pod_add(_pod("b1", "db", node="a"), 1.0),
        lambda: inf.on_pod_delete(c.pods["default/r0"]),
        lambda: inf.on_node_update(None, _node("c", "z2")),            # c moves to z2
        lambda: inf.on_node_update(None, _node("e")),                  # e loses its zone
        lambda: inf.on_node_update(None, _node("f", "z1")),            # f gains one
    ]
    for k, step in enumerate(steps):
        step()
        res = inf.flush(eng, 2.0 + k)
        assert not res.needs_reload, k
        want = build_table(inf.cluster, prof, 2.0 + k, inf.static_classes)
        for col in want.cols:
            assert np.array_equal(eng.table.cols[col], want.cols[col]), (k, col)
    inf.on_node_update(None, _node("b", "z3"))
    assert inf.delta(9.0)[2].needs_reload
    t = inf.table(9.0)
    assert t.pts.ndom[0] == 3
    late = _pod("late", "web", [ts.TopologySpreadConstraint(1, "rack", ts.DO_NOT_SCHEDULE, WEB)])
    assert inf.register_pods([late])
    assert inf.table(10.0).pts.keys == 3
