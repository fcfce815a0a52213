"""InterPodAffinity: the host's count entries (koordinator_amd/interpodaffinity.py)
and the C oracle (oracle/ipa_oracle.c) against a literal restatement of
upstream k8s v1.24 interpodaffinity over objects (oracle/ipa_upstream.py) --
Filter, raw Score and the cycle, on hand cases (the first pod of a
self-affine series, namespace selectors, nodes without the topology label,
hardPodAffinityWeight) and seeded random clusters; informer deltas equal a
rebuild.  Upstream is not vendored: parity with upstream is unpinned; device
vs oracle is checked bit for bit in test_gpu_ipa.py."""
import random

import numpy as np
import pytest

import oracle
from oracle import ipa_upstream as U
from koordinator_amd import abi, k8s
from koordinator_amd import interpodaffinity as ia
from koordinator_amd import topologyspread as ts
from koordinator_amd.config import PLUGIN_IPA, Profile, shipped_profile, to_c_config, with_interpod_affinity
from koordinator_amd.marshal import ClusterState, MarshalError, build_table, pod_ext_records, pod_records

GI = 1 << 30
Q = k8s.Q
ZONE = "topology.kubernetes.io/zone"
HOST = ts.HOSTNAME
T = ia.PodAffinityTerm
W = ia.WeightedPodAffinityTerm
S = ts.LabelSelector.of


def node(name, zone=None, extra=None, cpu=64):
    lb = {HOST: name}
    if zone:
        lb[ZONE] = zone
    lb.update(extra or {})
    return k8s.Node(name=name, allocatable={k8s.CPU: Q(cpu), k8s.MEMORY: Q(256 * GI), k8s.PODS: Q(110)}, labels=lb)


def pod(name, labels, ns="default", node_name="", aff=(), anti=(), paff=(), panti=(), cpu="1"):
    r = {k8s.CPU: Q(cpu), k8s.MEMORY: Q(GI)}
    return k8s.Pod(name=name, uid=f"{ns}/{name}", namespace=ns, node_name=node_name, labels=dict(labels),
                   priority=9500, containers=[k8s.Container(requests=dict(r), limits=dict(r))],
                   pod_affinity_required=list(aff), pod_anti_affinity_required=list(anti),
                   pod_affinity_preferred=list(paff), pod_anti_affinity_preferred=list(panti))


def ipa_profile(weight=1, filt=True, hard=1):
    return with_interpod_affinity(Profile(filters=(), scores={}), weight=weight, filter=filt,
                                  hard_pod_affinity_weight=hard)


def snapshot(nodes, running, pending, prof, ns_labels=None):
    c = ClusterState(nodes=list(nodes), pods={p.key: p for p in running})
    for p in running:
        c.node_pods.setdefault(p.node_name, []).append(p)
    c.spread = ts.SpreadRegistry()
    c.ipa = ia.IpaRegistry(c.spread, ns_labels, prof.interpodaffinity.hard_pod_affinity_weight)
    for p in pending:
        c.ipa.register(p)
    t = build_table(c, prof, 0.0)
    return c, t, pod_records(pending, prof), pod_ext_records(pending, prof, c.spread, c.ipa)


def check_eval(nodes, running, pending, prof, ns_labels=None):
    """Per pending pod on the initial state: the oracle's IPA status bit and
    raw plane equal the literal upstream Filter and Score."""
    c, t, pods, ext = snapshot(nodes, running, pending, prof, ns_labels)
    r = oracle.Oracle(to_c_config(prof), t).eval_ext(pods, ext, k=0)
    node_pods = {k: list(v) for k, v in c.node_pods.items()}
    hw = prof.interpodaffinity.hard_pod_affinity_weight
    for j, p in enumerate(pending):
        feas, raw, _ = U.evaluate(p, nodes, node_pods, ns_labels, hw)
        got_feas = [i for i in range(len(nodes)) if not r["status"][j, i] & abi.ST_IPA_FAIL]
        assert got_feas == feas, (p.name, got_feas, feas)
        assert r["scores"][j, abi.NPLUGINS + 4].tolist() == raw, (p.name, r["scores"][j, abi.NPLUGINS + 4], raw)
    return c, t, pods, ext


def check_stream(nodes, running, pending, prof, ns_labels=None):
    c, t, pods, ext = snapshot(nodes, running, pending, prof, ns_labels)
    o = oracle.Oracle(to_c_config(prof), t)
    got = o.place_stream_ext(pods, ext)
    want, _ = U.place_stream(pending, nodes, {k: list(v) for k, v in c.node_pods.items()}, ns_labels,
                             prof.interpodaffinity.hard_pod_affinity_weight, prof.scores.get(PLUGIN_IPA, 0))
    assert got.tolist() == want
    return got, o, t


# ------------------------------------------------------------------ hand cases
NODES = [node("a", "z1"), node("b", "z1"), node("c", "z2"), node("d", "z2"), node("e")]
WEB = S({"app": "web"})
DB = S({"app": "db"})


def test_required_affinity_to_a_zone():
    """web pods need a db pod in their zone: only z2's nodes (db on d) pass;
    e has no zone label and fails."""
    running = [pod("db0", {"app": "db"}, node_name="d")]
    p = pod("w", {"app": "web"}, aff=[T(DB, ZONE)])
    c, t, pods, ext = check_eval(NODES, running, [p], ipa_profile())
    r = oracle.Oracle(to_c_config(ipa_profile()), t).eval_ext(pods, ext)
    assert [i for i in range(5) if not r["status"][0, i] & abi.ST_IPA_FAIL] == [2, 3]


def test_first_pod_of_a_self_affine_series():
    """No pod matches the term anywhere and the pod matches its own term: every
    node carrying the key passes (the node without the zone still fails)."""
    p = pod("w", {"app": "web"}, aff=[T(WEB, ZONE)])
    c, t, pods, ext = check_eval(NODES, [], [p], ipa_profile())
    assert ext["ipa_flags"][0] == abi.IPA_SELF
    r = oracle.Oracle(to_c_config(ipa_profile()), t).eval_ext(pods, ext)
    assert [i for i in range(5) if not r["status"][0, i] & abi.ST_IPA_FAIL] == [0, 1, 2, 3]
    # ... and a pod that does not match its own term stays pending
    q = pod("x", {"app": "other"}, aff=[T(WEB, ZONE)])
    check_eval(NODES, [], [q], ipa_profile())


def test_anti_affinity_both_ways():
    """The pod's own anti-affinity (no web pod on the same host) and a running
    pod's anti-affinity to web pods in its zone."""
    running = [pod("w0", {"app": "web"}, node_name="a"),
               pod("g", {"app": "guard"}, node_name="c", anti=[T(WEB, ZONE)])]
    p = pod("w1", {"app": "web"}, anti=[T(WEB, HOST)])
    check_eval(NODES, running, [p], ipa_profile())
    c, t, pods, ext = snapshot(NODES, running, [p], ipa_profile())
    r = oracle.Oracle(to_c_config(ipa_profile()), t).eval_ext(pods, ext)
    assert [i for i in range(5) if not r["status"][0, i] & abi.ST_IPA_FAIL] == [1, 4]


def test_preferred_terms_and_hard_weight():
    """Preferred affinity to db (weight 5), preferred anti-affinity to web
    (weight 3) and a running pod's required affinity to web pods (scored with
    hardPodAffinityWeight), at hardPodAffinityWeight 1 and 0."""
    running = [pod("db0", {"app": "db"}, node_name="a"), pod("db1", {"app": "db"}, node_name="c"),
               pod("w0", {"app": "web"}, node_name="b"),
               pod("f", {"app": "fan"}, node_name="d", aff=[T(WEB, ZONE)])]
    p = pod("w1", {"app": "web"}, paff=[W(5, T(DB, ZONE))], panti=[W(3, T(WEB, HOST))])
    for hw in (1, 0):
        check_eval(NODES, running, [p], ipa_profile(hard=hw))


def test_namespaces_and_selectors():
    """A term listing namespaces, one with a namespace selector, one with an
    empty (every namespace) selector; a nil label selector matches nothing."""
    ns_labels = {"default": {"team": "x"}, "prod": {"team": "y"}, "dev": {"team": "x"}}
    running = [pod("db0", {"app": "db"}, ns="prod", node_name="a"), pod("db1", {"app": "db"}, ns="dev", node_name="c")]
    terms = [T(DB, ZONE, namespaces=("prod",)), T(DB, ZONE, namespace_selector=S({"team": "x"})),
             T(DB, ZONE, namespace_selector=ts.LabelSelector()), T(None, ZONE, namespaces=("prod",))]
    pending = [pod(f"p{j}", {"app": "web"}, aff=[t]) for j, t in enumerate(terms)]
    check_eval(NODES, running, pending, ipa_profile(), ns_labels)


def test_streams_hand():
    running = [pod("db0", {"app": "db"}, node_name="c")]
    pending = ([pod(f"w{j}", {"app": "web"}, anti=[T(WEB, HOST)], paff=[W(10, T(DB, ZONE))]) for j in range(6)]
               + [pod("z", {"app": "zz"}, aff=[T(S({"app": "zz"}), ZONE)])]
               + [pod(f"v{j}", {"app": "v"}, panti=[W(7, T(S({"app": "v"}), ZONE))]) for j in range(4)])
    got, o, t = check_stream(NODES, running, pending, ipa_profile())
    assert sorted(got[:5].tolist()) == [0, 1, 2, 3, 4] and got[5] == -1   # one web pod per host, then none
    # the counts advance with each placement: the oracle's entries equal a rebuild after the binds
    c2 = ClusterState(nodes=NODES, node_pods={})
    for p, i in zip(pending, got):
        if i >= 0:
            c2.node_pods.setdefault(NODES[i].name, []).append(p)
    c2.node_pods.setdefault("c", []).insert(0, running[0])
    reg = o.table.ipa
    assert reg is not None


# ------------------------------------------------------------------ random clusters
POOL_SEL = [S({"app": "a"}), S({"app": "b"}), S({"app": "c"}), S({}, [ts.LabelRequirement("tier", "In", ("fe",))]),
            S({}, [ts.LabelRequirement("app", "NotIn", ("a",))])]


def random_case(seed, n_nodes=14, n_running=16, n_pending=30):
    rnd = random.Random(seed)
    keys = [ZONE, HOST, "rack"]
    nodes = []
    for j in range(n_nodes):
        extra = {"rack": f"r{rnd.randrange(4)}"} if rnd.random() < 0.8 else {}
        nodes.append(node(f"n{j}", f"z{rnd.randrange(3)}" if rnd.random() < 0.85 else None, extra))

    pool = [T(rnd.choice(POOL_SEL), rnd.choice(keys), namespaces=(("default", "other") if rnd.random() < 0.2 else ()))
            for _ in range(5)]

    def term():
        return rnd.choice(pool)

    def mkpod(name, node_name=""):
        lb = {"app": rnd.choice("abc")}
        if rnd.random() < 0.5:
            lb["tier"] = rnd.choice(["fe", "be"])
        kw = {}
        r = rnd.random()
        if r < 0.25:
            kw["anti"] = [term()]
        elif r < 0.4:
            kw["aff"] = [term()] if rnd.random() < 0.7 else list(dict.fromkeys([term(), term()]))
        if rnd.random() < 0.35:
            kw["paff"] = [W(rnd.choice([10, 50]), term())]
        if rnd.random() < 0.3:
            kw["panti"] = [W(rnd.choice([10, 50]), term())]
        return pod(name, lb, ns=rnd.choice(["default", "default", "other"]), node_name=node_name, **kw)

    running = [mkpod(f"r{j}", nodes[rnd.randrange(n_nodes)].name) for j in range(n_running)]
    pending = [mkpod(f"p{j}") for j in range(n_pending)]
    return nodes, running, pending


def fitting(nodes, running, pending):
    """The longest prefix of `pending` whose entries fit KOORDHIP_IPA_ENTRIES."""
    for m in (len(pending), 20, 12, 6):
        try:
            snapshot(nodes, running, pending[:m], ipa_profile())
            return pending[:m]
        except ia.IpaError:
            continue
    pytest.skip("entries beyond the envelope")


@pytest.mark.parametrize("seed", range(8))
def test_random_eval_matches_upstream(seed):
    nodes, running, pending = random_case(seed)
    pending = fitting(nodes, running, pending)
    assert len(pending) >= 6
    check_eval(nodes, running, pending, ipa_profile())


@pytest.mark.parametrize("seed", range(8))
def test_random_stream_matches_upstream(seed):
    nodes, running, pending = random_case(100 + seed)
    pending = fitting(nodes, running, pending)
    assert len(pending) >= 6
    check_stream(nodes, running, pending, ipa_profile(weight=3))


def test_entry_limit_and_coverage():
    reg = ia.IpaRegistry(ts.SpreadRegistry())
    with pytest.raises(ia.IpaError):
        for j in range(abi.IPA_ENTRIES + 1):
            reg.register(pod(f"p{j}", {"app": "x"}, anti=[T(S({"app": f"v{j}"}), HOST)]))
    c, t, pods, ext = snapshot(NODES, [], [pod("w", {"app": "web"}, anti=[T(WEB, HOST)])], ipa_profile())
    late = pod("late", {"app": "web"}, aff=[T(DB, ZONE)])
    with pytest.raises(MarshalError):
        pod_ext_records([late], ipa_profile(), c.spread, c.ipa)


# ------------------------------------------------------------------ informer
class _TableEngine:
    def __init__(self, table):
        self.table = table.copy()

    def update_nodes(self, idx, rows):
        for col in rows.cols:
            self.table.cols[col][idx] = rows.cols[col]


def test_informer_ipa_events_rows_equal_rebuild():
    from koordinator_amd.informer import Informer
    prof = with_interpod_affinity(shipped_profile())
    nodes = [node("a", "z1"), node("b", "z1"), node("c", "z2"), node("d", "z2")]
    inf = Informer(prof, nodes, 0.0)
    inf.on_pod_add(pod("db0", {"app": "db"}, node_name="a"), 0.0)
    inf.on_pod_add(pod("g", {"app": "guard"}, node_name="c", anti=[T(WEB, ZONE)]), 0.0)
    pending = [pod("w", {"app": "web"}, anti=[T(WEB, HOST)], paff=[W(5, T(DB, ZONE))])]
    assert inf.register_pods(pending)
    eng = _TableEngine(inf.table(0.0))
    assert eng.table.has_ipa and not inf.register_pods(pending)
    steps = [
        lambda: inf.on_pod_add(pod("w0", {"app": "web"}, node_name="b"), 1.0),     # counts in web entries
        lambda: inf.on_pod_add(pod("db1", {"app": "db"}, node_name="d"), 1.0),
        lambda: inf.on_pod_delete(pod("db0", {"app": "db"}, node_name="a")),
        lambda: inf.on_node_update(None, node("b", "z2")),
    ]
    for k, step in enumerate(steps):
        step()
        res = inf.flush(eng, 2.0 + k)
        assert not res.needs_reload, k
        want = build_table(inf.cluster, prof, 2.0 + k, inf.static_classes)
        for col in want.cols:
            assert np.array_equal(eng.table.cols[col], want.cols[col]), (k, col)
    # a running pod carrying an anti-affinity term the pending web pod carries too: its entry exists
    inf.on_pod_add(pod("g2", {"app": "guard2"}, node_name="d", anti=[T(WEB, HOST)]), 8.0)
    assert not inf.flush(eng, 8.0).needs_reload
    # ... one on a new key: reload
    inf.on_pod_add(pod("g3", {"app": "guard3"}, node_name="d", anti=[T(WEB, "rack")]), 9.0)
    assert inf.delta(9.0)[2].needs_reload
    t = inf.table(9.0)
    assert len(t.ipa.ent_key) > len(eng.table.ipa.ent_key)
    x = inf.pod_ext_records(pending)
    assert x["ipa_anti"][0] != 0
