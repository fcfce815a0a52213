"""NodeNUMAResource's reservation restore: reservations holding a cpuset
(koordhip_node_soa.resv_cpus; nodenumaresource/reservation.go:68-122).

A cpuset pod nominated into a reservation (Reservation PreScore) sees the
reservation's reserved CPUs -- its cpuset less the CPUs of its assigned pods
(RestoreReservation, reservation.go:76-113) -- as preferred CPUs in the
NodeNUMAResource Score and Reserve (getResourceOptions, plugin.go:455-524):
they join the available CPUs, and takePreferredCPUs (cpu_accumulator.go:29-85)
takes them first.

Known answers:
  * TestRestoreReservation (plugin_test.go:1325-1428): a reservation holding
    CPUs 6-9 with pod-a (6,7) assigned restores 8,9; with pod-b (8,9) assigned
    too nothing is restored;
  * TestPlugin_Reserve "succeed allocate from reservation reserved cpus"
    (plugin_test.go:1044-1058): 2 sockets x 4 cores x 2 threads, the
    reservation holds 4-10, a 4-CPU FullPCPUs pod gets 4,5,6,7.
Random workloads (several reservations per node, a share holding cpusets, a
share of those partly taken by assigned pods, cpuset pods matching them)
compare the device's evaluation and greedy streams with the oracle bit for bit:
placements, cpusets, the NUMA state and every slot's reserved CPUs."""
import numpy as np
import pytest

import oracle
from koordinator_amd import abi, synth
from koordinator_amd import reservation as rv
from koordinator_amd.config import PLUGIN_NUMA, PLUGIN_RESERVATION, Profile, shipped_profile, to_c_config
from koordinator_amd.numa import ClassTable, format_cpuset, reference_test_topology
from koordinator_amd.snapshot import NodeTable, pod_array


def test_restore_reservation_kat():
    """TestRestoreReservation, plugin_test.go:1351-1427."""
    r = rv.Reservation("test-reservation", "test-node", cpus=[6, 7, 8, 9], assigned_cpus=[6, 7])
    assert r.reserved_cpus() == [8, 9]
    r.assigned_cpus += [8, 9]
    assert r.reserved_cpus() == []


def _reserve_case(reserved=(4, 5, 6, 7, 8, 9, 10), need=4):
    """TestPlugin_Reserve's reservation row (plugin_test.go:1044-1058, node
    setup :1062-1099): one node, topology buildCPUTopologyForTest(2, 1, 4, 2),
    the reservation's cpuset allocated with CPUExclusivePolicyNone."""
    prof = Profile(filters=(PLUGIN_NUMA, PLUGIN_RESERVATION), scores={PLUGIN_NUMA: 1, PLUGIN_RESERVATION: 5000})
    t = NodeTable.empty(1)
    t["alloc0"][0], t["alloc1"][0] = 96000, 512 * 2**30
    t["alloc_pods"][0] = 110
    t["la_alloc_cpu_m"][0], t["la_alloc_mem"][0] = t["alloc0"][0], t["alloc1"][0]
    topo = reference_test_topology(2, 1, 4, 2)
    ct = ClassTable()
    t["numa_class"][0] = ct.add(topo)
    t.numa_classes = ct.records()
    free = topo.mask([c for c in topo.cpu_of if c not in reserved])
    for w in range(abi.NUMA_WORDS):
        t[f"numa_free{w}"][0] = free[w]
    t["numa_alloc_cnt"][0] = len(reserved)
    # the reserve pod is a NodeInfo pod (Requested), its Allocatable = its cpuset
    cpu = 1000 * len(reserved)
    t["requested0"][0] = t["nz_cpu_m"][0] = cpu
    t["npods"][0] = 1
    t["resv_flags"][0] = abi.RESV_PRESENT | abi.RESV_KEY_CPU
    t["resv_alloc0"][0] = t["resv_nz0"][0] = cpu
    m = topo.mask(list(reserved))
    for w in range(abi.NUMA_WORDS):
        t[f"resv_cpus{w}"][0] = m[w]
    p = pod_array(1)
    p["req"][0, abi.RES_CPU] = need * 1000
    p["nz_cpu_m"][0] = need * 1000
    p["flags"][0] = abi.POD_CPUSET | abi.POD_HAS_REQ | abi.POD_PROD | abi.POD_KEY_CPU
    p["numa_cpus"][0] = need
    p["numa_policy"][0] = abi.numa_policy(0, 1, 0)   # preferred FullPCPUs
    p["resv_match"][0] = 1
    return prof, t, p, topo


def test_reserve_from_reserved_cpus_kat_oracle():
    prof, t, p, topo = _reserve_case()
    o = oracle.Oracle(to_c_config(prof), t)
    rc, cpus = o.commit(p, 0)
    assert rc == 0
    assert format_cpuset(topo.cpus(cpus)) == "4-7"
    left = o.resv_state()["cpus"][:, 0]
    assert format_cpuset(topo.cpus(left)) == "8-10"
    # the preferred CPUs were allocated already: the allocated count stays
    assert o.numa_state()["alloc_cnt"][0] == 7


def test_reserve_without_reserved_cpus_takes_free_ones_oracle():
    """The same pod with the reservation's CPUs not restored (its Reserve
    nominates nothing: the reservation does not match) takes free CPUs."""
    prof, t, p, topo = _reserve_case()
    p["resv_match"][0] = 0
    o = oracle.Oracle(to_c_config(prof), t)
    rc, cpus = o.commit(p, 0)
    assert rc == 0 and not set(topo.cpus(cpus)) & set(range(4, 11))


def _workload(n, pods, seed=5, slots=2, cpuset=0.5, match=0.7):
    prof = shipped_profile(numa=True, reservation=True)
    t = synth.make_cluster(synth.ClusterSpec(n, seed=seed), prof)
    synth.add_numa(t, synth.NumaSpec(), prof, seed=seed)
    synth.add_reservations(t, synth.ResvSpec(node_frac=0.5, groups=2, ordered_frac=0.1, slots=slots,
                                             multi_frac=0.5, allocate_once_frac=0.2), seed=seed)
    synth.add_reserved_cpus(t, frac=0.7, seed=seed)
    p = synth.make_pods(synth.StreamSpec(pods, be_frac=0.2, seed=seed, cpuset_frac=cpuset, resv_match_frac=match,
                                         resv_groups=2), prof)
    return prof, t, p


def _resv_cpu_masks(t):
    return np.stack([np.concatenate([t[f"resv_cpus{w}" + (f"@{q}" if q else "")] for q in range(t.resv_slots)])
                     for w in range(abi.NUMA_WORDS)])


def test_synth_reserved_cpus_are_allocated():
    _, t, _ = _workload(600, 10)
    m = _resv_cpu_masks(t)
    assert (m != 0).any(axis=0).sum() > 50
    n = t.n
    for q in range(t.resv_slots):
        for w in range(abi.NUMA_WORDS):
            assert not (m[w, q * n:(q + 1) * n] & t[f"numa_free{w}"]).any()
    # the soa carries them (and drops them when every mask is zero)
    assert t.as_soa().resv_cpus[0]
    z = t.copy()
    for c in list(z.cols):
        if c.startswith("resv_cpus"):
            z[c][:] = 0
    assert not z.as_soa().resv_cpus[0]


def test_oracle_stream_takes_reserved_cpus():
    """Pods nominated into CPU-holding reservations get their CPUs from them."""
    prof, t, pods = _workload(400, 600)
    before = _resv_cpu_masks(t)
    o = oracle.Oracle(to_c_config(prof), t)
    o.place_stream(pods, threads=4)
    after = o.resv_state()["cpus"]
    assert (after != before).any(axis=0).sum() > 10
    assert not (after & ~before).any()   # reserved CPUs only ever shrink


@pytest.fixture(scope="module")
def Engine():
    import torch  # noqa: F401
    from koordinator_amd.engine import PlacementEngine
    return PlacementEngine


@pytest.mark.gpu
def test_reserve_from_reserved_cpus_kat_gpu(Engine):
    prof, t, p, topo = _reserve_case()
    with Engine(prof, device=0) as e:
        e.load_snapshot(t)
        cpus = e.commit(p, 0)
        left = e.read_reservations()["cpus"][:, 0]
        cnt = e.read_numa()["alloc_cnt"][0]
    assert format_cpuset(topo.cpus(cpus)) == "4-7"
    assert format_cpuset(topo.cpus(left)) == "8-10"
    assert cnt == 7


@pytest.mark.gpu
def test_gpu_resv_cpus_eval_parity(Engine):
    prof, t, pods = _workload(1500, 48)
    ref = oracle.Oracle(to_c_config(prof), t).eval(pods, k=16)
    with Engine(prof, device=0) as e:
        e.load_snapshot(t)
        got = e.eval(pods, k=16)
    assert np.array_equal(ref["status"], got["status"])
    # the NodeNUMAResource score of a pair failing the NUMA Filter is unspecified
    # (include/koordhip.h koordhip_eval: the framework never scores such a node)
    live = (ref["status"] & abi.ST_NUMA_FAIL) == 0
    for pl in range(abi.NPLUGINS):
        a, b = ref["scores"][:, pl], got["scores"][:, pl]
        assert np.array_equal(a[live], b[live]) if pl == 2 else np.array_equal(a, b), pl
    assert np.array_equal(ref["topk"], got["topk"])


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["fused", "split"])
def test_gpu_resv_cpus_stream_parity(Engine, mode, monkeypatch):
    if mode == "split":
        monkeypatch.setenv("KOORDHIP_EVAL", "split")
    prof, t, pods = _workload(2500, 2000)
    o = oracle.Oracle(to_c_config(prof), t)
    ref, cs_ref = o.place_stream(pods, threads=8, cpusets=True)
    with Engine(prof, device=0) as e:
        e.load_snapshot(t)
        got = e.place_stream(pods)
        assert np.array_equal(ref, got), np.flatnonzero(ref != got)[:10]
        assert np.array_equal(e.fetch_cpusets(len(pods)), cs_ref)
        gr, rr = e.read_reservations(), o.resv_state()
        for k in ("allocated", "assigned", "cpus"):
            assert np.array_equal(gr[k], rr[k]), k
        gn, rn = e.read_numa(), o.numa_state()
        for k in rn:
            assert np.array_equal(gn[k], rn[k]), k
    assert (rr["cpus"] != _resv_cpu_masks(t)).any(axis=0).sum() > 10


@pytest.mark.gpu
def test_gpu_resv_cpus_config5_variant(Engine):
    """A config-5-shaped variant at reduced size (20k nodes x 4k pods, the
    shipped profile with NodeNUMAResource + Reservation): up to 2 reservations
    per node, 70 % of them holding a cpuset, half the LS pods cpuset pods;
    placements, cpusets and every state column bit-exact vs the oracle."""
    prof, t, pods = _workload(20000, 4000, seed=9)
    o = oracle.Oracle(to_c_config(prof), t)
    ref, cs_ref = o.place_stream(pods, threads=16, cpusets=True)
    with Engine(prof, device=0) as e:
        e.load_snapshot(t)
        got = e.place_stream(pods)
        assert np.array_equal(ref, got), np.flatnonzero(ref != got)[:10]
        assert np.array_equal(e.fetch_cpusets(len(pods)), cs_ref)
        gr, rr = e.read_reservations(), o.resv_state()
        for k in ("allocated", "assigned", "cpus"):
            assert np.array_equal(gr[k], rr[k]), k
        gs, rs = e.read_nodes(), o.state()
        for k in ("requested", "nz", "npods", "la_used"):
            assert np.array_equal(gs[k], rs[k]), k
    assert (rr["cpus"] != _resv_cpu_masks(t)).any(axis=0).sum() > 50


@pytest.mark.gpu
def test_gpu_resv_cpus_update_nodes(Engine):
    """koordhip_update_nodes replaces a row's reserved CPUs with the rows' own
    (clearing them when the rows carry none): a stream after the update
    matches the oracle on the updated table."""
    prof, t, pods = _workload(1500, 800, seed=13)
    t2 = t.copy()
    rng = np.random.default_rng(2)
    has = np.flatnonzero(_resv_cpu_masks(t).any(axis=0)[:t.n])
    idx = np.sort(rng.choice(has, size=min(60, len(has)), replace=False))
    # half of them: the reservation's CPUs all went to assigned pods (nothing restored)
    for i in idx[::2]:
        for w in range(abi.NUMA_WORDS):
            t2[f"resv_cpus{w}"][i] = 0
    ref = oracle.Oracle(to_c_config(prof), t2).place_stream(pods, threads=8)
    with Engine(prof, device=0) as e:
        e.load_snapshot(t)
        e.update_nodes(idx, t2.rows(idx))
        got = e.place_stream(pods)
    assert np.array_equal(ref, got), np.flatnonzero(ref != got)[:10]
    # rows carrying no reserved CPUs at all clear them
    rows = t.rows(idx[:4])
    for c in list(rows.cols):
        if c.startswith("resv_cpus"):
            rows[c][:] = 0
    assert not rows.as_soa().resv_cpus[0]
    with Engine(prof, device=0) as e:
        e.load_snapshot(t)
        e.update_nodes(idx[:4], rows)
        left = e.read_reservations()["cpus"]
    n = t.n
    for q in range(t.resv_slots):
        assert not left[:, q * n + idx[:4]].any()


def _two_node_case():
    """_reserve_case's node twice: two feasible nodes, so PreScore runs."""
    from koordinator_amd.snapshot import concat
    prof, t, p, topo = _reserve_case()
    t2 = concat([t, t.copy()])
    return prof, t2, p, topo


def test_single_feasible_node_skips_the_nomination_oracle():
    """(upstream) schedulePod returns the only feasible node without
    prioritizeNodes, so no reservation is nominated before the NUMA Reserve:
    the pod takes free CPUs (the Reservation Reserve still assumes it into the
    reservation).  With two feasible nodes PreScore nominates and the pod gets
    the reserved 4-7."""
    prof, t, p, topo = _reserve_case()
    o = oracle.Oracle(to_c_config(prof), t)
    node, cs = o.place_stream(p, cpusets=True)
    assert node[0] == 0 and not set(topo.cpus(cs[0])) & set(range(4, 11))
    assert o.resv_state()["assigned"][0] == 1
    prof, t2, p, topo = _two_node_case()
    node, cs = oracle.Oracle(to_c_config(prof), t2).place_stream(p, cpusets=True)
    assert node[0] == 0 and format_cpuset(topo.cpus(cs[0])) == "4-7"


@pytest.mark.gpu
def test_gpu_single_feasible_node_skips_the_nomination(Engine):
    for case in (_reserve_case, _two_node_case):
        prof, t, p, topo = case()
        ref_node, ref_cs = oracle.Oracle(to_c_config(prof), t).place_stream(p, cpusets=True)
        with Engine(prof, device=0) as e:
            e.load_snapshot(t)
            got = e.place_stream(p)
            cs = e.fetch_cpusets(1)
        assert np.array_equal(got, ref_node) and np.array_equal(cs, ref_cs), case.__name__


@pytest.mark.gpu
def test_gpu_resv_cpus_checkpoint_restore(Engine):
    """koordhip_checkpoint / koordhip_restore roll the reserved CPUs back with
    the other mutable columns: a restored second pass repeats the first."""
    prof, t, pods = _workload(2000, 1500, seed=17)
    with Engine(prof, device=0) as e:
        e.load_snapshot(t)
        e.checkpoint()
        e.stage_pods(pods)
        e.place_staged()
        a = e.fetch_placements(len(pods))
        ra = e.read_reservations()
        e.restore()
        assert np.array_equal(e.read_reservations()["cpus"], _resv_cpu_masks(t))
        e.place_staged()
        b = e.fetch_placements(len(pods))
        rb = e.read_reservations()
    assert np.array_equal(a, b)
    for k in ("allocated", "assigned", "cpus"):
        assert np.array_equal(ra[k], rb[k]), k
    assert (ra["cpus"] != _resv_cpu_masks(t)).any()
