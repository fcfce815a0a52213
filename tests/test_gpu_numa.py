"""NodeNUMAResource on the GPU vs the oracle (bit-exact): the accumulator's
cpuset choice (reference KATs + randomized states), Filter/Score masks, and the
greedy stream with cpuset Reserves, Reserve failures and the final NUMA state."""
import json
import os

import numpy as np
import pytest

import oracle
import golden_cases as G
from koordinator_amd import abi, synth
from koordinator_amd.config import PLUGIN_FIT, PLUGIN_LOADAWARE, PLUGIN_NUMA, shipped_profile, to_c_config
from koordinator_amd.numa import (ClassTable, format_cpuset, linux_topology, parse_cpuset, reference_test_topology)
from koordinator_amd.snapshot import NodeTable, pod_array

pytestmark = pytest.mark.gpu

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "cpu_accumulator.json")))
POL = {"FullPCPUs": abi.CPUBIND_FULL_PCPUS, "SpreadByPCPUs": abi.CPUBIND_SPREAD_BY_PCPUS}
EXCL = {"None": abi.CPUEXCL_NONE, "PCPULevel": abi.CPUEXCL_PCPU, "NUMANodeLevel": abi.CPUEXCL_NUMA}


@pytest.fixture(scope="module")
def Engine():
    import torch  # noqa: F401
    from koordinator_amd.engine import PlacementEngine
    return PlacementEngine


def numa_table(topos, free, ep=None, en=None, flags=None, alloc_cnt=None):
    """A small snapshot, one node per entry of `topos`, with roomy Fit columns."""
    n = len(topos)
    t = NodeTable.empty(n)
    ct = ClassTable()
    for i, topo in enumerate(topos):
        t["numa_class"][i] = ct.add(topo) if topo is not None else -1
        t["alloc0"][i] = (topo.num_cpus if topo is not None else 64) * 1000
        for w in range(abi.NUMA_WORDS):
            t[f"numa_free{w}"][i] = free[i][w]
            if ep is not None:
                t[f"numa_excl_pcpu{w}"][i] = ep[i][w]
            if en is not None:
                t[f"numa_excl_numa{w}"][i] = en[i][w]
    t.numa_classes = ct.records()
    t["alloc1"][:] = 1 << 40
    t["alloc_pods"][:] = 1000
    t["la_alloc_cpu_m"][:] = t["alloc0"]
    t["la_alloc_mem"][:] = t["alloc1"]
    t["laf_total_m0"][:] = t["alloc0"]
    t["laf_total_m1"][:] = t["alloc1"] * 1000
    if flags is not None:
        t["numa_flags"][:] = flags
    if alloc_cnt is not None:
        t["numa_alloc_cnt"][:] = alloc_cnt
    return t


def cpuset_pod(need, required=0, preferred=abi.CPUBIND_FULL_PCPUS, excl=0):
    p = pod_array(1)
    p["req"][0, abi.RES_CPU] = need * 1000
    p["req"][0, abi.RES_MEM] = 1 << 30
    p["nz_cpu_m"] = need * 1000
    p["nz_mem"] = 1 << 30
    p["flags"] = abi.POD_PROD | abi.POD_HAS_REQ | abi.POD_CPUSET
    p["numa_cpus"] = need
    p["numa_policy"] = abi.numa_policy(required, preferred, excl)
    return p


@pytest.mark.parametrize("case", GOLDEN["take_cpus"], ids=[c["name"] for c in GOLDEN["take_cpus"]])
def test_gpu_accumulator_golden(Engine, case):
    topo = reference_test_topology(*case["topology"])
    allocated = parse_cpuset(case["allocated"])
    free = topo.mask([c for c in topo.cpu_of if c not in allocated])
    am = topo.mask(allocated)
    ae = case["allocated_exclusive_policy"]
    flags = abi.NODE_NUMA_MOST_ALLOCATED if case["strategy"] == "MostAllocated" else 0
    t = numa_table([topo], [free], ep=[am] if ae == "PCPULevel" else None, en=[am] if ae == "NUMANodeLevel" else None,
                   flags=flags, alloc_cnt=len(allocated))
    prof = shipped_profile(numa=True)
    pod = cpuset_pod(case["need"], preferred=POL[case["bind_policy"]], excl=EXCL[case["exclusive_policy"]])
    with Engine(prof, device=0) as e:
        e.load_snapshot(t)
        got = e.commit(pod[0], 0)
        st = e.read_numa()
    assert format_cpuset(topo.cpus(got)) == format_cpuset(parse_cpuset(case["want"])), case["source"]
    assert int(st["alloc_cnt"][0]) == len(allocated) + case["need"]
    assert np.array_equal(st["free"][:, 0], free & ~got)


def _random_nodes(rng, n, topos):
    tl, free, ep, en, flags, cnt = [], [], [], [], [], []
    for _ in range(n):
        topo = topos[rng.integers(len(topos))]
        cpc = topo.cpus_per_core
        used = rng.random(topo.num_cpus) < rng.random() * 0.7
        if rng.random() < 0.5:  # whole-core allocations
            used = np.repeat(used[::cpc], cpc)
        excl_p = used & (rng.random(topo.num_cpus) < 0.2)
        excl_n = used & ~excl_p & (rng.random(topo.num_cpus) < 0.2)
        pos = np.arange(topo.num_cpus)
        m = lambda sel: topo.mask([topo.cpu_of[p] for p in pos[sel]])
        tl.append(topo)
        free.append(m(~used))
        ep.append(m(excl_p))
        en.append(m(excl_n))
        flags.append(int(rng.integers(0, 3)) | (abi.NODE_NUMA_MOST_ALLOCATED if rng.random() < 0.5 else 0))
        cnt.append(int(used.sum()))
    return numa_table(tl, free, ep, en, np.array(flags, np.uint8), np.array(cnt, np.int32))


TOPOS = [linux_topology(2, 1, 8, 2), linux_topology(2, 2, 4, 2), reference_test_topology(2, 2, 4, 2),
         reference_test_topology(1, 2, 6, 1), linux_topology(2, 1, 24, 2)]


def test_gpu_accumulator_random_vs_oracle(Engine):
    rng = np.random.default_rng(11)
    t = _random_nodes(rng, 64, TOPOS)
    prof = shipped_profile(numa=True)
    cfg = to_c_config(prof)
    o = oracle.Oracle(cfg, t)
    pods = []
    for j in range(400):
        req = int(rng.integers(0, 3))
        pref = int(rng.integers(1, 3)) if req == 0 else req
        pods.append(cpuset_pod(int(rng.integers(1, 24)), req, pref, int(rng.integers(0, 3))))
    with Engine(prof, device=0) as e:
        e.load_snapshot(t)
        for j, p in enumerate(pods):
            node = j % t.n
            rc, want = o.commit(p[0], node)
            try:
                got = e.commit(p[0], node)
                grc = 0
            except abi.KoordhipError as ex:
                got, grc = np.zeros(abi.NUMA_WORDS, np.uint64), ex.code
            assert grc == rc, (j, node)
            if rc == 0:
                assert np.array_equal(got, want), (j, node)
        s, rs = e.read_numa(), o.numa_state()
    for k in ("free", "excl_pcpu", "excl_numa", "alloc_cnt"):
        assert np.array_equal(s[k], rs[k]), k


def test_gpu_numa_eval_parity(Engine):
    """Filter statuses / per-plugin scores / top-k with every policy mix, incl. the
    closed-form Allocate feasibility vs the oracle's literal accumulator."""
    rng = np.random.default_rng(5)
    t = _random_nodes(rng, 300, TOPOS)
    t["numa_class"][::37] = -1
    prof = shipped_profile(numa=True)
    cfg = to_c_config(prof)
    pods = pod_array(0)
    plist = []
    for j in range(48):
        req = j % 3
        pref = (j // 3) % 2 + 1 if req == 0 else req
        plist.append(cpuset_pod(int(rng.integers(1, 20)), req, pref, (j // 6) % 3))
    ls = synth.make_pods(synth.StreamSpec(16, be_frac=0.5), prof)
    pods = np.concatenate([np.concatenate(plist), ls])
    with Engine(prof, device=0) as e:
        e.load_snapshot(t)
        got = e.eval(pods, k=8)
    ref = oracle.Oracle(cfg, t).eval(pods, k=8)
    assert np.array_equal(got["status"], ref["status"])
    assert np.array_equal(got["topk"], ref["topk"])
    assert np.array_equal(got["scores"][:, :2], ref["scores"][:, :2])
    # the NUMA Score of a pair that fails the NUMA Filter is never computed by the
    # framework (koordhip.h: unspecified); every scored pair must match
    ok = (ref["status"] & abi.ST_NUMA_FAIL) == 0
    bad = np.argwhere(ok & (got["scores"][:, 2] != ref["scores"][:, 2]))
    assert len(bad) == 0, bad[:5]


@pytest.mark.parametrize("n_nodes,n_pods,batch,cpuset_frac,scoring", [
    (600, 1000, 0, 0.5, "LeastAllocated"), (300, 800, 17, 0.8, "LeastAllocated"),
    (2000, 1500, 64, 0.3, "LeastAllocated"),
    (600, 1000, 0, 0.5, "MostAllocated"),     # non-monotone score: M and M' re-evaluated for every pod
    (300, 800, 17, 0.8, "MostAllocated")])
def test_gpu_numa_stream_bit_exact(Engine, n_nodes, n_pods, batch, cpuset_frac, scoring):
    prof = shipped_profile(numa=True)
    prof.numa.scoring_type = scoring
    prof.batch_pods = batch
    table = synth.make_cluster(synth.ClusterSpec(n_nodes), prof)
    synth.add_numa(table, synth.NumaSpec(), prof)
    pods = synth.make_pods(synth.StreamSpec(n_pods, be_frac=0.2, cpuset_frac=cpuset_frac), prof)
    cfg = to_c_config(prof)
    with Engine(prof, device=0) as e:
        e.load_snapshot(table)
        got = e.place_stream(pods)
        cs = e.fetch_cpusets(len(pods))
        st, nst = e.read_nodes(), e.read_numa()
    o = oracle.Oracle(cfg, table)
    ref, rcs = o.place_stream(pods, cpusets=True)
    assert np.array_equal(got, ref), int(np.flatnonzero(got != ref)[0])
    assert np.array_equal(cs, rcs)
    rs, rn = o.state(), o.numa_state()
    for k in ("requested", "npods", "la_used"):
        assert np.array_equal(st[k], rs[k]), k
    for k in rn:
        assert np.array_equal(nst[k], rn[k]), k


def test_gpu_reserve_failure(Engine):
    """A preferred-policy cpuset pod passes Filter everywhere, the winner cannot
    allocate: -2, nothing committed (plugin.go:398-401); the next pod places."""
    topo = linux_topology(2, 1, 8, 2)
    few = topo.mask(topo.cpu_of[:2])
    t = numa_table([topo, topo], [few, few], alloc_cnt=np.array([30, 30], np.int32))
    prof = shipped_profile(numa=True)
    pods = np.concatenate([cpuset_pod(4), cpuset_pod(2), cpuset_pod(1)])
    cfg = to_c_config(prof)
    with Engine(prof, device=0) as e:
        e.load_snapshot(t)
        got = e.place_stream(pods)
        nst = e.read_numa()
    o = oracle.Oracle(cfg, t)
    ref = o.place_stream(pods)
    assert ref[0] == abi.RESERVE_FAILED
    assert np.array_equal(got, ref)
    for k, v in o.numa_state().items():
        assert np.array_equal(nst[k], v), k


@pytest.mark.parametrize("name,case", G.numa_score_cases(), ids=[c[0] for c in G.numa_score_cases()])
def test_gpu_numa_score_kat(Engine, name, case):
    """TestPlugin_Score (scoring_test.go:373-595) through libkoordhip.so."""
    prof, table, pod = G.build_numa_score_case(case)
    with Engine(prof, device=0) as e:
        e.load_snapshot(table)
        got = e.eval(pod)["scores"][0, 2, 0]
    assert got == case["want"], case["source"]


def test_gpu_accumulator_go118_socket_sort(Engine):
    """The device replay reproduces go 1.18's unstable sort.Slice on 7 tied sockets."""
    from test_numa_oracle import _seven_socket_case
    topo, free, want = _seven_socket_case()
    t = numa_table([topo], [topo.mask(free)], flags=abi.NODE_NUMA_MOST_ALLOCATED,
                   alloc_cnt=topo.num_cpus - len(free))
    prof = shipped_profile(numa=True)
    with Engine(prof, device=0) as e:
        e.load_snapshot(t)
        got = e.commit(cpuset_pod(8)[0], 0)
    assert topo.cpus(got) == want


def test_gpu_class_core_order_checked(Engine):
    """Positions inside a core must ascend by CPU id (the header's core-major
    rule, which the resolve's lane-parallel spread take relies on): a class
    whose first core lists its CPUs in descending id is rejected at load."""
    topo = linux_topology(1, 1, 4, 2)
    t = numa_table([topo], [topo.mask(topo.cpu_of)])
    recs = t.numa_classes.copy()
    a, b = int(recs[0]["cpu_id"][0]), int(recs[0]["cpu_id"][1])
    recs[0]["cpu_id"][0], recs[0]["cpu_id"][1] = b, a
    t.numa_classes = recs
    prof = shipped_profile(numa=True)
    with Engine(prof, device=0) as e:
        with pytest.raises(abi.KoordhipError, match="ascend by CPU id"):
            e.load_snapshot(t)
