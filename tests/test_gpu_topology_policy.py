"""NUMA topology policies on the GPU vs the oracle (bit-exact): TestNUMANodeScore
through libkoordhip.so, Filter / Score / top-k on random policy nodes, and
greedy streams whose Reserves move zone allocations and cpusets."""
import numpy as np
import pytest

import golden_cases as G
import oracle
from koordinator_amd import abi, synth
from koordinator_amd.config import shipped_profile, to_c_config
from koordinator_amd.snapshot import pod_array

pytestmark = pytest.mark.gpu

GI = 1 << 30


@pytest.fixture(scope="module")
def Engine():
    import torch  # noqa: F401
    from koordinator_amd.engine import PlacementEngine
    return PlacementEngine


@pytest.mark.parametrize("name,case", G.numa_node_score_cases(), ids=[c[0] for c in G.numa_node_score_cases()])
def test_gpu_numa_node_score_kat(Engine, name, case):
    """TestNUMANodeScore (scoring_test.go:47-371)."""
    prof, table, pod = G.build_numa_node_score_case(case)
    with Engine(prof, device=0) as e:
        e.load_snapshot(table)
        r = e.eval(pod)
    assert not (r["status"][0] & abi.ST_NUMA_FAIL).any()
    assert r["scores"][0, 2].tolist() == case["want"]


def _policy_cluster(n, prof, policy_frac=0.8, seed=11):
    t = synth.make_cluster(synth.ClusterSpec(n, seed=seed), prof)
    synth.add_numa(t, synth.NumaSpec(policy_frac=policy_frac), prof, seed=seed)
    return t


def _mixed_pods(rng, n, prof):
    """non-cpuset pods of every size (small ones fit a zone, big ones need 2-4
    zones or fit nowhere), cpuset pods under every bind policy, skip pods"""
    plist = []
    for j in range(n):
        p = pod_array(1)
        kind = j % 4
        cpu = int(rng.choice([500, 2000, 8000, 20000, 40000, 70000]))
        mem = int(rng.choice([0, 1, 8, 32, 96, 200])) * GI
        if kind == 3:
            cpu = 0 if j % 8 == 3 else cpu  # memory-only pods: one hint list
        p["req"][0, abi.RES_CPU] = cpu
        p["req"][0, abi.RES_MEM] = mem
        p["nz_cpu_m"] = cpu or 100
        p["nz_mem"] = mem or 200 << 20
        p["flags"] = abi.POD_HAS_REQ | (abi.POD_PROD if j % 2 else 0)
        if kind == 1:  # cpuset
            need = max(1, cpu // 1000) if cpu else 2
            need = min(need, 40)
            p["req"][0, abi.RES_CPU] = need * 1000
            p["nz_cpu_m"] = need * 1000
            p["flags"] |= abi.POD_CPUSET
            p["numa_cpus"] = need
            req = (j // 4) % 3
            pref = (j // 12) % 2 + 1 if req == 0 else req
            p["numa_policy"] = abi.numa_policy(req, pref, (j // 8) % 3)
        if cpu == 0 and mem == 0:
            p["flags"] |= abi.POD_NUMA_SKIP
        plist.append(p)
    return np.concatenate(plist)


@pytest.mark.parametrize("scoring", ["LeastAllocated", "MostAllocated"])
def test_gpu_policy_eval_parity(Engine, scoring):
    rng = np.random.default_rng(21)
    prof = shipped_profile(numa=True)
    prof.numa.scoring_type = scoring
    t = _policy_cluster(400, prof)
    assert (t["numa_flags"] >> abi.NODE_NUMA_POLICY_SHIFT).any()
    pods = _mixed_pods(rng, 64, prof)
    with Engine(prof, device=0) as e:
        e.load_snapshot(t)
        got = e.eval(pods, k=8)
    ref = oracle.Oracle(to_c_config(prof), t).eval(pods, k=8)
    assert np.array_equal(got["status"], ref["status"])
    assert np.array_equal(got["topk"], ref["topk"])
    ok = (ref["status"] & abi.ST_NUMA_FAIL) == 0
    bad = np.argwhere(ok & (got["scores"][:, 2] != ref["scores"][:, 2]))
    assert len(bad) == 0, bad[:5]
    assert np.array_equal(got["scores"][:, :2], ref["scores"][:, :2])


@pytest.mark.parametrize("n_nodes,n_pods,batch,cpuset_frac,scoring", [
    (400, 800, 0, 0.4, "LeastAllocated"), (300, 600, 17, 0.7, "MostAllocated"), (1500, 1200, 64, 0.3, "LeastAllocated")])
def test_gpu_policy_stream_bit_exact(Engine, n_nodes, n_pods, batch, cpuset_frac, scoring):
    prof = shipped_profile(numa=True)
    prof.numa.scoring_type = scoring
    prof.batch_pods = batch
    table = _policy_cluster(n_nodes, prof, policy_frac=0.6, seed=n_nodes)
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
    assert rn["zone_used"].sum() != table["numa_zone_used"].sum()  # zone Reserves happened


def test_gpu_policy_commit_and_uncommit(Engine):
    """koordhip_commit on a policy node moves the zone amounts like the oracle's
    Reserve; Unreserve there is rejected (its zone amounts are not passed back)."""
    _, case = G.numa_node_score_cases()[4]
    prof, table, pod = G.build_numa_node_score_case(case)
    o = oracle.Oracle(to_c_config(prof), table)
    with Engine(prof, device=0) as e:
        e.load_snapshot(table)
        cpus = e.commit(pod, 1)
        nst = e.read_numa()
        with pytest.raises(abi.KoordhipError) as ei:
            e.uncommit(pod, 1, cpus)
        assert ei.value.code == abi.E_INVAL
    rc, rcpus = o.commit(pod, 1)
    assert rc == 0 and np.array_equal(cpus, rcpus)
    for k, v in o.numa_state().items():
        assert np.array_equal(nst[k], v), k


# ------------------------------------------------------------ CPU amplification
def _amp_cluster(n, prof, seed=5):
    t = synth.make_cluster(synth.ClusterSpec(n, seed=seed), prof)
    synth.add_numa(t, synth.NumaSpec(amp_frac=0.6), prof, seed=seed)
    return t


def test_gpu_amplified_eval_parity(Engine):
    """filterAmplifiedCPUs / scoreWithAmplifiedCPUs / amplified cpuset scores on
    random amplified nodes (ratios 1.25 / 1.5 / 2)."""
    rng = np.random.default_rng(33)
    prof = shipped_profile(numa=True)
    t = _amp_cluster(400, prof)
    assert (t["numa_amp_cpu"] > 1).sum() > 100
    pods = _mixed_pods(rng, 64, prof)
    with Engine(prof, device=0) as e:
        e.load_snapshot(t)
        got = e.eval(pods, k=8)
    ref = oracle.Oracle(to_c_config(prof), t).eval(pods, k=8)
    assert np.array_equal(got["status"], ref["status"])
    assert np.array_equal(got["topk"], ref["topk"])
    ok = (ref["status"] & abi.ST_NUMA_FAIL) == 0
    bad = np.argwhere(ok & (got["scores"][:, 2] != ref["scores"][:, 2]))
    assert len(bad) == 0, bad[:5]


@pytest.mark.parametrize("scoring", ["LeastAllocated", "MostAllocated"])
def test_gpu_amplified_stream_bit_exact(Engine, scoring):
    prof = shipped_profile(numa=True)
    prof.numa.scoring_type = scoring
    table = _amp_cluster(600, prof, seed=8)
    pods = synth.make_pods(synth.StreamSpec(1200, be_frac=0.2, cpuset_frac=0.5), prof)
    with Engine(prof, device=0) as e:
        e.load_snapshot(table)
        got = e.place_stream(pods)
        cs = e.fetch_cpusets(len(pods))
        st, nst = e.read_nodes(), e.read_numa()
    o = oracle.Oracle(to_c_config(prof), table)
    ref, rcs = o.place_stream(pods, cpusets=True)
    assert np.array_equal(got, ref), int(np.flatnonzero(got != ref)[0])
    assert np.array_equal(cs, rcs)
    for k, v in o.state().items():
        assert np.array_equal(st[k], v), k
    for k, v in o.numa_state().items():
        assert np.array_equal(nst[k], v), k


# ------------------------------------------- 8 NUMA zones (2-socket NPS4 hosts)
def _nps4_cluster(n, prof, seed):
    t = synth.make_cluster(synth.ClusterSpec(n, seed=seed), prof)
    synth.add_numa(t, synth.NumaSpec(policy_frac=0.8, nodes_per_socket=4), prof, seed=seed)
    assert (t.numa_classes["num_nodes"] == 8).all()
    pol = (t["numa_flags"] >> abi.NODE_NUMA_POLICY_SHIFT) & 3
    assert {1, 2, 3} <= set(pol.tolist())       # best-effort, restricted, single-numa-node all present
    return t


@pytest.mark.parametrize("scoring", ["LeastAllocated", "MostAllocated"])
def test_gpu_policy_eval_parity_8_zones(Engine, scoring):
    """Hint generation over 255 zone masks and the policy merges
    (frameworkext/topologymanager/policy.go:124-169, resource_manager.go:384-428)
    on 8-zone nodes: status, scores and top-k vs the oracle's literal merge."""
    rng = np.random.default_rng(41)
    prof = shipped_profile(numa=True)
    prof.numa.scoring_type = scoring
    t = _nps4_cluster(400, prof, seed=13)
    pods = _mixed_pods(rng, 64, prof)
    with Engine(prof, device=0) as e:
        e.load_snapshot(t)
        got = e.eval(pods, k=8)
    ref = oracle.Oracle(to_c_config(prof), t).eval(pods, k=8)
    assert np.array_equal(got["status"], ref["status"])
    assert np.array_equal(got["topk"], ref["topk"])
    ok = (ref["status"] & abi.ST_NUMA_FAIL) == 0
    bad = np.argwhere(ok & (got["scores"][:, 2] != ref["scores"][:, 2]))
    assert len(bad) == 0, bad[:5]


@pytest.mark.parametrize("n_nodes,n_pods,cpuset_frac,scoring", [
    (300, 500, 0.4, "LeastAllocated"), (400, 500, 0.6, "MostAllocated")])
def test_gpu_policy_stream_8_zones(Engine, n_nodes, n_pods, cpuset_frac, scoring):
    prof = shipped_profile(numa=True)
    prof.numa.scoring_type = scoring
    table = _nps4_cluster(n_nodes, prof, seed=n_nodes + 1)
    pods = synth.make_pods(synth.StreamSpec(n_pods, be_frac=0.2, cpuset_frac=cpuset_frac), prof)
    with Engine(prof, device=0) as e:
        e.load_snapshot(table)
        got = e.place_stream(pods)
        cs = e.fetch_cpusets(len(pods))
        nst = e.read_numa()
    o = oracle.Oracle(to_c_config(prof), table)
    # (the oracle merges hints literally: every permutation of the cpu and
    # memory hint lists, up to 255 x 255 per node on 8 zones -- 8 threads)
    ref, rcs = o.place_stream(pods, cpusets=True, threads=8)
    assert np.array_equal(got, ref), int(np.flatnonzero(got != ref)[0])
    assert np.array_equal(cs, rcs)
    for k, v in o.numa_state().items():
        assert np.array_equal(nst[k], v), k
    assert o.numa_state()["zone_used"][:, :, 4:].sum() != table["numa_zone_used"][:, :, 4:].sum()  # zones 4-7 used
