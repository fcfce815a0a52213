"""HIP path vs the CPU oracle, through the C-ABI (libkoordhip.so) on a real
MI355X.  Integer/index outputs must be bit-exact: Filter masks, per-plugin
scores, top-k, greedy placements and the committed node state."""
import numpy as np
import pytest

import oracle
from koordinator_amd import abi, synth
from koordinator_amd.config import PLUGIN_FIT, PLUGIN_LOADAWARE, Profile, shipped_profile, to_c_config

import golden_cases as G

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def Engine():
    import torch  # noqa: F401  (device discovery only; the engine is plain HIP)
    from koordinator_amd.engine import PlacementEngine
    return PlacementEngine


def workload(n_nodes, n_pods, be=0.3, seed=synth.SEED, profile=None):
    prof = profile or shipped_profile()
    table = synth.make_cluster(synth.ClusterSpec(n_nodes, seed=seed), prof)
    pods = synth.make_pods(synth.StreamSpec(n_pods, be_frac=be, seed=seed), prof)
    return prof, table, pods


# ---------------------------------------------------------------- golden KATs
@pytest.mark.parametrize("name,case,node", G.score_cases(), ids=[c[0] for c in G.score_cases()])
def test_kat_loadaware_score_on_gpu(Engine, name, case, node):
    profile, table, rec = G.build_case(case, node)
    with Engine(profile, device=0) as e:
        e.load_snapshot(table)
        out = e.eval(rec)
    assert out["scores"][0, 1, 0] == case["want"], case["source"]


@pytest.mark.parametrize("name,case,node", G.filter_cases(), ids=[c[0] for c in G.filter_cases()])
def test_kat_loadaware_filter_on_gpu(Engine, name, case, node):
    profile, table, rec = G.build_case(case, node, test_pod_key="test_pod")
    with Engine(profile, device=0) as e:
        e.load_snapshot(table)
        out = e.eval(rec, scores=False)
    assert ((out["status"][0, 0] & abi.ST_LA_FAIL) == 0) == case["want_ok"], case["source"]


# ---------------------------------------------------------- eval parity
@pytest.mark.parametrize("n_nodes,n_pods,be", [(500, 40, 0.3), (1, 5, 0.5), (63, 7, 0.0), (4097, 70, 0.3)])
def test_eval_masks_scores_topk_bit_exact(Engine, n_nodes, n_pods, be):
    prof, table, pods = workload(n_nodes, n_pods, be)
    cfg = to_c_config(prof)
    with Engine(prof, device=0) as e:
        e.load_snapshot(table)
        got = e.eval(pods, k=16)
    ref = oracle.Oracle(cfg, table).eval(pods, k=16)
    assert np.array_equal(got["status"], ref["status"])
    assert np.array_equal(got["scores"], ref["scores"])
    assert np.array_equal(got["topk"]["node"], ref["topk"]["node"])
    assert np.array_equal(got["topk"]["score"], ref["topk"]["score"])


def test_eval_prod_usage_and_thresholds(Engine):
    """ScoreAccordingProdUsage + prod thresholds + raw-allocatable (la_alloc != alloc)."""
    prof = shipped_profile()
    prof.loadaware.score_according_prod_usage = True
    prof.loadaware.prod_usage_thresholds = {"cpu": 40, "memory": 90}
    table = synth.make_cluster(synth.ClusterSpec(777), prof)
    rng = np.random.default_rng(7)
    table["la_used_prod_cpu_m"][:] = (table["la_used_cpu_m"] * rng.uniform(0, 1, table.n)).astype(np.int64)
    table["la_used_prod_mem"][:] = (table["la_used_mem"] * rng.uniform(0, 1, table.n)).astype(np.int64)
    table["laf_prod_used_m0"][:] = table["la_used_prod_cpu_m"]
    table["laf_prod_used_m1"][:] = table["la_used_prod_mem"] * 1000
    table["la_flags"][:] |= np.where(rng.uniform(0, 1, table.n) < 0.7, abi.LA_HAS_PODS_METRIC, 0).astype(np.uint8)
    table["la_alloc_cpu_m"][:] = table["alloc0"] - 1000          # raw-allocatable override
    table["la_flags"][::13] |= abi.LA_SCORE_EXPIRED
    table["la_flags"][::17] |= abi.LA_FILTER_SKIP
    pods = synth.make_pods(synth.StreamSpec(50, be_frac=0.4), prof)
    pods["flags"][::5] |= abi.POD_DAEMONSET
    cfg = to_c_config(prof)
    with Engine(prof, device=0) as e:
        e.load_snapshot(table)
        got = e.eval(pods, k=8)
    ref = oracle.Oracle(cfg, table).eval(pods, k=8)
    for key in ("status", "scores"):
        assert np.array_equal(got[key], ref[key]), key
    assert np.array_equal(got["topk"], ref["topk"])


def test_eval_fit_edge_cases(Engine):
    """Over-committed nodes, zero requests, ephemeral storage, pod-count limit."""
    prof, table, pods = workload(300, 30, 0.3)
    table["requested0"][::7] = table["alloc0"][::7] + 5           # Requested > Allocatable
    table["requested1"][::11] = table["alloc1"][::11] + 1
    table["alloc2"][:] = 10 * 2**30
    table["requested2"][::5] = 11 * 2**30
    table["npods"][::9] = table["alloc_pods"][::9]                 # full
    pods["req"][::4, abi.RES_EPH] = 2**30
    pods["req"][1::6, abi.RES_CPU] = 0
    pods["flags"][2::8] &= ~np.uint32(abi.POD_HAS_REQ)
    prof.fit.resources["ephemeral-storage"] = 3
    cfg = to_c_config(prof)
    with Engine(prof, device=0) as e:
        e.load_snapshot(table)
        got = e.eval(pods, k=4)
    ref = oracle.Oracle(cfg, table).eval(pods, k=4)
    for key in ("status", "scores", "topk"):
        assert np.array_equal(got[key], ref[key]), key


# ------------------------------------------------------------ stream parity
@pytest.mark.parametrize("n_nodes,n_pods,be,batch", [
    (500, 1000, 0.0, 0),      # BASELINE config 1 (500 nodes x 1k pods)
    (500, 1000, 0.3, 64),
    (200, 700, 0.3, 1),
    (77, 500, 0.5, 17),       # pile-ups: more pods than nodes, unschedulable tail
    (3000, 1500, 0.3, 32),
])
def test_place_stream_bit_exact(Engine, n_nodes, n_pods, be, batch):
    prof, table, pods = workload(n_nodes, n_pods, be)
    prof.batch_pods = batch
    cfg = to_c_config(prof)
    with Engine(prof, device=0) as e:
        e.load_snapshot(table)
        got = e.place_stream(pods)
        state = e.read_nodes()
    o = oracle.Oracle(cfg, table)
    ref = o.place_stream(pods)
    assert np.array_equal(got, ref), int(np.flatnonzero(got != ref)[0])
    rs = o.state()
    for k in ("requested", "nz", "npods", "la_used", "la_used_prod"):
        assert np.array_equal(state[k], rs[k]), k


def test_place_stream_config2_subset(Engine):
    """BASELINE config 2 shape (5k nodes), first 3k pods of the 10k stream."""
    prof, table, pods = workload(5000, 3000, 0.0)
    cfg = to_c_config(prof)
    with Engine(prof, device=0) as e:
        e.load_snapshot(table)
        got = e.place_stream(pods)
    ref = oracle.Oracle(cfg, table).place_stream(pods, threads=8)
    assert np.array_equal(got, ref)


def test_empty_and_unschedulable(Engine):
    prof, table, pods = workload(10, 20, 0.0)
    table["alloc_pods"][:] = 0                     # every node full -> all unschedulable
    with Engine(prof, device=0) as e:
        e.load_snapshot(table)
        assert len(e.place_stream(pods[:0])) == 0
        got = e.place_stream(pods)
    assert (got == abi.UNSCHEDULABLE).all()


def test_commit_uncommit_and_update_nodes(Engine):
    prof, table, pods = workload(400, 64, 0.3)
    cfg = to_c_config(prof)
    o = oracle.Oracle(cfg, table)
    with Engine(prof, device=0) as e:
        e.load_snapshot(table)
        for j in range(20):
            e.commit(pods[j], j * 7 % 400)
            o.commit(pods[j], j * 7 % 400)
        e.uncommit(pods[3], 21)
        o.commit(pods[3], 21, -1)
        s = e.read_nodes()
        rs = o.state()
        for k in s:
            assert np.array_equal(s[k], rs[k]), k
        # informer delta: rewrite 50 rows (NodeMetric refresh), evaluate again
        idx = np.arange(0, 400, 8, dtype=np.int32)
        rows = table.rows(idx)
        rows["laf_used_m0"][:] = rows["laf_total_m0"] * 9 // 10   # now above the 65% cpu threshold
        for r in range(abi.NRES):   # the informer row carries the current NodeInfo accounting
            rows[f"requested{r}"][:] = s["requested"][r][idx]
        rows["nz_cpu_m"][:], rows["nz_mem"][:] = s["nz"][0][idx], s["nz"][1][idx]
        rows["npods"][:] = s["npods"][idx]
        rows["la_used_cpu_m"][:], rows["la_used_mem"][:] = s["la_used"][0][idx], s["la_used"][1][idx]
        rows["la_used_prod_cpu_m"][:] = s["la_used_prod"][0][idx]
        rows["la_used_prod_mem"][:] = s["la_used_prod"][1][idx]
        e.update_nodes(idx, rows)
        got = e.eval(pods[:16], k=8)
    t2 = table.copy()
    st = o.state()
    for r in range(abi.NRES):
        t2[f"requested{r}"][:] = st["requested"][r]
    t2["nz_cpu_m"][:], t2["nz_mem"][:] = st["nz"]
    t2["npods"][:] = st["npods"]
    t2["la_used_cpu_m"][:], t2["la_used_mem"][:] = st["la_used"]
    t2["la_used_prod_cpu_m"][:], t2["la_used_prod_mem"][:] = st["la_used_prod"]
    for c in rows.cols:
        t2[c][idx] = rows[c]
    ref = oracle.Oracle(cfg, t2).eval(pods[:16], k=8)
    for key in ("status", "scores", "topk"):
        assert np.array_equal(got[key], ref[key]), key
    has_metric = (rows["la_flags"] & abi.LA_HAS_METRIC) != 0   # missing NodeMetric -> Filter passes
    assert (got["status"][:, idx[has_metric]] & abi.ST_LA_FAIL).all()


def test_plugin_subsets(Engine):
    for filters, scores in [((PLUGIN_FIT,), {PLUGIN_FIT: 3}), ((PLUGIN_LOADAWARE,), {PLUGIN_LOADAWARE: 2}),
                            ((), {PLUGIN_FIT: 1, PLUGIN_LOADAWARE: 5})]:
        prof = shipped_profile()
        prof.filters = filters
        prof.scores = scores
        _, table, pods = workload(600, 300, 0.3, profile=prof)
        cfg = to_c_config(prof)
        with Engine(prof, device=0) as e:
            e.load_snapshot(table)
            got = e.place_stream(pods)
        ref = oracle.Oracle(cfg, table).place_stream(pods)
        assert np.array_equal(got, ref), (filters, scores)


# ------------------------------------------------- node-sharded groups (§8(e))
@pytest.mark.parametrize("world,n_nodes,n_pods,be,batch", [
    (2, 3000, 1500, 0.3, 0),
    (3, 1001, 800, 0.3, 32),
    (4, 77, 500, 0.5, 17),     # tiny shards, pile-ups, unschedulable tail
    (4, 3, 40, 0.3, 8),        # a shard with no nodes
])
def test_sharded_group_bit_exact(Engine, world, n_nodes, n_pods, be, batch):
    """Node-index shards evaluated by `world` contexts on one GPU, per-shard
    top-k exchanged by the local group (the RCCL path's layout and merge), then
    the replicated resolve: every rank must return the unsharded placements."""
    from koordinator_amd.engine import place_stream_group
    prof, table, pods = workload(n_nodes, n_pods, be)
    prof.batch_pods = batch
    cfg = to_c_config(prof)
    engines = [Engine(prof, device=0) for _ in range(world)]
    try:
        for e in engines:
            e.load_snapshot(table)
        Engine.comm_init_local(engines)
        outs = place_stream_group(engines, pods)
        states = [e.read_nodes() for e in engines]
    finally:
        for e in engines:
            e.close()
    o = oracle.Oracle(cfg, table)
    ref = o.place_stream(pods)
    for r in range(world):
        assert np.array_equal(outs[r], ref), (r, int(np.flatnonzero(outs[r] != ref)[0]))
    rs = o.state()
    for s in states:
        for k in ("requested", "npods", "la_used"):
            assert np.array_equal(s[k], rs[k]), k


@pytest.mark.parametrize("numa,n_nodes,n_pods", [(False, 3000, 1200), (True, 600, 700)])
def test_rccl_one_rank_exchange(Engine, numa, n_nodes, n_pods):
    """koordhip_comm_init with world 1: a real one-rank RCCL communicator, so
    every round goes through the multi-GPU exchange path on this GPU
    (ncclAllGather of the lists on the engine stream, k_topk_merge, the
    per-round list signal, the lag-1 persistent resolve over the merged lists)
    and must place exactly like the oracle."""
    prof = shipped_profile(numa=numa)
    table = synth.make_cluster(synth.ClusterSpec(n_nodes), prof)
    if numa:
        synth.add_numa(table, synth.NumaSpec(), prof)
    pods = synth.make_pods(synth.StreamSpec(n_pods, be_frac=0.3, cpuset_frac=0.4 if numa else 0.0), prof)
    with Engine(prof, device=0) as e:
        e.comm_init(Engine.comm_unique_id(), 1, 0)
        e.load_snapshot(table)
        got = e.place_stream(pods)
        again = e.place_stream(pods[: n_pods // 3])
    o = oracle.Oracle(to_c_config(prof), table)
    ref = o.place_stream(pods)
    assert np.array_equal(got, ref), int(np.flatnonzero(got != ref)[0])
    o2 = oracle.Oracle(to_c_config(prof), table)
    o2.place_stream(pods)
    ref2 = o2.place_stream(pods[: n_pods // 3])
    assert np.array_equal(again, ref2)


# ----------------------------------------------------------- launch modes
@pytest.mark.parametrize("mode", ["KOORDHIP_ROUND_LAUNCH", "KOORDHIP_SERIAL", "KOORDHIP_CU_RESERVE", "KOORDHIP_ONE_EVAL_STREAM", "KOORDHIP_NO_KEY_TABLES",
                                  "KOORDHIP_FOLD_WAIT", "KOORDHIP_SELECT_ONEWG", "KOORDHIP_LAG1",
                                  "KOORDHIP_TOPK_R=1", "KOORDHIP_SCAN_PPW=auto", "KOORDHIP_SCAN_PPW=3"])
@pytest.mark.parametrize("numa", [False, True])
def test_launch_modes_bit_exact(Engine, monkeypatch, mode, numa):
    """The per-round resolve launch (local groups), the single-stream
    profiling order and the opt-in pipeline knobs (CU-masked streams, the wait
    folded into the select, one select workgroup per pod) place exactly like
    the default persistent pipeline and the oracle."""
    name, _, val = mode.partition("=")
    monkeypatch.setenv(name, val or "1")
    prof = shipped_profile(numa=numa)
    prof.batch_pods = 16
    table = synth.make_cluster(synth.ClusterSpec(400), prof)
    if numa:
        synth.add_numa(table, synth.NumaSpec(), prof)
    pods = synth.make_pods(synth.StreamSpec(700, be_frac=0.3, cpuset_frac=0.4 if numa else 0.0), prof)
    with Engine(prof, device=0) as e:
        e.load_snapshot(table)
        got = e.place_stream(pods)
    ref = oracle.Oracle(to_c_config(prof), table).place_stream(pods)
    assert np.array_equal(got, ref), int(np.flatnonzero(got != ref)[0])


# ------------------------------------------- node-sharded rank on class lists
@pytest.mark.gpu
def test_shard_local_fallback_bit_exact(Engine, monkeypatch):
    """A rank of a node-sharded job whose batch the class-incremental lists
    cover evaluates the full replica without the per-round exchange (api.hip
    `local`: never slower than one GPU);
    KOORDHIP_SHARD_LOCAL_SIM takes that decision on one GPU.  The kernel stats
    report it (KSTAT_LOCAL) and the placements equal the oracle's."""
    from koordinator_amd import abi
    monkeypatch.setenv("KOORDHIP_SHARD_LOCAL_SIM", "1")
    prof = shipped_profile()
    table = synth.make_cluster(synth.ClusterSpec(3000), prof)
    pods = synth.make_pods(synth.StreamSpec(4000, be_frac=0.3), prof)
    with Engine(prof, device=0) as e:
        e.load_snapshot(table)
        got = e.place_stream(pods)
        ks = e.kernel_stats()
        names = e.kernel_names()
    assert int(ks["flags"]) & abi.KSTAT_LOCAL, ks
    assert names["eval"].startswith("kh::k_cls_run"), names
    ref = oracle.Oracle(to_c_config(prof), table).place_stream(pods)
    assert np.array_equal(got, ref), int(np.flatnonzero(got != ref)[0])


# ----------------------------------------------------- bench.py --gpus N's per-rank setup
@pytest.mark.parametrize("workload", ["config4", "config5"])
def test_torch_nccl_group_beside_library_comm(Engine, workload):
    """What every rank of `bench.py --gpus N` holds, on one GPU (world 1):
    torch's nccl process group (RCCL, its own streams) beside the library's
    communicator pair (`koordhip_comm_init` splits a second one for the second
    evaluation stream) and its three CU-masked queues (the
    hardware-queue budget).  The unique id travels by dist.broadcast as in
    bench.py; placements equal the oracle's, and torch's collectives still
    work after the persistent pipeline ran."""
    import socket
    import torch
    import torch.distributed as dist
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        resv = workload == "config5"
        prof = shipped_profile(numa=resv, reservation=resv)
        n, p = (3000, 3000) if resv else (4000, 6000)
        table = synth.make_cluster(synth.ClusterSpec(n), prof)
        if resv:
            synth.add_numa(table, synth.NumaSpec(), prof)
            synth.add_reservations(table, synth.ResvSpec())
        pods = synth.make_pods(synth.StreamSpec(p, be_frac=0.3, resv_match_frac=0.2 if resv else 0.0), prof)
        t = torch.tensor(list(Engine.comm_unique_id()), dtype=torch.uint8, device="cuda")
        dist.broadcast(t, 0)
        with Engine(prof, device=0) as e:
            e.comm_init(bytes(t.cpu().tolist()), 1, 0)
            e.load_snapshot(table)
            e.checkpoint()
            e.stage_pods(pods)
            e.restore()
            e.place_staged()
            dist.barrier()
            torch.cuda.synchronize()
            e.synchronize()
            got = e.fetch_placements(len(pods))
        x = torch.ones(4, device="cuda")
        dist.all_reduce(x)
        assert x.tolist() == [1.0] * 4
    finally:
        dist.destroy_process_group()
    ref = oracle.Oracle(to_c_config(prof), table).place_stream(pods, threads=8)
    assert np.array_equal(got, ref), int(np.flatnonzero(got != ref)[0])
