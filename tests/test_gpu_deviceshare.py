"""DeviceShare and the normalized upstream Scores through libkoordhip.so's
exact sequential cycle (seq.hip) against the oracle (oracle/dev_oracle.c,
the reference cycle with DefaultNormalizeScore over the feasible list):
eval_ext planes / status / top-k, and greedy streams -- placements, device
allocations, deviceUsed, the extended scalars' Requested and the node state
-- bit for bit, beside Fit / LoadAware / NodeNUMAResource / Reservation."""
import numpy as np
import pytest

import oracle
from koordinator_amd import abi, synth
from koordinator_amd.config import shipped_profile, to_c_config, with_deviceshare, with_normalized_scores

pytestmark = pytest.mark.gpu


def _cluster(n, prof, numa=False, resv=False, seed=synth.SEED, gpu_frac=0.3):
    t = synth.make_cluster(synth.ClusterSpec(n, seed=seed), prof)
    if numa:
        synth.add_numa(t, synth.NumaSpec(), prof, seed=seed)
    if resv:
        synth.add_reservations(t, synth.ResvSpec(), seed=seed)
    synth.add_devices(t, synth.DevSpec(gpu_frac=gpu_frac), seed=seed)
    return t


def _pods(n, prof, seed=synth.SEED, cpuset=0.0, resv_match=0.0, dev_frac=0.25):
    pods = synth.make_pods(synth.StreamSpec(n, be_frac=0.3, seed=seed, cpuset_frac=cpuset,
                                            resv_match_frac=resv_match), prof)
    ext = synth.make_device_ext(n, synth.DevStreamSpec(frac=dev_frac, seed=seed))
    return pods, ext


def _static_scores(t, pods, seed=3):
    """Random NodeAffinity / TaintToleration raw scores per (static class, node)."""
    rng = np.random.default_rng(seed)
    ncls = 6
    pods["static_class"] = rng.integers(0, ncls, len(pods))
    ss = t["static_score"]
    ss[:, 0, :ncls] = rng.choice([0, 0, 10, 30, 60, 100], size=(t.n, ncls))
    ss[:, 1, :ncls] = rng.choice([0, 0, 0, 1, 2], size=(t.n, ncls))


def _engine(prof):
    import torch  # noqa: F401
    from koordinator_amd.engine import PlacementEngine
    return PlacementEngine(prof, device=0)


def _compare_stream(prof, t, pods, ext, cpusets=False, names=False):
    with _engine(prof) as e:
        e.load_snapshot(t)
        got = e.place_stream_ext(pods, ext)
        kn = e.kernel_names()
        gdev = e.fetch_devices(len(pods))
        gst = e.read_nodes()
        gdv = e.read_devices()
        gcs = e.fetch_cpusets(len(pods)) if cpusets else None
    o = oracle.Oracle(to_c_config(prof), t)
    res = o.place_stream_ext(pods, ext, cpusets=cpusets, devices=True)
    ref, rcs, rdev = (res[0], res[1], res[2]) if cpusets else (res[0], None, res[1])
    bad = np.flatnonzero(got != ref)
    assert bad.size == 0, f"first mismatch at pod {bad[0]}: hip {got[bad[0]]} oracle {ref[bad[0]]}"
    assert np.array_equal(gdev, rdev)
    ost = o.state()
    for k in ("requested", "nz", "npods", "la_used"):
        assert np.array_equal(gst[k], ost[k]), k
    ods = o.dev_state()
    if t.dev_slots:
        assert np.array_equal(gdv["dev_used"], ods["dev_used"])
    assert np.array_equal(gdv["xrequested"], ods["xrequested"])
    if cpusets:
        assert np.array_equal(gcs, rcs)
    return (got, kn) if names else got


def test_eval_ext_parity_deviceshare():
    prof = with_deviceshare(shipped_profile())
    t = _cluster(700, prof)
    pods, ext = _pods(48, prof, dev_frac=0.5)
    with _engine(prof) as e:
        e.load_snapshot(t)
        g = e.eval_ext(pods, ext, k=8)
    r = oracle.Oracle(to_c_config(prof), t).eval_ext(pods, ext, k=8)
    assert np.array_equal(g["status"], r["status"])
    assert np.array_equal(g["scores"], r["scores"])
    assert np.array_equal(g["topk"], r["topk"])


@pytest.mark.parametrize("route", ["pipelined", "sequential"])
@pytest.mark.parametrize("seed", [1, 2])
def test_stream_deviceshare_fit_loadaware(seed, route, monkeypatch):
    """Device pods among plain pods: placed inside the pipelined greedy (the
    resolve hands each one to k_ext_worker on the exact state), or the whole
    batch in the sequential cycle (KOORDHIP_EXT_SEQ) -- the same placements."""
    if route == "sequential":
        monkeypatch.setenv("KOORDHIP_EXT_SEQ", "1")
    prof = with_deviceshare(shipped_profile())
    t = _cluster(1500, prof, seed=synth.SEED + seed)
    pods, ext = _pods(2500, prof, seed=synth.SEED + seed)
    got, kn = _compare_stream(prof, t, pods, ext, names=True)
    assert ("k_resolve" in kn["resolve"]) == (route == "pipelined"), kn
    dev = (ext["flags"] & abi.PODX_DEVICE) != 0
    assert (got[dev] >= 0).sum() > 50   # device pods do land (and take devices)


@pytest.mark.parametrize("mode", ["default", "lag1_split", "one_stream"])
def test_stream_device_pods_in_pipeline_low_fraction(mode, monkeypatch):
    """config4dsmix's shape at test size: 2 % device pods among plain pods (the
    class lists on), plus the lag-1 split-select and one-evaluation-stream
    pipelines; placements, device slots, deviceUsed, the extended scalars and
    the node rows bit-exact with the oracle."""
    if mode == "lag1_split":
        monkeypatch.setenv("KOORDHIP_LAG1", "1")
        monkeypatch.setenv("KOORDHIP_CLS_OFF", "1")
    elif mode == "one_stream":
        monkeypatch.setenv("KOORDHIP_ONE_EVAL_STREAM", "1")
    prof = with_deviceshare(shipped_profile())
    t = _cluster(3000, prof, seed=synth.SEED + 11)
    pods, ext = _pods(6000, prof, seed=synth.SEED + 11, dev_frac=0.02)
    got, kn = _compare_stream(prof, t, pods, ext, names=True)
    assert "k_resolve" in kn["resolve"], kn
    dev = (ext["flags"] & abi.PODX_DEVICE) != 0
    assert dev.sum() > 60 and (got[dev] >= 0).sum() > 30


def test_stream_device_pods_in_pipeline_edge_cases():
    """Every pod a device pod, runs of consecutive device pods, device pods at
    round starts / ends, extended-scalar-only pods (xmask without a device
    request) and device pods no node can take (UNSCHEDULABLE)."""
    prof = with_deviceshare(shipped_profile())
    t = _cluster(800, prof, seed=synth.SEED + 13, gpu_frac=0.2)
    # all device pods: the worker places every pod
    pods, ext = _pods(400, prof, seed=synth.SEED + 13, dev_frac=1.0)
    _compare_stream(prof, t, pods, ext)
    # runs and round boundaries (24-pod rounds), xmask-only pods, oversized requests
    pods, ext = _pods(1200, prof, seed=synth.SEED + 14, dev_frac=0.0)
    _, full = _pods(1200, prof, seed=synth.SEED + 15, dev_frac=1.0)
    sel = np.zeros(1200, bool)
    sel[[0, 23, 24, 25, 26, 47, 95, 96, 500]] = True
    sel[600:640] = True                       # a run over two round boundaries
    sel[np.arange(700, 1200, 37)] = True
    ext[sel] = full[sel]
    xonly = np.flatnonzero(sel)[::5]
    ext["flags"][xonly] = 0                    # extended scalars only: the Fit of xrequested
    ext["dev_req"][xonly] = 0
    big = np.flatnonzero(sel)[1::7]
    ext["dev_req"][big, abi.DEV_GPU, 0] = 800  # eight whole GPUs: fits only the 8-GPU nodes' free ones
    ext["dev_req"][big, abi.DEV_GPU, 1] = 800
    got, kn = _compare_stream(prof, t, pods, ext, names=True)
    assert "k_resolve" in kn["resolve"], kn


def test_stream_deviceshare_most_allocated():
    prof = with_deviceshare(shipped_profile())
    prof.deviceshare.scoring_type = "MostAllocated"
    prof.deviceshare.resources = {"koordinator.sh/gpu-core": 1, "koordinator.sh/gpu-memory-ratio": 2,
                                  "koordinator.sh/rdma": 1}
    t = _cluster(900, prof, seed=synth.SEED + 5)
    pods, ext = _pods(1500, prof, seed=synth.SEED + 5)
    _compare_stream(prof, t, pods, ext)


def test_stream_deviceshare_numa_reservation():
    """DeviceShare (weight 1) beside Fit, LoadAware, NodeNUMAResource (cpuset
    pods) and Reservation (weight 5000): the shipped koord-scheduler profile."""
    prof = with_deviceshare(shipped_profile(numa=True, reservation=True))
    t = _cluster(1200, prof, numa=True, resv=True, seed=synth.SEED + 7)
    pods, ext = _pods(1500, prof, seed=synth.SEED + 7, cpuset=0.3, resv_match=0.2)
    _compare_stream(prof, t, pods, ext, cpusets=True)


def test_stream_normalized_upstream_scores():
    """NodeAffinity (preferred terms) and TaintToleration (PreferNoSchedule)
    Scores, normalized over the feasible nodes (TaintToleration reversed)."""
    prof = with_normalized_scores(shipped_profile(), affinity=2, taint=1)
    t = synth.make_cluster(synth.ClusterSpec(1000, seed=synth.SEED + 11), prof)
    t.enable_ext(0)
    pods = synth.make_pods(synth.StreamSpec(1500, be_frac=0.3, seed=synth.SEED + 11), prof)
    _static_scores(t, pods)
    _compare_stream(prof, t, pods, None)
    with _engine(prof) as e:
        e.load_snapshot(t)
        g = e.eval_ext(pods[:32], None, k=6)
    r = oracle.Oracle(to_c_config(prof), t).eval_ext(pods[:32], None, k=6)
    for k in ("status", "scores", "topk"):
        assert np.array_equal(g[k], r[k]), k


def test_stream_everything_normalized():
    """DeviceShare + NodeAffinity + TaintToleration Scores + NUMA in one profile."""
    prof = with_normalized_scores(with_deviceshare(shipped_profile(numa=True), weight=3), affinity=1, taint=2)
    t = _cluster(800, prof, numa=True, seed=synth.SEED + 13)
    pods, ext = _pods(1200, prof, seed=synth.SEED + 13, cpuset=0.3)
    _static_scores(t, pods, seed=5)
    _compare_stream(prof, t, pods, ext, cpusets=True)


def test_update_nodes_device_rows_then_stream():
    """koordhip_update_nodes of device rows (a Device CR / pod allocation
    event), then a stream: equal to the oracle on the updated table."""
    prof = with_deviceshare(shipped_profile())
    t = _cluster(600, prof, seed=synth.SEED + 17)
    pods, ext = _pods(800, prof, seed=synth.SEED + 17)
    rng = np.random.default_rng(4)
    idx = np.sort(rng.choice(t.n, 60, replace=False)).astype(np.int32)
    with _engine(prof) as e:
        e.load_snapshot(t)
        t2 = t.copy()
        t2["dev_used"][idx] = 0                       # pods holding devices finished
        t2["xrequested"][idx] = 0
        t2["dev_present"][idx[:10]] = 1 - t2["dev_present"][idx[:10]]
        e.update_nodes(idx, t2.rows(idx))
        got = e.place_stream_ext(pods, ext)
    ref = oracle.Oracle(to_c_config(prof), t2).place_stream_ext(pods, ext)
    assert np.array_equal(got, ref)


def test_checkpoint_restore_devices():
    """The sequential cycle's mutable columns (deviceUsed, extended scalars)
    roll back with koordhip_restore: two steps from one snapshot agree."""
    prof = with_deviceshare(shipped_profile())
    t = _cluster(500, prof, seed=synth.SEED + 19)
    pods, ext = _pods(600, prof, seed=synth.SEED + 19)
    with _engine(prof) as e:
        e.load_snapshot(t)
        e.checkpoint()
        a = e.place_stream_ext(pods, ext)
        da = e.read_devices()
        e.restore()
        b = e.place_stream_ext(pods, ext)
        db = e.read_devices()
    assert np.array_equal(a, b)
    assert np.array_equal(da["dev_used"], db["dev_used"])
    assert np.array_equal(da["xrequested"], db["xrequested"])


@pytest.mark.parametrize("numa", [False, True])
def test_stream_static_filters_and_scores(numa):
    """The upstream static filters (static_allow) with the NodeAffinity /
    TaintToleration Scores of the same classes (synth.add_static: preferred
    terms, PreferNoSchedule taints), BalancedAllocation and DeviceShare."""
    from koordinator_amd.config import with_upstream
    prof = with_normalized_scores(with_deviceshare(with_upstream(shipped_profile(numa=numa), balanced_weight=2)),
                                  affinity=3, taint=2)
    t = _cluster(1500, prof, numa=numa, seed=synth.SEED + 23)
    pods, ext = _pods(2000, prof, seed=synth.SEED + 23, cpuset=0.3 if numa else 0.0)
    synth.add_static(t, pods, synth.StaticSpec(), prof, seed=synth.SEED + 23)
    assert t["static_score"][:, 0].any() and t["static_score"][:, 1].any()
    got = _compare_stream(prof, t, pods, ext, cpusets=numa)
    ok = got >= 0
    cls = pods["static_class"][ok].astype(np.uint32)
    assert (((t["static_allow"][got[ok]] >> cls) & 1) == 1).all()


@pytest.mark.gpu
@pytest.mark.parametrize("numa_resv", [False, True])
def test_deviceshare_profile_batch_without_devices_runs_pipelined(numa_resv):
    """The shipped profile enables DeviceShare; a batch in which no pod
    requests a device (PreFilter skip for every pod: Filter passes, Score 0 on
    every node so its normalisation is 0, no Reserve; deviceshare/plugin.go:
    162-182, scoring.go:33-40) runs on the pipelined greedy, bit-exact with the
    oracle's sequential cycle; the next batch with device pods runs the
    sequential cycle on the state the first left."""
    prof = with_deviceshare(shipped_profile(numa=numa_resv, reservation=numa_resv))
    t = _cluster(4000, prof, numa=numa_resv, resv=numa_resv, seed=31)
    pods, _ = _pods(1500, prof, seed=32, resv_match=0.2 if numa_resv else 0.0)
    none = abi.pod_ext_array(len(pods))
    pods2, ext2 = _pods(600, prof, seed=33, dev_frac=0.3)
    o = oracle.Oracle(to_c_config(prof), t)
    ref1 = o.place_stream_ext(pods, none)
    ref2 = o.place_stream_ext(pods2, ext2)
    with _engine(prof) as e:
        e.load_snapshot(t)
        got1 = e.place_stream_ext(pods, none)
        k1 = e.kernel_names()["resolve"]
        got2 = e.place_stream_ext(pods2, ext2)
        k2 = e.kernel_names()["resolve"]
        gst = e.read_nodes()
        # the device batch: inside the pipeline on the plain build (k_ext_worker),
        # the sequential cycle beside NodeNUMAResource / Reservation
        assert "k_resolve" in k1 and ("k_seq" in k2) == numa_resv, (k1, k2)
    assert np.array_equal(got1, ref1), np.flatnonzero(got1 != ref1)[:10]
    assert np.array_equal(got2, ref2), np.flatnonzero(got2 != ref2)[:10]
    ost = o.state()
    for k in ("requested", "npods"):
        assert np.array_equal(gst[k], ost[k]), k


@pytest.mark.gpu
def test_fetch_devices_after_pipelined_batch_is_zero():
    """A device batch runs the sequential cycle and fills the device slots;
    the next batch, without device requests, runs pipelined and allocates no
    device: koordhip_fetch_devices must then return zeros, not the previous
    batch's slots (the bind loop would annotate phantom GPU minors)."""
    prof = with_deviceshare(shipped_profile())
    t = _cluster(2000, prof, seed=51)
    pods1, ext1 = _pods(400, prof, seed=52, dev_frac=0.5)
    pods2, _ = _pods(400, prof, seed=53)
    none = abi.pod_ext_array(len(pods2))
    o = oracle.Oracle(to_c_config(prof), t)
    ref1, dref1 = o.place_stream_ext(pods1, ext1, devices=True)
    ref2 = o.place_stream_ext(pods2, none)
    with _engine(prof) as e:
        e.load_snapshot(t)
        got1 = e.place_stream_ext(pods1, ext1)
        d1 = e.fetch_devices(len(pods1))
        got2 = e.place_stream_ext(pods2, none)
        assert "k_resolve" in e.kernel_names()["resolve"]
        d2 = e.fetch_devices(len(pods2))
    assert np.array_equal(got1, ref1) and np.array_equal(d1, dref1)
    assert (d1 != 0).any()
    assert np.array_equal(got2, ref2)
    assert not d2.any(), np.flatnonzero(d2.any(axis=1))[:10]


@pytest.mark.gpu
def test_device_totals_beyond_exact_range_rejected():
    """The device scorer divides by f64 reciprocal with one exact fix-up
    (dev.hpp dev_pct_div), exact for operands below 2^45: larger dev_total /
    dev_used are refused at load_snapshot, not silently mis-scored."""
    prof = with_deviceshare(shipped_profile())
    t = _cluster(200, prof, seed=61)
    t["dev_total"][0, abi.DEV_GPU, 0, 2] = 1 << 46
    with _engine(prof) as e:
        with pytest.raises(abi.KoordhipError, match="2\\^45"):
            e.load_snapshot(t)


@pytest.mark.gpu
def test_spread_affinity_profile_batch_without_ext_runs_pipelined():
    """PodTopologySpread + InterPodAffinity + DeviceShare in the profile: a
    batch whose koordhip_pod_ext records are empty (no constraint, no term,
    counted by no entry) couples no nodes and runs on the pipelined greedy; a
    batch with spread / affinity pods then runs the sequential cycle on the state
    the first left, both bit-exact with the oracle."""
    from koordinator_amd.config import with_interpod_affinity, with_topology_spread
    prof = with_interpod_affinity(with_topology_spread(with_deviceshare(shipped_profile())))
    t = _cluster(3000, prof, seed=41)
    pods = synth.make_pods(synth.StreamSpec(1200, be_frac=0.3, seed=42), prof)
    none = abi.pod_ext_array(len(pods))
    pods2 = synth.make_pods(synth.StreamSpec(500, be_frac=0.3, seed=43), prof)
    ext2 = synth.make_device_ext(len(pods2), synth.DevStreamSpec(frac=0.2, seed=43))
    synth.add_spread(t, ext2, synth.SpreadSpec())
    synth.add_ipa(t, ext2, synth.IpaSpec())
    o = oracle.Oracle(to_c_config(prof), t)
    ref1 = o.place_stream_ext(pods, none)
    ref2 = o.place_stream_ext(pods2, ext2)
    with _engine(prof) as e:
        e.load_snapshot(t)
        got1 = e.place_stream_ext(pods, none)
        k1 = e.kernel_names()["resolve"]
        got2 = e.place_stream_ext(pods2, ext2)
        k2 = e.kernel_names()["resolve"]
    assert "k_resolve" in k1 and "k_seq" in k2, (k1, k2)
    assert np.array_equal(got1, ref1), np.flatnonzero(got1 != ref1)[:10]
    assert np.array_equal(got2, ref2), np.flatnonzero(got2 != ref2)[:10]
    assert ((ext2["pts_n"] > 0) & (got2 >= 0)).sum() > 100


def _state(e):
    s = e.read_nodes()
    d = e.read_devices()
    return {"requested": s["requested"], "nz": s["nz"], "npods": s["npods"], "la_used": s["la_used"],
            "dev_used": d["dev_used"], "xrequested": d["xrequested"], "pts": e.read_pts(), "ipa": e.read_ipa()}


def _ostate(o):
    s, d = o.state(), o.dev_state()
    return {"requested": s["requested"], "nz": s["nz"], "npods": s["npods"], "la_used": s["la_used"],
            "dev_used": d["dev_used"], "xrequested": d["xrequested"], "pts": o.pts_counts(), "ipa": o.ipa_counts()}


@pytest.mark.gpu
def test_commit_ext_uncommit_ext_then_stream():
    """koordhip_commit_ext / koordhip_uncommit_ext (the Go shim's Reserve of a
    node it chose, and the Unreserve after a failed Permit / PreBind) for
    device pods with PodTopologySpread / InterPodAffinity records: each Reserve
    equals the oracle cycle's Reserve of that pod on that node (node state,
    deviceUsed, the extended scalars, the spread / affinity counts, the device
    slots); Unreserve restores the state exactly, and a stream placed afterwards
    equals the oracle's from the untouched snapshot."""
    from koordinator_amd.config import with_interpod_affinity, with_topology_spread
    prof = with_interpod_affinity(with_topology_spread(with_deviceshare(shipped_profile())))
    t = _cluster(1500, prof, seed=71)
    pods = synth.make_pods(synth.StreamSpec(300, be_frac=0.3, seed=72), prof)
    ext = synth.make_device_ext(len(pods), synth.DevStreamSpec(frac=0.5, seed=72))
    synth.add_spread(t, ext, synth.SpreadSpec())
    synth.add_ipa(t, ext, synth.IpaSpec())
    cfg = to_c_config(prof)
    # pods with device requests and spread / affinity content
    pick = [j for j in range(len(pods)) if ext["flags"][j] & abi.PODX_DEVICE and
            (ext["pts_match"][j] or ext["ipa_inc"][j])][:6]
    assert len(pick) >= 3
    with _engine(prof) as e:
        e.load_snapshot(t)
        base = _state(e)
        o0 = oracle.Oracle(cfg, t)
        assert all(np.array_equal(base[k], v) for k, v in _ostate(o0).items())
        for j in pick:
            o = oracle.Oracle(cfg, t)   # the cycle's choice of node for this pod alone, and its Reserve
            w, rdev = o.place_stream_ext(pods[j:j + 1], ext[j:j + 1], devices=True)
            if w[0] < 0:
                continue
            cpus, dev = e.commit_ext(pods[j], ext[j], int(w[0]))
            assert np.array_equal(dev, rdev[0]), (j, dev, rdev[0])
            got, want = _state(e), _ostate(o)
            for k in want:
                assert np.array_equal(got[k], want[k]), (j, k)
            e.uncommit_ext(pods[j], ext[j], int(w[0]), cpus, dev)
            got = _state(e)
            for k in base:
                assert np.array_equal(got[k], base[k]), ("after uncommit", j, k)
        rest = slice(100, 300)
        ref = oracle.Oracle(cfg, t).place_stream_ext(pods[rest], ext[rest])
        gotp = e.place_stream_ext(pods[rest], ext[rest])
    assert np.array_equal(gotp, ref), np.flatnonzero(gotp != ref)[:10]
