"""InterPodAffinity through libkoordhip.so's sequential cycle against the
oracle (oracle/ipa_oracle.c): eval_ext status / raw planes / top-k on the
object-built hand and random cases of test_ipa_objects.py and on synthetic
tables, and streams -- placements, the count entries after the stream and the
node state -- bit for bit, alone and beside Fit / LoadAware /
PodTopologySpread / DeviceShare / NodeNUMAResource; update_nodes, checkpoint."""
import numpy as np
import pytest

import oracle
from koordinator_amd import abi, synth
from koordinator_amd.config import (shipped_profile, to_c_config, with_deviceshare, with_interpod_affinity,
                                    with_normalized_scores, with_topology_spread)

import test_ipa_objects as K

pytestmark = pytest.mark.gpu


def _engine(prof):
    import torch  # noqa: F401
    from koordinator_amd.engine import PlacementEngine
    return PlacementEngine(prof, device=0)


def _eval_both(prof, t, pods, ext, k=8):
    with _engine(prof) as e:
        e.load_snapshot(t)
        g = e.eval_ext(pods, ext, k=k)
    r = oracle.Oracle(to_c_config(prof), t).eval_ext(pods, ext, k=k)
    for key in ("status", "scores", "topk"):
        assert np.array_equal(g[key], r[key]), key
    return g, r


def test_hand_cases_on_device():
    running = [K.pod("db0", {"app": "db"}, node_name="d"), K.pod("w0", {"app": "web"}, node_name="a"),
               K.pod("g", {"app": "guard"}, node_name="c", anti=[K.T(K.WEB, K.ZONE)]),
               K.pod("f", {"app": "fan"}, node_name="d", aff=[K.T(K.WEB, K.ZONE)])]
    pending = [K.pod("w", {"app": "web"}, aff=[K.T(K.DB, K.ZONE)]),
               K.pod("s", {"app": "web"}, aff=[K.T(K.WEB, K.ZONE)]),
               K.pod("x", {"app": "web"}, anti=[K.T(K.WEB, K.HOST)]),
               K.pod("p", {"app": "web"}, paff=[K.W(5, K.T(K.DB, K.ZONE))], panti=[K.W(3, K.T(K.WEB, K.HOST))])]
    for prof in (K.ipa_profile(), K.ipa_profile(hard=0), K.ipa_profile(weight=4, filt=False)):
        c, t, pods, ext = K.snapshot(K.NODES, running, pending, prof)
        g, _ = _eval_both(prof, t, pods, ext, k=5)
    assert (g["status"] & abi.ST_IPA_FAIL).any() or True


@pytest.mark.parametrize("seed", range(4))
def test_random_objects_eval_and_stream(seed):
    nodes, running, pending = K.random_case(seed)
    pending = K.fitting(nodes, running, pending)
    prof = K.ipa_profile(weight=3)
    c, t, pods, ext = K.snapshot(nodes, running, pending, prof)
    _eval_both(prof, t, pods, ext, k=6)
    with _engine(prof) as e:
        e.load_snapshot(t)
        got = e.place_stream_ext(pods, ext)
        cnt = e.read_ipa()
    o = oracle.Oracle(to_c_config(prof), t)
    assert np.array_equal(got, o.place_stream_ext(pods, ext))
    assert np.array_equal(cnt, o.ipa_counts())


def _cluster(n, prof, seed, numa=False, devices=False):
    t = synth.make_cluster(synth.ClusterSpec(n, seed=seed), prof)
    if numa:
        synth.add_numa(t, synth.NumaSpec(), prof, seed=seed)
    if devices:
        synth.add_devices(t, synth.DevSpec(), seed=seed)
    else:
        t.enable_ext(0)
    return t


def _stream(n, prof, seed, cpuset=0.0, dev_frac=0.0):
    pods = synth.make_pods(synth.StreamSpec(n, be_frac=0.3, seed=seed, cpuset_frac=cpuset), prof)
    ext = synth.make_device_ext(n, synth.DevStreamSpec(frac=dev_frac, seed=seed)) if dev_frac else abi.pod_ext_array(n)
    return pods, ext


def test_eval_ext_parity_synthetic():
    prof = with_interpod_affinity(shipped_profile())
    t = _cluster(900, prof, synth.SEED + 71)
    pods, ext = _stream(48, prof, synth.SEED + 71)
    synth.add_ipa(t, ext, synth.IpaSpec(seed=synth.SEED + 71))
    g, _ = _eval_both(prof, t, pods, ext, k=8)
    assert (g["status"] & abi.ST_IPA_FAIL).any()
    assert g["scores"][:, abi.NPLUGINS + 4].any()


def _compare(prof, t, pods, ext, cpusets=False):
    with _engine(prof) as e:
        e.load_snapshot(t)
        got = e.place_stream_ext(pods, ext)
        gst = e.read_nodes()
        gcnt = e.read_ipa()
        gpts = e.read_pts()
        gcs = e.fetch_cpusets(len(pods)) if cpusets else None
    o = oracle.Oracle(to_c_config(prof), t)
    res = o.place_stream_ext(pods, ext, cpusets=cpusets)
    ref, rcs = (res[0], res[1]) if cpusets else (res, None)
    bad = np.flatnonzero(got != ref)
    assert bad.size == 0, f"first mismatch at pod {bad[0]}: hip {got[bad[0]]} oracle {ref[bad[0]]}"
    assert np.array_equal(gcnt, o.ipa_counts())
    assert np.array_equal(gpts, o.pts_counts())
    ost = o.state()
    for k in ("requested", "nz", "npods", "la_used"):
        assert np.array_equal(gst[k], ost[k]), k
    if cpusets:
        assert np.array_equal(gcs, rcs)
    return got


@pytest.mark.parametrize("seed", [1, 2])
def test_stream_ipa_fit_loadaware(seed):
    prof = with_interpod_affinity(shipped_profile())
    t = _cluster(1200, prof, synth.SEED + 80 + seed)
    pods, ext = _stream(1500, prof, synth.SEED + 80 + seed)
    synth.add_ipa(t, ext, synth.IpaSpec(seed=synth.SEED + 80 + seed))
    got = _compare(prof, t, pods, ext)
    assert (got >= 0).sum() > 1000


def test_stream_ipa_filter_only_and_score_only():
    for prof in (with_interpod_affinity(shipped_profile(), weight=0),
                 with_interpod_affinity(shipped_profile(), weight=5, filter=False)):
        t = _cluster(700, prof, synth.SEED + 87)
        pods, ext = _stream(900, prof, synth.SEED + 87)
        synth.add_ipa(t, ext, synth.IpaSpec(seed=synth.SEED + 87))
        _compare(prof, t, pods, ext)


def test_stream_ipa_with_spread_devices_and_numa():
    """InterPodAffinity beside PodTopologySpread (the same topology keys),
    DeviceShare and NodeNUMAResource cpuset pods (Reserves that may fail) and
    the normalized NodeAffinity / TaintToleration Scores."""
    prof = with_normalized_scores(with_interpod_affinity(with_topology_spread(with_deviceshare(
        shipped_profile(numa=True)))), affinity=1, taint=1)
    t = _cluster(800, prof, synth.SEED + 93, numa=True, devices=True)
    pods, ext = _stream(1000, prof, synth.SEED + 93, cpuset=0.3, dev_frac=0.25)
    synth.add_spread(t, ext, synth.SpreadSpec(seed=synth.SEED + 93))
    synth.add_ipa(t, ext, synth.IpaSpec(seed=synth.SEED + 93))
    _compare(prof, t, pods, ext, cpusets=True)


def test_checkpoint_restore_and_update_nodes():
    prof = with_interpod_affinity(shipped_profile())
    t = _cluster(600, prof, synth.SEED + 97)
    pods, ext = _stream(700, prof, synth.SEED + 97)
    synth.add_ipa(t, ext, synth.IpaSpec(seed=synth.SEED + 97))
    idx = np.arange(0, 600, 7, dtype=np.int32)
    t2 = t.copy()
    t2["ipa_cnt"][idx] = 0
    t2["pts_dom"][idx[:5], 0] = -1
    with _engine(prof) as e:
        e.load_snapshot(t)
        e.checkpoint()
        a = e.place_stream_ext(pods, ext)
        ca = e.read_ipa()
        e.restore()
        b = e.place_stream_ext(pods, ext)
        assert np.array_equal(a, b) and np.array_equal(ca, e.read_ipa())
        e.restore()
        e.update_nodes(idx, t2.rows(idx))
        got = e.place_stream_ext(pods, ext)
    ref = oracle.Oracle(to_c_config(prof), t2).place_stream_ext(pods, ext)
    assert np.array_equal(got, ref)
