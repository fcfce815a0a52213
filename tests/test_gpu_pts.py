"""PodTopologySpread through libkoordhip.so's sequential cycle against the
oracle (oracle/pts_oracle.c): the hand-worked cases of test_pts_oracle.py on
the device, eval_ext planes / status / top-k, and streams -- placements, the
constraint counts after the stream and the node state -- bit for bit, alone
and beside Fit / LoadAware / DeviceShare / NodeNUMAResource."""
import numpy as np
import pytest

import oracle
from koordinator_amd import abi, synth
from koordinator_amd.config import (shipped_profile, to_c_config, with_deviceshare, with_normalized_scores,
                                    with_topology_spread)
from koordinator_amd.snapshot import pod_array

import test_pts_oracle as K

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
    return g, r


@pytest.mark.parametrize("cons", [((0, True, 1),), ((0, True, 3),), ((1, True, 1),), ((0, False, 1),),
                                  ((1, False, 2),), ((0, False, 1), (0, False, 3)), ((0, True, 2), (1, False, 1))],
                         ids=str)
def test_hand_cases_on_device(cons):
    t = K.table()
    x = K.ext(*cons)
    g, r = _eval_both(K.profile(), t, pod_array(1), x, k=5)
    for key in ("status", "scores", "topk"):
        assert np.array_equal(g[key], r[key]), key


def test_affinity_restricted_pairs_on_device():
    t = K.table(elig_hard=0b00011)
    g, r = _eval_both(K.profile(), t, pod_array(1), K.ext((0, True, 1)), k=5)
    assert np.array_equal(g["status"], r["status"])


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


def test_eval_ext_parity_spread_classes():
    prof = with_topology_spread(shipped_profile())
    t = _cluster(900, prof, synth.SEED + 31)
    pods, ext = _stream(40, prof, synth.SEED + 31)
    synth.add_spread(t, ext, synth.SpreadSpec(seed=synth.SEED + 31))
    g, r = _eval_both(prof, t, pods, ext, k=8)
    for key in ("status", "scores", "topk"):
        assert np.array_equal(g[key], r[key]), key
    assert (g["status"] & abi.ST_PTS_FAIL).any()
    assert g["scores"][:, abi.NPLUGINS + 3].any()


def _compare(prof, t, pods, ext, cpusets=False):
    with _engine(prof) as e:
        e.load_snapshot(t)
        got = e.place_stream_ext(pods, ext)
        gst = e.read_nodes()
        gcnt = e.read_pts()
        gcs = e.fetch_cpusets(len(pods)) if cpusets else None
    o = oracle.Oracle(to_c_config(prof), t)
    res = o.place_stream_ext(pods, ext, cpusets=cpusets)
    ref, rcs = (res[0], res[1]) if cpusets else (res, None)
    bad = np.flatnonzero(got != ref)
    assert bad.size == 0, f"first mismatch at pod {bad[0]}: hip {got[bad[0]]} oracle {ref[bad[0]]}"
    assert np.array_equal(gcnt, o.pts_counts())
    ost = o.state()
    for k in ("requested", "nz", "npods", "la_used"):
        assert np.array_equal(gst[k], ost[k]), k
    if cpusets:
        assert np.array_equal(gcs, rcs)
    return got


@pytest.mark.parametrize("seed", [1, 2])
def test_stream_spread_fit_loadaware(seed):
    prof = with_topology_spread(shipped_profile())
    t = _cluster(1200, prof, synth.SEED + 40 + seed)
    pods, ext = _stream(1500, prof, synth.SEED + 40 + seed)
    synth.add_spread(t, ext, synth.SpreadSpec(seed=synth.SEED + 40 + seed))
    got = _compare(prof, t, pods, ext)
    assert (got >= 0).sum() > 1000


def test_stream_spread_filter_only_and_score_only():
    for prof in (with_topology_spread(shipped_profile(), weight=0),
                 with_topology_spread(shipped_profile(), weight=3, filter=False)):
        t = _cluster(700, prof, synth.SEED + 47)
        pods, ext = _stream(900, prof, synth.SEED + 47)
        synth.add_spread(t, ext, synth.SpreadSpec(seed=synth.SEED + 47))
        _compare(prof, t, pods, ext)


def test_stream_spread_with_devices_and_numa():
    """PodTopologySpread beside DeviceShare (a Reserve that may fail: the
    commit result goes through its own hand-off) and NodeNUMAResource cpuset
    pods, plus the normalized NodeAffinity / TaintToleration Scores."""
    prof = with_normalized_scores(with_topology_spread(with_deviceshare(shipped_profile(numa=True))), affinity=1,
                                  taint=1)
    t = _cluster(800, prof, synth.SEED + 53, numa=True, devices=True)
    pods, ext = _stream(1000, prof, synth.SEED + 53, cpuset=0.3, dev_frac=0.25)
    synth.add_spread(t, ext, synth.SpreadSpec(seed=synth.SEED + 53))
    _compare(prof, t, pods, ext, cpusets=True)


def test_checkpoint_restore_counts():
    prof = with_topology_spread(shipped_profile())
    t = _cluster(500, prof, synth.SEED + 59)
    pods, ext = _stream(600, prof, synth.SEED + 59)
    synth.add_spread(t, ext, synth.SpreadSpec(seed=synth.SEED + 59))
    with _engine(prof) as e:
        e.load_snapshot(t)
        e.checkpoint()
        a = e.place_stream_ext(pods, ext)
        ca = e.read_pts()
        e.restore()
        b = e.place_stream_ext(pods, ext)
        cb = e.read_pts()
    assert np.array_equal(a, b) and np.array_equal(ca, cb)


def test_update_nodes_spread_rows():
    """update_nodes of the pts_* rows (pods finished, a node relabelled out of
    its zone), then a stream equal to the oracle on the updated table."""
    prof = with_topology_spread(shipped_profile())
    t = _cluster(600, prof, synth.SEED + 61)
    pods, ext = _stream(700, prof, synth.SEED + 61)
    synth.add_spread(t, ext, synth.SpreadSpec(seed=synth.SEED + 61))
    idx = np.arange(0, 600, 7, dtype=np.int32)
    t2 = t.copy()
    t2["pts_cnt"][idx] = 0
    t2["pts_dom"][idx[:5], 0] = -1
    with _engine(prof) as e:
        e.load_snapshot(t)
        e.update_nodes(idx, t2.rows(idx))
        got = e.place_stream_ext(pods, ext)
    ref = oracle.Oracle(to_c_config(prof), t2).place_stream_ext(pods, ext)
    assert np.array_equal(got, ref)
