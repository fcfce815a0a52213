"""DeviceShare beside the Reservation plugin: the nomination of a device pod.

The reservation filter plugins of NominateReservation (reservation/nominator.go:
47-54, RunReservationFilterPlugins) include DeviceShare's FilterReservation
(deviceshare/plugin.go:325-356).  For a pod requesting devices it looks the
reservation up in the node's RestoreReservation state, which keeps only the
reservations holding devices (deviceshare/reservation.go:134-161); one holding
none is not found (allocIndex -1) and FilterReservation returns an error
status, so NominateReservation skips it.  Worked by hand for one node with one
GPU and one matched 4C8G reservation holding no devices:

  * a device pod (2C4G + half a GPU): no reservation nominated -> DeviceShare
    Reserve allocates from the node (allocateWithNominatedReservation sees no
    nominated reservation, plugin.go:379-382), the Reservation Reserve assumes
    nothing (plugin.go:550-561): placed, the reservation's Allocated and
    AssignedPods unchanged, the GPU half used;
  * the same pod without the device request: nominated -> assumed into the
    reservation (Allocated 2C4G, one assigned pod).

The oracle (CPU) and libkoordhip.so's sequential cycle (GPU) against those
answers; parity of random streams is test_gpu_deviceshare.py's
test_stream_deviceshare_numa_reservation."""
import numpy as np
import pytest

import golden_cases as G
import oracle
from koordinator_amd import abi, marshal
from koordinator_amd import reservation as rv
from koordinator_amd.config import to_c_config, with_deviceshare

NODE = [("test-node", {"cpu": "32", "memory": "64Gi", "pods": "110"})]
GIB = 1 << 30


def _case():
    prof = with_deviceshare(G.resv_profile())
    r = rv.Reservation("r-4c8g", "test-node", allocatable=G.rlist({"cpu": "4", "memory": "8Gi"}),
                       owners=G.match_all_owner(), allocate_once=False)
    t, idx = G.build_resv_nodes(NODE, [r], prof)
    t.enable_ext(dev_slots=4)
    t["dev_present"][:] = 1
    t["dev_minor"][:] = -1
    t["dev_minor"][0, abi.DEV_GPU, 0] = 0
    t["dev_total"][0, abi.DEV_GPU, 0] = [100, 100, 16 * GIB]
    pods = marshal.pod_records([G.resv_pod({"cpu": "2", "memory": "4Gi"}, name="p0"),
                                G.resv_pod({"cpu": "2", "memory": "4Gi"}, name="p1")], prof, idx)
    ext = abi.pod_ext_array(2)
    ext["flags"][0] = abi.PODX_DEVICE
    ext["dev_req"][0, abi.DEV_GPU] = [50, 50, -1]
    return prof, t, pods, ext


def _check(out, resv, used):
    assert out.tolist() == [0, 0]
    # pod 0 (devices) took no reservation; pod 1 (plain) was assumed into it
    assert int(resv["assigned"].ravel()[0]) == 1
    assert int(resv["allocated"][0].ravel()[0]) == 2000
    assert used[0, abi.DEV_GPU, 0].tolist() == [50, 50, 8 * GIB]


def test_device_pod_is_not_nominated_oracle():
    prof, t, pods, ext = _case()
    o = oracle.Oracle(to_c_config(prof), t)
    assert o.resv_nominate(pods[1:2], 0) == 0
    out, _ = o.place_stream_ext(pods, ext, devices=True)
    _check(out, o.resv_state(), o.dev_state()["dev_used"])


@pytest.mark.gpu
def test_device_pod_is_not_nominated_gpu():
    import torch  # noqa: F401
    from koordinator_amd.engine import PlacementEngine
    prof, t, pods, ext = _case()
    with PlacementEngine(prof, device=0) as e:
        e.load_snapshot(t)
        out = e.place_stream_ext(pods, ext)
        _check(out, e.read_reservations(), e.read_devices()["dev_used"])
    # one at a time through koordhip_commit_ext: the same state
    prof, t, pods, ext = _case()
    with PlacementEngine(prof, device=0) as e:
        e.load_snapshot(t)
        for j in range(2):
            e.commit_ext(pods[j], ext[j], 0)
        _check(np.zeros(2, np.int32), e.read_reservations(), e.read_devices()["dev_used"])


# ------------------------------------------------- reservations holding devices
# Known answers: deviceshare/reservation_test.go:224-660 (Test_tryAllocateFromReservation):
# one node with GPUs 0, 1 (100 core / 100 ratio / 8Gi each), its matched
# reservation holding GPU 0 (allocatable A, allocated D; remained = A - D), the
# node's deviceUsed, a pod requesting half a GPU (50 core, 4Gi); the cases whose
# restore state is consistent with A / D (remained = SubtractWithNonNegativeResult(A, D)).
HALF = [50, 50, 4 * GIB]
QUARTER = [25, 25, 2 * GIB]
FULL = [100, 100, 8 * GIB]
ZERO = [0, 0, 0]
# (name, policy, A, D, used[minor0, minor1], request (core, mem), fromResv, want: (1 minor | 0 | -1))
TRY_CASES = [
    ("allocate from default policy reservation", rv.POLICY_DEFAULT, QUARTER, ZERO, [ZERO, ZERO], (50, 4 * GIB), False, 0),
    ("default policy, required from reservation, reservation empty", rv.POLICY_DEFAULT, HALF, HALF,
     [[150, 150, 12 * GIB], ZERO], (50, 4 * GIB), True, None),
    ("allocate from Aligned policy reservation", rv.POLICY_ALIGNED, HALF, ZERO, [FULL, FULL], (50, 4 * GIB), False, 0),
    ("Aligned: bigger request, no remaining resources on node", rv.POLICY_ALIGNED, HALF, ZERO, [FULL, FULL],
     (60, 5 * GIB), False, -1),
    ("Aligned: remaining little not fits request", rv.POLICY_ALIGNED, HALF, QUARTER, [[125, 125, 10 * GIB], FULL],
     (30, 1 * GIB), False, -1),
    ("allocate from Restricted policy reservation", rv.POLICY_RESTRICTED, HALF, ZERO, [FULL, FULL], (50, 4 * GIB),
     False, 0),
    ("Restricted: node remains resources but reservation not fits", rv.POLICY_RESTRICTED, HALF, QUARTER,
     [[75, 75, 6 * GIB], FULL], (50, 4 * GIB), False, -1),
]


def _dev_resv_table(policy, A, D, used, match=True):
    prof = with_deviceshare(G.resv_profile())
    owners = G.match_all_owner() if match else [rv.ReservationOwner(labels={"app": "nobody"})]
    r = rv.Reservation("r", "test-node", allocatable=G.rlist({"cpu": "4", "memory": "8Gi"}), owners=owners,
                       allocate_once=False, allocate_policy=policy)
    t, idx = G.build_resv_nodes(NODE, [r], prof)
    t.enable_ext(dev_slots=2)
    t["dev_present"][:] = 1
    for s in range(2):
        t["dev_minor"][0, abi.DEV_GPU, s] = s
        t["dev_total"][0, abi.DEV_GPU, s] = FULL
        t["dev_used"][0, abi.DEV_GPU, s] = used[s]
    t.enable_resv_dev()
    t["resv_dev_slot"][0] = 0
    t["resv_dev"][0, 0, abi.DEV_GPU, 0] = A
    t["resv_dev"][0, 1, abi.DEV_GPU, 0] = D
    pod = marshal.pod_records([G.resv_pod({"cpu": "2", "memory": "4Gi"}, name="p")], prof, idx)
    return prof, t, pod


def _gpu_ext(core, mem):
    x = abi.pod_ext_array(1)
    x["flags"][0] = abi.PODX_DEVICE
    x["dev_req"][0, abi.DEV_GPU] = [core, -1, mem]
    return x


@pytest.mark.parametrize("case", TRY_CASES, ids=[c[0] for c in TRY_CASES])
def test_try_allocate_from_reservation_kat(case):
    name, pol, A, D, used, (core, mem), from_resv, want = case
    prof, t, pod = _dev_resv_table(pol, A, D, used)
    o = oracle.Oracle(to_c_config(prof), t)
    r, slots = o.dev_try_from_reservation(pod, _gpu_ext(core, mem), 0, from_resv)
    if want is None:
        assert r == 0
    elif want < 0:
        assert r == -1
    else:
        assert r == 1 and int(slots[abi.DEV_GPU]) == 1 << want


def _dev_resv_cluster(n, seed):
    """A DeviceShare + Reservation + NodeNUMAResource cluster whose reservations
    on GPU nodes hold devices (synth.add_device_reservations)."""
    from koordinator_amd.config import shipped_profile
    from koordinator_amd import synth
    prof = with_deviceshare(shipped_profile(numa=True, reservation=True))
    t = synth.make_cluster(synth.ClusterSpec(n, seed=seed), prof)
    synth.add_numa(t, synth.NumaSpec(), prof, seed=seed)
    synth.add_reservations(t, synth.ResvSpec(node_frac=0.6), seed=seed)
    synth.add_devices(t, synth.DevSpec(gpu_frac=0.6), seed=seed)
    synth.add_device_reservations(t, synth.DevResvSpec(), seed=seed)
    return prof, t


def _dev_resv_pods(n, prof, seed, dev_frac=0.4):
    from koordinator_amd import synth
    pods = synth.make_pods(synth.StreamSpec(n, be_frac=0.3, seed=seed, cpuset_frac=0.2, resv_match_frac=0.6), prof)
    ext = synth.make_device_ext(n, synth.DevStreamSpec(frac=dev_frac, seed=seed))
    return pods, ext


def test_device_holding_reservations_oracle_stream_runs():
    """The oracle's reference cycle over a cluster with device-holding
    reservations: device pods land in them (their allocated grows) and on the
    rest of the nodes."""
    prof, t = _dev_resv_cluster(300, seed=41)
    assert (t["resv_dev_slot"] >= 0).sum() > 20
    pods, ext = _dev_resv_pods(600, prof, seed=41)
    o = oracle.Oracle(to_c_config(prof), t)
    out, _ = o.place_stream_ext(pods, ext, devices=True)
    dev = (ext["flags"] & abi.PODX_DEVICE) != 0
    assert (out[dev] >= 0).sum() > 50
    grew = o.resv_dev_state()[:, 1].sum() - t["resv_dev"][:, 1].sum()
    assert grew > 0


@pytest.mark.gpu
@pytest.mark.parametrize("case", TRY_CASES, ids=[c[0] for c in TRY_CASES])
def test_device_holding_reservation_kat_gpu(case):
    """The same cases through libkoordhip.so: the Filter verdict and the
    placement / allocation of a one-pod stream equal the oracle's."""
    import torch  # noqa: F401
    from koordinator_amd.engine import PlacementEngine
    name, pol, A, D, used, (core, mem), from_resv, want = case
    prof, t, pod = _dev_resv_table(pol, A, D, used)
    x = _gpu_ext(core, mem)
    o = oracle.Oracle(to_c_config(prof), t)
    r = o.eval_ext(pod, x, k=1)
    ref_out, ref_dev = o.place_stream_ext(pod, x, devices=True)
    with PlacementEngine(prof, device=0) as e:
        e.load_snapshot(t)
        g = e.eval_ext(pod, x, k=1)
        out = e.place_stream_ext(pod, x)
        gdev = e.fetch_devices(1)
        grd = e.read_resv_devices()
    assert np.array_equal(g["status"], r["status"]) and np.array_equal(g["scores"], r["scores"])
    assert np.array_equal(out, ref_out) and np.array_equal(gdev, ref_dev)
    assert np.array_equal(grd, o.resv_dev_state())


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [41, 42])
def test_device_holding_reservations_stream_gpu(seed):
    """The full shipped profile (DeviceShare + Reservation + NodeNUMAResource)
    with reservations holding devices: placements, device slots, deviceUsed,
    the reservations' allocated devices, CPU / memory and cpusets bit-exact
    with the oracle."""
    import torch  # noqa: F401
    from koordinator_amd.engine import PlacementEngine
    prof, t = _dev_resv_cluster(400, seed=seed)
    pods, ext = _dev_resv_pods(800, prof, seed=seed)
    o = oracle.Oracle(to_c_config(prof), t)
    ref, rcs, rdev = o.place_stream_ext(pods, ext, cpusets=True, devices=True)
    with PlacementEngine(prof, device=0) as e:
        e.load_snapshot(t)
        got = e.place_stream_ext(pods, ext)
        gdev = e.fetch_devices(len(pods))
        gcs = e.fetch_cpusets(len(pods))
        gdv = e.read_devices()
        grd = e.read_resv_devices()
        gst = e.read_nodes()
        grs = e.read_reservations()
    bad = np.flatnonzero(got != ref)
    assert bad.size == 0, f"first mismatch at pod {bad[0]}: hip {got[bad[0]]} oracle {ref[bad[0]]}"
    assert np.array_equal(gdev, rdev) and np.array_equal(gcs, rcs)
    assert np.array_equal(gdv["dev_used"], o.dev_state()["dev_used"])
    assert np.array_equal(grd, o.resv_dev_state())
    ost, ors = o.state(), o.resv_state()
    for k in ("requested", "nz", "npods"):
        assert np.array_equal(gst[k], ost[k]), k
    assert np.array_equal(grs["allocated"], ors["allocated"]) and np.array_equal(grs["assigned"], ors["assigned"])
    dev = (ext["flags"] & abi.PODX_DEVICE) != 0
    assert (got[dev] >= 0).sum() > 50
    assert grd[:, 1].sum() > t["resv_dev"][:, 1].sum()   # device pods were assumed into the reservations
