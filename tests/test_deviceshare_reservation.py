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


# ------------------------------ the extended scalars of a device-holding reservation
# (ABI 14).  Worked by hand from reservation/transformer.go:227-293 and
# scoring.go:177-200.  One node with two GPUs (100 core / 100 ratio / 8Gi each):
# NodeResourcesFit's Allocatable gpu-core = gpu-memory-ratio = 200.  Its Default
# reservation R (4C8G + gpu-core 100 + gpu-memory-ratio 100) holds GPU 0; one
# assigned pod (1C1G + 50 core / 50 ratio on GPU 0) is in it: Allocated = 1C1G +
# 50 / 50.  NodeInfo.Requested's scalars: the reserve pod's 100 + the assigned
# pod's 50 = 150 of each.
#   * a pod R matches requesting a whole GPU as gpu-core 100 + gpu-memory-ratio 100:
#     RemovePod(reservePod) leaves 150 - 100 = 50 requested, 100 <= 200 - 50: Fit
#     passes (on the raw 150 it would fail: 100 > 50);
#   * a pod R does not match: restoreUnmatchedReservations -> 150 - 100 +
#     SubtractWithNonNegativeResult(100, 50) = 100, 100 <= 200 - 100: passes
#     exactly (raw: fails);
#   * a plain 1C1G pod R matches: scoreReservation over RemoveZeros(Allocatable) =
#     {cpu, memory, gpu-core, gpu-memory-ratio}: cpu (1 + 1) / 4 -> 50, memory
#     (1 + 1) / 8 -> 25, gpu-core (0 + 50) / 100 -> 50, ratio 50: 175 / 4 = 43
#     (cpu / memory alone: 37).
def _scalar_case(match=True):
    from koordinator_amd import deviceshare as ds
    prof = with_deviceshare(G.resv_profile())
    owners = G.match_all_owner() if match else [rv.ReservationOwner(label_selector=rv.LabelSelector(
        match_labels={"app": "nobody"}))]
    # (the cpu / memory columns from the object; the device and scalar columns set below by hand)
    r = rv.Reservation("r", "test-node", allocatable=G.rlist({"cpu": "4", "memory": "8Gi"}),
                       allocated=G.rlist({"cpu": "1", "memory": "1Gi"}), assigned=1, owners=owners, allocate_once=False)
    t, idx = G.build_resv_nodes(NODE, [r], G.resv_profile())
    t.enable_ext(dev_slots=2)
    t["dev_present"][:] = 1
    for s in range(2):
        t["dev_minor"][0, abi.DEV_GPU, s] = s
        t["dev_total"][0, abi.DEV_GPU, s] = FULL
    t["dev_used"][0, abi.DEV_GPU, 0] = [150, 150, 12 * GIB]       # the reserve pod's GPU 0 + the assigned pod's half
    t["xalloc"][0, ds.XRES_INDEX[ds.GPU_CORE]] = 200
    t["xalloc"][0, ds.XRES_INDEX[ds.GPU_MEMORY_RATIO]] = 200
    t["xrequested"][0, ds.XRES_INDEX[ds.GPU_CORE]] = 150
    t["xrequested"][0, ds.XRES_INDEX[ds.GPU_MEMORY_RATIO]] = 150
    t.enable_resv_dev()
    t["resv_dev_slot"][0] = 0
    t["resv_dev"][0, 0, abi.DEV_GPU, 0] = FULL
    t["resv_dev"][0, 1, abi.DEV_GPU, 0] = HALF
    t["resv_xalloc"][0, ds.XRES_INDEX[ds.GPU_CORE]] = 100
    t["resv_xalloc"][0, ds.XRES_INDEX[ds.GPU_MEMORY_RATIO]] = 100
    t["resv_xallocated"][0, ds.XRES_INDEX[ds.GPU_CORE]] = 50
    t["resv_xallocated"][0, ds.XRES_INDEX[ds.GPU_MEMORY_RATIO]] = 50
    gpu_pod = G.resv_pod({"cpu": "1", ds.GPU_CORE: "100", ds.GPU_MEMORY_RATIO: "100"}, name="g")
    plain = G.resv_pod({"cpu": "1", "memory": "1Gi"}, name="p")
    pods = marshal.pod_records([gpu_pod, plain], prof, idx)
    ext = ds.pod_ext_records([gpu_pod, plain])
    return prof, t, pods, ext


@pytest.mark.parametrize("match", [True, False], ids=["matched", "unmatched"])
def test_resv_scalar_restore_kat_oracle(match):
    prof, t, pods, ext = _scalar_case(match)
    o = oracle.Oracle(to_c_config(prof), t)
    r = o.eval_ext(pods[:1], ext[:1])
    assert not (int(r["status"][0, 0]) & abi.ST_XFIT_FAIL)      # fits only through the restore
    # without the scalar columns the raw Requested (150) fails the 100 request
    t2 = t.copy()
    t2["resv_xalloc"][:] = 0
    t2["resv_xallocated"][:] = 0
    assert int(oracle.Oracle(to_c_config(prof), t2).eval_ext(pods[:1], ext[:1])["status"][0, 0]) & abi.ST_XFIT_FAIL
    if match:
        assert o.resv_score(pods[1:2], 0) == 43                 # scoring.go:177-200 over 4 resources
        assert oracle.Oracle(to_c_config(prof), t2).resv_score(pods[1:2], 0) == 37


def test_resv_scalar_reserve_oracle():
    """Reserve into the reservation (the plain pod is nominated): its Allocated
    grows by the pod's requests masked to ResourceNames -- no scalar for a pod
    requesting none; the GPU pod placed beside it adds its scalars to the node's
    Requested only (it is not nominated: DeviceShare's FilterReservation with
    requiredFromReservation finds GPU 0 full)."""
    from koordinator_amd import deviceshare as ds
    prof, t, pods, ext = _scalar_case(True)
    o = oracle.Oracle(to_c_config(prof), t)
    out, _ = o.place_stream_ext(pods, ext, devices=True)
    assert out.tolist() == [0, 0]
    rs = o.resv_scalar_state()
    assert int(rs[0, ds.XRES_INDEX[ds.GPU_CORE]]) == 50      # unchanged: the GPU pod was not assumed into it
    xr = o.dev_state()["xrequested"]
    assert int(xr[0, ds.XRES_INDEX[ds.GPU_CORE]]) == 250


@pytest.mark.gpu
@pytest.mark.parametrize("match", [True, False], ids=["matched", "unmatched"])
def test_resv_scalar_kat_gpu(match):
    """The same cases through libkoordhip.so's sequential cycle: eval planes,
    placements, devices, the scalars' Requested and the reservation's scalar
    Allocated equal the oracle's."""
    import torch  # noqa: F401
    from koordinator_amd.engine import PlacementEngine
    prof, t, pods, ext = _scalar_case(match)
    o = oracle.Oracle(to_c_config(prof), t)
    r = o.eval_ext(pods, ext, k=1)
    ref, rdev = o.place_stream_ext(pods, ext, devices=True)
    with PlacementEngine(prof, device=0) as e:
        e.load_snapshot(t)
        g = e.eval_ext(pods, ext, k=1)
        got = e.place_stream_ext(pods, ext)
        gdev = e.fetch_devices(len(pods))
        gx = e.read_devices()["xrequested"]
        grs = e.read_resv_scalars()
        gr = e.read_reservations()
    assert np.array_equal(g["status"], r["status"]) and np.array_equal(g["scores"], r["scores"])
    assert np.array_equal(g["topk"], r["topk"])
    assert np.array_equal(got, ref) and np.array_equal(gdev, rdev)
    assert np.array_equal(gx, o.dev_state()["xrequested"])
    assert np.array_equal(grs, o.resv_scalar_state())
    assert np.array_equal(gr["allocated"], o.resv_state()["allocated"])


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [43, 44])
def test_resv_scalar_streams_gpu(seed):
    """Shipped-profile streams over reservations holding devices AND listing
    their gpu-core / gpu-memory-ratio scalars (synth.DevResvSpec.scalars):
    every batch runs in the sequential cycle, device pods whose requests use the
    core + ratio form meet those keys in the restore, fitsNode, FilterReservation
    and scoreReservation; plain pods' nominations count them too.  Placements,
    devices, the scalars' Requested and the reservations' scalar Allocated
    bit-exact with the oracle."""
    import torch  # noqa: F401
    from koordinator_amd.engine import PlacementEngine
    prof, t = _dev_resv_cluster(400, seed=seed)
    assert t["resv_xalloc"].any()
    pods, ext = _dev_resv_pods(800, prof, seed=seed)
    o = oracle.Oracle(to_c_config(prof), t)
    ref, rcs, rdev = o.place_stream_ext(pods, ext, cpusets=True, devices=True)
    with PlacementEngine(prof, device=0) as e:
        e.load_snapshot(t)
        got = e.place_stream_ext(pods, ext)
        gdev = e.fetch_devices(len(pods))
        gdv = e.read_devices()
        grs = e.read_resv_scalars()
        grd = e.read_resv_devices()
        gr = e.read_reservations()
        # a batch of plain pods on the same snapshot: the sequential cycle too (scalar reservations)
        plain = _dev_resv_pods(200, prof, seed=seed + 100, dev_frac=0.0)[0]
        got2 = e.place_stream_ext(plain, None)
    bad = np.flatnonzero(got != ref)
    assert bad.size == 0, f"first mismatch at pod {bad[0]}: hip {got[bad[0]]} oracle {ref[bad[0]]}"
    assert np.array_equal(gdev, rdev)
    assert np.array_equal(gdv["dev_used"], o.dev_state()["dev_used"])
    assert np.array_equal(gdv["xrequested"], o.dev_state()["xrequested"])
    assert np.array_equal(grs, o.resv_scalar_state())
    assert np.array_equal(grd, o.resv_dev_state())
    assert np.array_equal(gr["allocated"], o.resv_state()["allocated"])
    assert np.array_equal(got2, o.place_stream_ext(plain, None))


def _object_cluster():
    """Reservation + Device + Pod objects: node n0 with two GPUs; Reservation R
    (Default, owners app=web) bound to n0 holding GPU 0 (its device-allocated
    annotation) and listing gpu-core / gpu-memory-ratio 100; one pod assigned to
    R through its reservation-allocated annotation, holding half of GPU 0."""
    import json as _json
    from koordinator_amd import deviceshare as ds, k8s
    from koordinator_amd.config import shipped_profile
    prof = with_deviceshare(shipped_profile(reservation=True))
    nodes = [k8s.Node(name=f"n{i}", allocatable=G.rlist({"cpu": "32", "memory": "64Gi", "pods": "110",
                                                          ds.GPU_CORE: "200", ds.GPU_MEMORY_RATIO: "200"}))
             for i in range(3)]
    devs = [ds.Device(name=f"n{i}", devices=[ds.DeviceInfo(ds.GPU, m, True, G.rlist(
        {ds.GPU_CORE: "100", ds.GPU_MEMORY_RATIO: "100", ds.GPU_MEMORY: "8Gi"})) for m in range(2)]) for i in range(3)]
    alloc_r = {"gpu": [{"minor": 0, "resources": {ds.GPU_CORE: "100", ds.GPU_MEMORY_RATIO: "100",
                                                  ds.GPU_MEMORY: "8Gi"}}]}
    owner = rv.ReservationOwner(label_selector=rv.LabelSelector(match_labels={"app": "web"}))
    r = rv.Reservation("r-web", "n0", uid="ruid-1", owners=[owner], allocate_once=False,
                       allocatable=G.rlist({"cpu": "4", "memory": "8Gi", ds.GPU_CORE: "100",
                                            ds.GPU_MEMORY_RATIO: "100"}),
                       annotations={ds.ANNOTATION_DEVICE_ALLOCATED: _json.dumps(alloc_r)})
    half = {"gpu": [{"minor": 0, "resources": {ds.GPU_CORE: "50", ds.GPU_MEMORY_RATIO: "50", ds.GPU_MEMORY: "4Gi"}}]}
    assigned = k8s.Pod(name="web-old", uid="w-old", node_name="n0", labels={"app": "web"},
                       annotations={ds.ANNOTATION_DEVICE_ALLOCATED: _json.dumps(half),
                                    rv.ANNOTATION_RESERVATION_ALLOCATED: _json.dumps({"uid": "ruid-1", "name": "r-web"})},
                       containers=[k8s.Container(requests=G.rlist({"cpu": "1", "memory": "1Gi", ds.GPU_CORE: "50",
                                                                   ds.GPU_MEMORY_RATIO: "50"}))])
    return prof, nodes, devs, r, assigned


def test_device_holding_reservation_object_path():
    """Reservation + Device + Pod objects -> Informer -> the device-holding
    reservation columns: the reserve pod (NodeInfo / nodeDevice pod) holds GPU 0,
    the assigned pod's half lies on it (allocated), the reservation's scalar
    Allocatable / Allocated come from its Allocatable and the assigned pod's
    requests masked to its keys; the node's Requested scalars hold both pods.
    The oracle's cycle over that snapshot places a web pod asking for a whole
    GPU in the gpu-core + ratio form on n0 only through the restore -- and the
    informer's row deltas after the assigned pod leaves equal a rebuild."""
    from koordinator_amd import deviceshare as ds
    from koordinator_amd.informer import Informer
    prof, nodes, devs, r, assigned = _object_cluster()
    inf = Informer(prof, nodes, 0.0)
    for d in devs:
        inf.on_device(d)
    inf.on_reservation(r)
    inf.on_pod_add(assigned, 0.0)
    t = inf.table(0.0)
    G_ = abi.DEV_GPU
    assert int(t["resv_dev_slot"][0]) == 0 and (t["resv_dev_slot"][1:] == -1).all()
    assert t["resv_dev"][0, 0, G_, 0].tolist() == FULL and t["resv_dev"][0, 1, G_, 0].tolist() == HALF
    jc, jr = ds.XRES_INDEX[ds.GPU_CORE], ds.XRES_INDEX[ds.GPU_MEMORY_RATIO]
    assert int(t["resv_xalloc"][0, jc]) == 100 and int(t["resv_xallocated"][0, jc]) == 50
    assert int(t["xrequested"][0, jc]) == 150 and int(t["xrequested"][0, jr]) == 150
    assert t["dev_used"][0, G_, 0].tolist() == [150, 150, 12 * GIB]
    assert int(t["resv_assigned"][0]) == 1 and int(t["resv_allocated0"][0]) == 1000
    # fill n1 and n2's GPUs so only n0's restore can host the pod
    web = G.resv_pod({"cpu": "1", ds.GPU_CORE: "100", ds.GPU_MEMORY_RATIO: "100"}, labels={"app": "web"}, name="web")
    recs = inf.pod_records([web])
    ext = inf.pod_ext_records([web])
    t["xrequested"][1:, jc] = 200
    t["xrequested"][1:, jr] = 200
    o = oracle.Oracle(to_c_config(prof), t)
    assert o.place_stream_ext(recs, ext)[0] == 0
    # the assigned pod leaves: a row delta (the allocated half / scalar Allocated go back to 0)
    class _RowsEngine:           # applies every column of the rows (the device columns too)
        def __init__(self, table):
            self.table = table.copy()

        def update_nodes(self, idx, rows):
            for c in rows.cols:
                self.table.cols[c][idx] = rows.cols[c]
    t0 = inf.table(0.0)
    eng = _RowsEngine(t0)
    inf.attach(t0, 0.0)
    inf.on_pod_delete(assigned)
    res = inf.flush(eng, 0.0)
    assert not res.needs_reload
    want = inf.table(0.0)
    for c in ("resv_dev_slot", "resv_dev", "resv_xalloc", "resv_xallocated", "xrequested", "dev_used",
              "resv_assigned", "resv_allocated0"):
        assert np.array_equal(eng.table.cols[c], want.cols[c]), c
    assert int(want["resv_xallocated"][0, jc]) == 0 and not want["resv_dev"][0, 1].any()


@pytest.mark.gpu
def test_update_rows_replace_device_reservation_slot():
    """row updates carrying the reservation columns
    replace the node's whole reservation state.  Rows without the
    device-holding columns clear the node's slot, device allocation and scalars
    (a CPU-only reservation moving into slot h does not inherit the old one's
    devices); rows carrying them replace them.  Streams after the update equal
    the oracle on the updated table."""
    import torch  # noqa: F401
    from koordinator_amd.engine import PlacementEngine
    prof, t = _dev_resv_cluster(160, seed=45)
    pods, ext = _dev_resv_pods(300, prof, seed=45)
    held = np.flatnonzero(t["resv_dev_slot"] >= 0)
    assert held.size >= 8
    t2 = t.copy()
    clear, keep = held[:4], held[4:8]
    for i in clear:                    # a CPU-only reservation in the slot now
        t2["resv_dev_slot"][i] = -1
        t2["resv_dev"][i] = 0
        t2["resv_xalloc"][i] = 0
        t2["resv_xallocated"][i] = 0
    for i in keep:                     # the same reservation, its assigned pods gone
        t2["resv_dev"][i, 1] = 0
        t2["resv_xallocated"][i] = 0
        t2["resv_assigned"][i] = 0
    o = oracle.Oracle(to_c_config(prof), t2)
    ref = o.place_stream_ext(pods, ext)
    with PlacementEngine(prof, device=0) as e:
        e.load_snapshot(t)
        e.update_nodes(clear, t2.rows(clear))      # rows without resv_dev columns (none held): cleared
        e.update_nodes(keep, t2.rows(keep))        # rows carrying them: replaced
        assert np.array_equal(e.read_resv_devices(), t2["resv_dev"])
        assert np.array_equal(e.read_resv_scalars(), t2["resv_xallocated"])
        got = e.place_stream_ext(pods, ext)
        grd = e.read_resv_devices()
    bad = np.flatnonzero(got != ref)
    assert bad.size == 0, f"first mismatch at pod {bad[0]}: hip {got[bad[0]]} oracle {ref[bad[0]]}"
    assert np.array_equal(grd, o.resv_dev_state())
