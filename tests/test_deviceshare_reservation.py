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
