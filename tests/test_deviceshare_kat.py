"""DeviceShare known-answer tests transcribed from the reference's
deviceshare/{scoring,plugin,utils}_test.go (tests/golden/deviceshare_cases.json,
each case with its file:line): on the oracle (CPU) and, marked gpu, through
libkoordhip.so's sequential cycle (eval_ext planes / status, place_stream_ext
device allocations and deviceUsed)."""
import numpy as np
import pytest

import oracle
from golden_cases import load
from koordinator_amd import abi, deviceshare as ds, k8s, synth
from koordinator_amd.config import (DeviceShareArgs, Profile, PLUGIN_DEVICESHARE, to_c_config)
from koordinator_amd.snapshot import NodeTable

CASES = load("deviceshare_cases.json")
TYPES = {"gpu": abi.DEV_GPU, "rdma": abi.DEV_RDMA, "fpga": abi.DEV_FPGA}
GPU_RES = ["gpu-core", "gpu-memory-ratio", "gpu-memory"]


def profile(most=False):
    return Profile(filters=(PLUGIN_DEVICESHARE,), scores={PLUGIN_DEVICESHARE: 1},
                   deviceshare=DeviceShareArgs(scoring_type="MostAllocated" if most else "LeastAllocated"))


def node_table(spec, slots=4, n=1):
    """n identical nodes of the case's device state (minor, total, used)."""
    t = NodeTable.empty(n)
    t.cols["alloc_pods"][:] = 110
    t.enable_ext(dev_slots=slots)
    t["dev_present"][:] = 1 if spec["present"] else 0
    for typ, items in (("gpu", spec["gpu"]), ("rdma", spec["rdma"]), ("fpga", spec["fpga"])):
        ti = TYPES[typ]
        for s, (minor, total, used) in enumerate(items):
            t["dev_minor"][:, ti, s] = minor
            if typ == "gpu":
                t["dev_total"][:, ti, s] = [total[r] for r in GPU_RES]
                t["dev_used"][:, ti, s] = [used[r] for r in GPU_RES]
            else:
                t["dev_total"][:, ti, s, 0] = total
                t["dev_used"][:, ti, s, 0] = used
    return t


def ext_of(req):
    """koordhip_pod_ext of a converted device request (the preFilterState's podRequests)."""
    x = abi.pod_ext_array(1)
    x["flags"] = abi.PODX_DEVICE
    g = x["dev_req"][0, abi.DEV_GPU]
    for r, name in enumerate(GPU_RES):
        if name in req:
            g[r] = req[name]
    x["dev_req"][0, abi.DEV_RDMA, 0] = req.get("rdma", 0)
    x["dev_req"][0, abi.DEV_FPGA, 0] = req.get("fpga", 0)
    return x


def pod_rec():
    p = np.zeros(1, abi.POD_DTYPE)
    return p


def minors_of(t, slots):
    return {typ: [int(t["dev_minor"][0, TYPES[typ], s]) for s in range(t.dev_slots) if (int(slots[TYPES[typ]]) >> s) & 1]
            for typ in TYPES if int(slots[TYPES[typ]])}


@pytest.mark.parametrize("c", CASES["score"], ids=lambda c: c["src"])
def test_score_kat_oracle(c):
    t = node_table(c["node"])
    o = oracle.Oracle(to_c_config(profile(c.get("most", False))), t)
    assert o.dev_score(ext_of(c["req"]), 0) == c["want"]


@pytest.mark.parametrize("c", CASES["score_device"], ids=lambda c: c["src"])
def test_score_device_kat_oracle(c):
    """scoreDevice of one device = scoreNode of a node with that one device."""
    used = c["total"] - c["free"]
    spec = {"present": True, "gpu": [(0, {"gpu-core": 100, "gpu-memory-ratio": c["total"], "gpu-memory": 1 << 34},
                                      {"gpu-core": 0, "gpu-memory-ratio": used, "gpu-memory": 0})], "rdma": [], "fpga": []}
    o = oracle.Oracle(to_c_config(profile(c.get("most", False))), node_table(spec))
    assert o.dev_score(ext_of({"gpu-memory-ratio": c["req"]}), 0) == c["want"]


@pytest.mark.parametrize("c", CASES["normalize"], ids=lambda c: c["src"])
def test_normalize_kat(c):
    assert oracle.default_normalize(c["scores"]).tolist() == c["want"]


@pytest.mark.parametrize("c", CASES["filter"], ids=lambda c: c["src"])
def test_filter_kat_oracle(c):
    o = oracle.Oracle(to_c_config(profile()), node_table(c["node"]))
    assert o.dev_filter(ext_of(c["req"]), 0) == c["pass"]


def _check_used(t, used_after, want):
    for typ, per in want.items():
        ti = TYPES[typ]
        for minor, v in per.items():
            s = [q for q in range(t.dev_slots) if int(t["dev_minor"][0, ti, q]) == int(minor)][0]
            exp = [v[r] for r in GPU_RES] if typ == "gpu" else [v, 0, 0]
            assert used_after[0, ti, s].tolist() == exp, (typ, minor)


@pytest.mark.parametrize("c", CASES["reserve"], ids=lambda c: c["src"])
def test_reserve_kat_oracle(c):
    t = node_table(c["node"])
    o = oracle.Oracle(to_c_config(profile()), t)
    ok, slots = o.dev_reserve(ext_of(c["req"]), 0)
    assert ok == c["ok"]
    if ok:
        assert minors_of(t, slots) == c["minors"]
        _check_used(t, o.dev_state()["dev_used"], c["used"])


@pytest.mark.parametrize("c", CASES["validate"], ids=lambda c: c["src"])
def test_validate_device_request(c):
    req = {n: k8s.Quantity(v) for n, v in c["req"].items()}
    if c.get("err"):
        with pytest.raises(ds.DeviceRequestError):
            ds.validate_device_request(req)
    else:
        assert ds.validate_device_request(req) == c["want"]


@pytest.mark.parametrize("c", CASES["convert"], ids=lambda c: c["src"])
def test_convert_device_request(c):
    req = {n: k8s.Quantity(v) for n, v in c["req"].items()}
    assert ds.convert_device_request(req, c["comb"]) == c["want"]


@pytest.mark.parametrize("c", CASES["fill"], ids=lambda c: c["src"])
def test_fill_gpu_total_mem_oracle(c):
    """fillGPUTotalMem: the Reserve of the request on one free GPU adds the filled request."""
    spec = {"present": True, "gpu": [(0, {"gpu-core": 100, "gpu-memory-ratio": 100, "gpu-memory": c["total_mem"]},
                                      {"gpu-core": 0, "gpu-memory-ratio": 0, "gpu-memory": 0})], "rdma": [], "fpga": []}
    t = node_table(spec)
    o = oracle.Oracle(to_c_config(profile()), t)
    ok, _ = o.dev_reserve(ext_of(c["req"]), 0)
    assert ok
    assert o.dev_state()["dev_used"][0, abi.DEV_GPU, 0].tolist() == [c["want"][r] for r in GPU_RES]


@pytest.mark.parametrize("c", CASES["multiple"], ids=lambda c: c["src"])
def test_multiple_devices_oracle(c):
    """isPodRequestsMultipleDevice: the Reserve takes that many devices (4 free ones of the type)."""
    dev = [(m, {"gpu-core": 100, "gpu-memory-ratio": 100, "gpu-memory": 16 << 30},
            {"gpu-core": 0, "gpu-memory-ratio": 0, "gpu-memory": 0}) if c["type"] == "gpu" else (m, 100, 0)
           for m in range(4)]
    spec = {"present": True, "gpu": [], "rdma": [], "fpga": []}
    spec[c["type"]] = dev
    t = node_table(spec)
    o = oracle.Oracle(to_c_config(profile()), t)
    ok, slots = o.dev_reserve(ext_of(c["req"]), 0)
    v = list(c["req"].values())[0]
    want = v // 100 if c["want"] else 1
    assert ok and bin(int(slots[TYPES[c["type"]]])).count("1") == want


def test_prepare_pod_objects():
    """PreparePod on pod objects: the converted request and its ext record."""
    p = k8s.Pod(name="g", containers=[k8s.Container(requests={ds.NVIDIA_GPU: k8s.Quantity(2), ds.RDMA: k8s.Quantity(100)})])
    skip, req = ds.prepare_pod(p)
    assert not skip and req == {ds.GPU_CORE: 200, ds.GPU_MEMORY_RATIO: 200, ds.RDMA: 100}
    x = ds.pod_ext_record(p)
    assert x["flags"] == abi.PODX_DEVICE and x["dev_req"][abi.DEV_GPU].tolist() == [200, 200, -1]
    assert x["dev_req"][abi.DEV_RDMA, 0] == 100
    assert x["xmask"] == (1 << ds.XRES_INDEX[ds.NVIDIA_GPU]) | (1 << ds.XRES_INDEX[ds.RDMA])
    assert ds.prepare_pod(k8s.Pod(name="c", containers=[k8s.Container(requests={k8s.CPU: k8s.Quantity(1)})]))[0]


# ------------------------------------------------------------------- GPU (libkoordhip.so)
@pytest.mark.gpu
@pytest.mark.parametrize("c", CASES["score"] + CASES["filter"], ids=lambda c: "gpu-" + c["src"])
def test_score_filter_kat_gpu(c):
    import torch  # noqa: F401
    from koordinator_amd.engine import PlacementEngine
    t = node_table(c["node"])
    with PlacementEngine(profile(c.get("most", False)), device=0) as e:
        e.load_snapshot(t)
        r = e.eval_ext(pod_rec(), ext_of(c["req"]))
    if "want" in c:
        assert int(r["scores"][0, abi.NPLUGINS + 0, 0]) == c["want"]
    else:
        assert (int(r["status"][0, 0]) & abi.ST_DEVICE_FAIL == 0) == c["pass"]


@pytest.mark.gpu
@pytest.mark.parametrize("c", CASES["reserve"] + [dict(x, fill=True) for x in CASES["fill"]],
                         ids=lambda c: "gpu-" + c["src"])
def test_reserve_kat_gpu(c):
    import torch  # noqa: F401
    from koordinator_amd.engine import PlacementEngine
    if c.get("fill"):
        node = {"present": True, "gpu": [(0, {"gpu-core": 100, "gpu-memory-ratio": 100, "gpu-memory": c["total_mem"]},
                                          {"gpu-core": 0, "gpu-memory-ratio": 0, "gpu-memory": 0})], "rdma": [], "fpga": []}
    else:
        node = c["node"]
    t = node_table(node)
    with PlacementEngine(profile(), device=0) as e:
        e.load_snapshot(t)
        out = e.place_stream_ext(pod_rec(), ext_of(c["req"]))
        slots = e.fetch_devices(1)[0]
        used = e.read_devices()["dev_used"]
    if c.get("fill"):
        assert out[0] == 0
        assert used[0, abi.DEV_GPU, 0].tolist() == [c["want"][r] for r in GPU_RES]
        return
    assert (out[0] == 0) == c["ok"]
    if c["ok"]:
        assert minors_of(t, slots) == c["minors"]
        _check_used(t, used, c["used"])
