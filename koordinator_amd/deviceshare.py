"""DeviceShare on the host: the plugin's PreFilter products per pod
(koordhip_pod_ext) and the node device columns (dev_*), plus the extended
scalar resources NodeResourcesFit checks for device pods.

  PreparePod / ValidateDeviceRequest / ConvertDeviceRequest
      pkg/scheduler/plugins/deviceshare/plugin.go:162-182, utils.go:86-181
  nodeDevice (deviceTotal / deviceUsed per minor)
      device_cache.go:44-50, buildDeviceResources :550-568
  the pods' device allocations (annotation scheduling.koordinator.sh/device-allocated)
      apis/extension/device_share.go, pod_handler.go

The device side (Filter, Score, Reserve) runs in libkoordhip.so's
sequential cycle (csrc/dev.hpp); the checker is oracle/dev_oracle.c.
"""
from __future__ import annotations

import json
from dataclasses import dataclass, field
from typing import Dict, Iterable, List, Optional, Tuple

import numpy as np

from . import abi, k8s

DOMAIN = "koordinator.sh/"
NVIDIA_GPU = "nvidia.com/gpu"
HYGON_DCU = "dcu.com/gpu"
KOORD_GPU = DOMAIN + "gpu"
GPU_CORE = DOMAIN + "gpu-core"
GPU_MEMORY = DOMAIN + "gpu-memory"
GPU_MEMORY_RATIO = DOMAIN + "gpu-memory-ratio"
RDMA = DOMAIN + "rdma"
FPGA = DOMAIN + "fpga"

# NodeResourcesFit's extended scalar slots (koordhip_pod_ext.xreq, xalloc columns)
XRES = [NVIDIA_GPU, HYGON_DCU, KOORD_GPU, GPU_CORE, GPU_MEMORY, GPU_MEMORY_RATIO, RDMA, FPGA]
XRES_INDEX = {n: j for j, n in enumerate(XRES)}
assert len(XRES) == abi.NXRES

GPU, RDMA_T, FPGA_T = "gpu", "rdma", "fpga"
TYPE_INDEX = {GPU: abi.DEV_GPU, RDMA_T: abi.DEV_RDMA, FPGA_T: abi.DEV_FPGA}
# DeviceResourceNames, device_resources.go:42-53
DEVICE_RESOURCE_NAMES = {
    GPU: [NVIDIA_GPU, HYGON_DCU, KOORD_GPU, GPU_CORE, GPU_MEMORY, GPU_MEMORY_RATIO],
    RDMA_T: [RDMA],
    FPGA_T: [FPGA],
}
# the per-type resource slots of the device columns (KOORDHIP_DEV_RES)
TYPE_RESOURCES = {GPU: [GPU_CORE, GPU_MEMORY_RATIO, GPU_MEMORY], RDMA_T: [RDMA], FPGA_T: [FPGA]}

# DeviceResourceFlags / ValidDeviceResourceCombinations, device_resources.go:31-76
F_NVIDIA, F_HYGON, F_KOORD_GPU, F_CORE, F_MEM, F_RATIO, F_FPGA, F_RDMA = (1 << i for i in range(8))
FLAGS = {NVIDIA_GPU: F_NVIDIA, HYGON_DCU: F_HYGON, KOORD_GPU: F_KOORD_GPU, GPU_CORE: F_CORE, GPU_MEMORY: F_MEM,
         GPU_MEMORY_RATIO: F_RATIO, FPGA: F_FPGA, RDMA: F_RDMA}
VALID = {F_NVIDIA, F_HYGON, F_KOORD_GPU, F_MEM, F_RATIO, F_CORE | F_MEM, F_CORE | F_RATIO, F_FPGA, F_RDMA}
PERCENTAGE = {KOORD_GPU, GPU_CORE, GPU_MEMORY_RATIO, FPGA, RDMA}   # DeviceResourceValidators

ANNOTATION_DEVICE_ALLOCATED = "scheduling.koordinator.sh/device-allocated"


class DeviceRequestError(ValueError):
    """PreFilter returns framework.Error (ValidateDeviceRequest)."""


def _value(q: k8s.Quantity) -> int:
    return q.value()


def validate_device_request(req: Dict[str, k8s.Quantity]) -> int:
    """ValidateDeviceRequest, utils.go:148-169."""
    if not req:
        raise DeviceRequestError("pod request should not be empty")
    comb = 0
    for name, q in req.items():
        comb |= FLAGS.get(name, 0)
        if name in PERCENTAGE:
            v = _value(q)
            if v > 100 and v % 100 != 0:
                raise DeviceRequestError(f"invalid resource unit {name}: {v}")
    if comb not in VALID:
        raise DeviceRequestError(f"invalid resource device requests: {sorted(req)}")
    return comb


def convert_device_request(req: Dict[str, k8s.Quantity], comb: int) -> Dict[str, int]:
    """ConvertDeviceRequest + ResourceCombinationsMapper, utils.go:86-139,171-181
    (values as Quantity.Value())."""
    v = lambda n: _value(req[n]) if n in req else 0
    if comb == F_MEM:
        return {GPU_MEMORY: v(GPU_MEMORY)}
    if comb == F_RATIO:
        return {GPU_MEMORY_RATIO: v(GPU_MEMORY_RATIO)}
    if comb == F_CORE | F_MEM:
        return {GPU_CORE: v(GPU_CORE), GPU_MEMORY: v(GPU_MEMORY)}
    if comb == F_CORE | F_RATIO:
        return {GPU_CORE: v(GPU_CORE), GPU_MEMORY_RATIO: v(GPU_MEMORY_RATIO)}
    if comb == F_KOORD_GPU:
        return {GPU_CORE: v(KOORD_GPU), GPU_MEMORY_RATIO: v(KOORD_GPU)}
    if comb == F_NVIDIA:
        return {GPU_CORE: v(NVIDIA_GPU) * 100, GPU_MEMORY_RATIO: v(NVIDIA_GPU) * 100}
    if comb == F_HYGON:
        return {GPU_CORE: v(HYGON_DCU) * 100, GPU_MEMORY_RATIO: v(HYGON_DCU) * 100}
    if comb == F_FPGA:
        return {FPGA: v(FPGA)}
    if comb == F_RDMA:
        return {RDMA: v(RDMA)}
    return {}


def prepare_pod(pod: k8s.Pod) -> Tuple[bool, Dict[str, int]]:
    """PreparePod, plugin.go:162-182: (skip, the converted device requests)."""
    requests, _ = k8s.pod_requests_and_limits(pod)
    requests = {n: q for n, q in requests.items() if not q.is_zero()}   # quotav1.RemoveZeros
    skip, out = True, {}
    for typ, names in DEVICE_RESOURCE_NAMES.items():
        masked = {n: requests[n] for n in names if n in requests}
        if not masked:
            continue
        comb = validate_device_request(masked)
        for n, x in convert_device_request(masked, comb).items():
            out[n] = out.get(n, 0) + x
        skip = False
    return skip, out


def fit_xreq(pod: k8s.Pod) -> Dict[str, int]:
    """The pod's extended scalar requests as upstream computePodResourceRequest
    sums them: containers added, init containers max'ed, overhead added
    (UPSTREAM-ASSUMED, like marshal.fit_request)."""
    acc: Dict[str, int] = {}
    for c in pod.containers:
        for n, q in c.requests.items():
            if n in XRES_INDEX:
                acc[n] = acc.get(n, 0) + q.value()
    for c in pod.init_containers:
        for n, q in c.requests.items():
            if n in XRES_INDEX:
                acc[n] = max(acc.get(n, 0), q.value())
    for n, q in (pod.overhead or {}).items():
        if n in XRES_INDEX:
            acc[n] = acc.get(n, 0) + q.value()
    return acc


def pod_ext_record(pod: k8s.Pod, out: Optional[np.ndarray] = None) -> np.ndarray:
    """One koordhip_pod_ext record: the DeviceShare PreFilter products and the
    extended scalar requests."""
    rec = out if out is not None else abi.pod_ext_array(1)[0]
    rec["dev_req"][:] = 0
    rec["dev_req"][abi.DEV_GPU, :] = -1
    skip, req = prepare_pod(pod)
    flags = 0
    if not skip:
        flags |= abi.PODX_DEVICE
        g = rec["dev_req"][abi.DEV_GPU]
        if GPU_CORE in req:
            g[0] = req[GPU_CORE]
        if GPU_MEMORY_RATIO in req:
            g[1] = req[GPU_MEMORY_RATIO]
        if GPU_MEMORY in req:
            g[2] = req[GPU_MEMORY]
        rec["dev_req"][abi.DEV_RDMA, 0] = req.get(RDMA, 0)
        rec["dev_req"][abi.DEV_FPGA, 0] = req.get(FPGA, 0)
    rec["flags"] = flags
    xr = fit_xreq(pod)
    rec["xmask"] = 0
    rec["xreq"][:] = 0
    for n, v in xr.items():
        j = XRES_INDEX[n]
        rec["xreq"][j] = v
        rec["xmask"] |= 1 << j
    return rec


def pod_ext_records(pods: Iterable[k8s.Pod]) -> np.ndarray:
    pods = list(pods)
    arr = abi.pod_ext_array(len(pods))
    for i, p in enumerate(pods):
        pod_ext_record(p, arr[i])
    return arr


# ---------------------------------------------------------------------------
# Node side

@dataclass
class DeviceInfo:
    """schedulingv1alpha1.DeviceInfo (apis/scheduling/v1alpha1/device_types.go)."""
    type: str                     # gpu / rdma / fpga
    minor: int
    health: bool = True
    resources: Dict[str, k8s.Quantity] = field(default_factory=dict)


@dataclass
class Device:
    """schedulingv1alpha1.Device: one per node (its name is the node's)."""
    name: str
    devices: List[DeviceInfo] = field(default_factory=list)


def device_rows(table, i: int, dev: Optional[Device], allocations: Iterable[Dict[str, List[Tuple[int, Dict[str, int]]]]] = ()):
    """Row i of the dev_* columns: the Device CR's minors per type (ascending;
    an unhealthy device has no resources, buildDeviceResources
    device_cache.go:550-568) and deviceUsed from the pods' allocations
    ({type: [(minor, {resource: value})]}, updateCacheUsed :116-127).
    dev None = no nodeDevice entry."""
    S = table.dev_slots
    table["dev_present"][i] = 0
    table["dev_minor"][i] = -1
    table["dev_total"][i] = 0
    table["dev_used"][i] = 0
    if dev is None:
        return
    table["dev_present"][i] = 1
    by_type: Dict[str, List[DeviceInfo]] = {}
    for d in dev.devices:
        if d.type not in TYPE_INDEX:
            raise ValueError(f"device type {d.type!r} is not supported (gpu, rdma, fpga)")
        by_type.setdefault(d.type, []).append(d)
    slot_of: Dict[Tuple[str, int], int] = {}
    for typ, ds in by_type.items():
        ds = sorted(ds, key=lambda d: d.minor)
        if len(ds) > S:
            raise ValueError(f"node {dev.name}: more than {S} {typ} devices (the table's dev_slots)")
        t = TYPE_INDEX[typ]
        for s, d in enumerate(ds):
            table["dev_minor"][i, t, s] = d.minor
            slot_of[(typ, d.minor)] = s
            if d.health:
                names = TYPE_RESOURCES[typ]
                extra = set(d.resources) - set(names)
                if extra:
                    raise ValueError(f"device {typ}/{d.minor}: resources {sorted(extra)} not supported")
                for r, n in enumerate(names):
                    table["dev_total"][i, t, s, r] = d.resources[n].value() if n in d.resources else 0
                if typ == GPU and table["dev_total"][i, t, s].any() and not table["dev_total"][i, t, s, 2]:
                    raise ValueError(f"GPU {d.minor} of node {dev.name} has no {GPU_MEMORY}")
    for alloc in allocations:
        for typ, items in alloc.items():
            t = TYPE_INDEX[typ]
            for minor, res in items:
                s = slot_of.get((typ, minor))
                if s is None:
                    continue   # a minor the Device CR no longer lists: deviceFree has no resources there
                for r, n in enumerate(TYPE_RESOURCES[typ]):
                    table["dev_used"][i, t, s, r] += res.get(n, 0)


def parse_device_allocated(annotations: Dict[str, str]) -> Dict[str, List[Tuple[int, Dict[str, int]]]]:
    """apiext.GetDeviceAllocations: {type: [{minor, resources}]} (Quantity strings)."""
    raw = (annotations or {}).get(ANNOTATION_DEVICE_ALLOCATED)
    if not raw:
        return {}
    data = json.loads(raw)
    out = {}
    for typ, items in data.items():
        out[typ] = [(int(x.get("minor", 0)), {n: k8s.Quantity(v).value() for n, v in (x.get("resources") or {}).items()})
                    for x in items]
    return out


def slot_minors(table, i: int, slots: np.ndarray) -> Dict[str, List[int]]:
    """koordhip_fetch_devices masks of one pod -> {type: [minor]} on node i."""
    out = {}
    for typ, t in TYPE_INDEX.items():
        m = int(slots[t])
        if m:
            out[typ] = [int(table["dev_minor"][i, t, s]) for s in range(table.dev_slots) if (m >> s) & 1]
    return out
