"""Snapshot marshaller: Kubernetes objects -> koordhip SoA rows and pod records.

This is the host half of the drop-in boundary (what the Go shim does before
crossing cgo).  Everything that depends on wall-clock time, listers or JSON
annotations is resolved here ONCE per snapshot at time `now`; the device only
sees integers.  Each rule cites the reference line it restates.
"""
from __future__ import annotations

import json
from dataclasses import dataclass, field
from typing import Dict, Iterable, List, Optional, Set, Tuple

import numpy as np

from . import abi, numa, k8s
from .config import PLUGIN_RESERVATION, LoadAwareSchedulingArgs, Profile
from .snapshot import NodeTable, pod_array

DEFAULT_MILLI_CPU_REQUEST = 250                 # estimator/default_estimator.go:35-38
DEFAULT_MEMORY_REQUEST = 200 * 1024 * 1024
NONZERO_DEFAULT_MILLI_CPU = 100                 # (upstream) scheduler/util/pod_resources.go
NONZERO_DEFAULT_MEMORY = 200 * 1024 * 1024
DEFAULT_REPORT_INTERVAL_S = 60.0                # load_aware.go:56


class MarshalError(ValueError):
    pass


class NewTopologyValue(MarshalError):
    """A node's topology label value has no domain in the loaded snapshot: rebuild it."""


# ---------------------------------------------------------------------------
# Pod side (PreFilter products)

def estimated_used_by_resource(requests, limits, name: str, factor: int) -> int:
    """estimatedUsedByResource, estimator/default_estimator.go:73-108."""
    lim = limits.get(name, k8s.Quantity(0))
    req = requests.get(name, k8s.Quantity(0))
    if lim.cmp(req) > 0:
        factor, q = 100, lim
    else:
        q = req
    if q.is_zero():
        if name in (k8s.CPU, k8s.BATCH_CPU):
            return DEFAULT_MILLI_CPU_REQUEST
        if name in (k8s.MEMORY, k8s.BATCH_MEMORY):
            return DEFAULT_MEMORY_REQUEST
        return 0
    if name == k8s.CPU:
        est = k8s.round_half_away(float(q.milli_value()) * float(factor) / 100)
        limit = lim.milli_value()
    else:
        est = k8s.round_half_away(float(q.value()) * float(factor) / 100)
        limit = lim.value()
    if limit > 0 and est > limit:
        est = limit
    return est


def estimate_pod(pod: k8s.Pod, args: LoadAwareSchedulingArgs) -> Dict[str, int]:
    """DefaultEstimator.EstimatePod, default_estimator.go:57-70."""
    requests, limits = k8s.pod_requests_and_limits(pod)
    pc = k8s.priority_class(pod)
    out = {}
    for name in args.resource_weights:
        real = k8s.translate_resource(pc, name)
        out[name] = estimated_used_by_resource(requests, limits, real, args.estimated_scaling_factors.get(name, 0))
    return out


_NATIVE_FIT = {k8s.CPU: abi.RES_CPU, k8s.MEMORY: abi.RES_MEM, k8s.EPHEMERAL: abi.RES_EPH}
_SCALAR_FIT = {k8s.BATCH_CPU: abi.RES_BCPU, k8s.BATCH_MEMORY: abi.RES_BMEM}
# DeviceShare's resources: NodeResourcesFit checks them as extended scalars
# (koordhip_pod_ext.xreq / the xalloc columns, deviceshare.XRES)
_DEVICE_SCALARS = {"nvidia.com/gpu", "dcu.com/gpu", "koordinator.sh/gpu", "koordinator.sh/gpu-core",
                   "koordinator.sh/gpu-memory", "koordinator.sh/gpu-memory-ratio", "koordinator.sh/rdma",
                   "koordinator.sh/fpga"}


def _is_scalar(name: str) -> bool:
    """(upstream) schedutil.IsScalarResourceName: extended, hugepages, prefixed-native, attachable."""
    return name not in (k8s.CPU, k8s.MEMORY, k8s.EPHEMERAL, k8s.PODS)


def _resource_add(acc: List[int], present: Set[str], rlist: k8s.ResourceList):
    """(upstream) framework.Resource.Add."""
    for n, q in rlist.items():
        if n == k8s.CPU:
            acc[abi.RES_CPU] += q.milli_value()
        elif n == k8s.MEMORY:
            acc[abi.RES_MEM] += q.value()
        elif n == k8s.EPHEMERAL:
            acc[abi.RES_EPH] += q.value()
        elif n == k8s.PODS:
            pass
        elif _is_scalar(n):
            if n in _DEVICE_SCALARS:      # extended scalars: koordhip_pod_ext.xreq (deviceshare.fit_xreq)
                present.add(n)
                continue
            if n not in _SCALAR_FIT:
                raise MarshalError(f"scalar resource {n!r} is not supported by the engine")
            acc[_SCALAR_FIT[n]] += q.value()
            present.add(n)


def _resource_setmax(acc: List[int], present: Set[str], rlist: k8s.ResourceList):
    """(upstream) framework.Resource.SetMaxResource."""
    for n, q in rlist.items():
        if n == k8s.CPU:
            acc[abi.RES_CPU] = max(acc[abi.RES_CPU], q.milli_value())
        elif n == k8s.MEMORY:
            acc[abi.RES_MEM] = max(acc[abi.RES_MEM], q.value())
        elif n == k8s.EPHEMERAL:
            acc[abi.RES_EPH] = max(acc[abi.RES_EPH], q.value())
        elif n == k8s.PODS:
            pass
        elif _is_scalar(n):
            if n in _DEVICE_SCALARS:
                present.add(n)
                continue
            if n not in _SCALAR_FIT:
                raise MarshalError(f"scalar resource {n!r} is not supported by the engine")
            i = _SCALAR_FIT[n]
            acc[i] = max(acc[i], q.value())
            present.add(n)


def fit_request(pod: k8s.Pod) -> Tuple[List[int], Set[str]]:
    """(upstream) noderesources computePodResourceRequest: max(sum containers, each init) + overhead.
    UPSTREAM-ASSUMED."""
    acc = [0] * abi.NRES
    present: Set[str] = set()
    for c in pod.containers:
        _resource_add(acc, present, c.requests)
    for c in pod.init_containers:
        _resource_setmax(acc, present, c.requests)
    if pod.overhead:
        _resource_add(acc, present, pod.overhead)
    return acc, present


def _nonzero(rlist: k8s.ResourceList) -> Tuple[int, int]:
    """(upstream) schedutil.GetNonzeroRequests: unset cpu/memory -> 100m / 200MiB."""
    cpu = rlist[k8s.CPU].milli_value() if k8s.CPU in rlist else NONZERO_DEFAULT_MILLI_CPU
    mem = rlist[k8s.MEMORY].value() if k8s.MEMORY in rlist else NONZERO_DEFAULT_MEMORY
    return cpu, mem


def nonzero_request(pod: k8s.Pod) -> Tuple[int, int]:
    """(upstream) framework calculateResource non0CPU/non0Mem (== resource_allocation
    calculatePodResourceRequest with nonZero=true for cpu/memory). UPSTREAM-ASSUMED."""
    cpu = mem = 0
    for c in pod.containers:
        a, b = _nonzero(c.requests)
        cpu += a
        mem += b
    for c in pod.init_containers:
        a, b = _nonzero(c.requests)
        cpu, mem = max(cpu, a), max(mem, b)
    if pod.overhead:
        if k8s.CPU in pod.overhead:
            cpu += pod.overhead[k8s.CPU].milli_value()
        if k8s.MEMORY in pod.overhead:
            mem += pod.overhead[k8s.MEMORY].value()
    return cpu, mem


def node_static(node: k8s.Node):
    """The node fields the upstream static filters read (nodefilters.NodeStatic)."""
    from .nodefilters import NodeStatic
    return NodeStatic(labels=dict(node.labels or {}), taints=list(node.taints), unschedulable=node.unschedulable,
                      name=node.name)


def pod_static(pod: k8s.Pod, profile: Optional[Profile] = None):
    """The pod fields the upstream static filters read (its static class key);
    spec.nodeName only when `profile` enables the NodeName filter."""
    from .config import PLUGIN_NODE_NAME
    from .nodefilters import PodStatic
    name = pod.node_name if profile is not None and PLUGIN_NODE_NAME in profile.resolved().filters else ""
    return PodStatic(node_selector=dict(pod.node_selector or {}), required_terms=pod.required_node_affinity,
                     tolerations=list(pod.tolerations), preferred_terms=list(pod.preferred_node_affinity or []),
                     node_name=name)


def static_filters_of(profile: Profile) -> List[str]:
    from .config import STATIC_FILTERS
    return [f for f in profile.resolved().filters if f in STATIC_FILTERS]


def static_scores_of(profile: Profile) -> List[str]:
    """The enabled NodeAffinity / TaintToleration Scores (static_score planes)."""
    from .config import PLUGIN_NODE_AFFINITY, PLUGIN_TAINT_TOLERATION
    return [f for f in (PLUGIN_NODE_AFFINITY, PLUGIN_TAINT_TOLERATION) if f in profile.scores]


def static_keyed(profile: Profile) -> bool:
    """Pods carry a static class (static_allow bits and / or static_score columns)."""
    return bool(static_filters_of(profile) or static_scores_of(profile))


def sequential_profile(profile: Profile) -> bool:
    """DeviceShare or a normalized Score: the engine runs the sequential cycle
    and the snapshot carries the ABI 9 columns (NodeTable.enable_ext)."""
    from .config import NORMALIZED_SCORES, PLUGIN_DEVICESHARE, PLUGIN_IPA, PLUGIN_PTS
    return (PLUGIN_DEVICESHARE in profile.filters or PLUGIN_PTS in profile.filters or PLUGIN_IPA in profile.filters
            or any(x in profile.scores for x in NORMALIZED_SCORES))


def _uses(profile: Profile, name: str) -> bool:
    return name in profile.filters or name in profile.scores


def static_class_of(pod: k8s.Pod, profile: Profile, static_classes) -> int:
    """The pod's static class in `static_classes` (nodefilters.StaticClasses).
    Its node bits were computed when the snapshot was built: a class first seen
    after that (index >= static_classes.frozen) has no bits on the device, so
    the snapshot must be rebuilt (MarshalError)."""
    if not static_keyed(profile):
        return 0
    if static_classes is None:
        raise MarshalError("the profile enables static node filters / Scores: pass the snapshot's StaticClasses")
    c = static_classes.classify(pod_static(pod, profile))
    if c >= getattr(static_classes, "frozen", abi.MAX_STATIC_CLASSES):
        raise MarshalError("pod static class first seen after the snapshot was built: rebuild it "
                           "(static_allow / static_score)")
    return c


def pod_record(pod: k8s.Pod, profile: Profile, out: Optional[np.ndarray] = None, resv_index=None,
               static_classes=None, reservations=None) -> np.ndarray:
    """One koordhip_pod record for `pod` (the per-pod PreFilter products);
    `resv_index` (reservation.ReservationIndex): the snapshot's reservation
    owner groups the pod is matched against; `static_classes`
    (nodefilters.StaticClasses): the snapshot's pod static classes (required
    when the profile enables NodeUnschedulable / NodeAffinity / TaintToleration);
    `reservations` (name -> reservation.Reservation): the reservations reserve
    pods belong to (required for a reserve pod when the profile enables the
    Reservation plugin; a pinned reserve pod's node goes in its
    koordhip_pod_ext record, pod_ext_records)."""
    p = profile.resolved()
    rec = out if out is not None else pod_array(1)[0]
    req, present = fit_request(pod)
    if present & _DEVICE_SCALARS and not sequential_profile(p):
        # NodeResourcesFit checks them through koordhip_pod_ext.xreq, which only
        # the sequential cycle reads (place_stream_ext / eval_ext)
        raise MarshalError(f"pod {pod.key} requests device resources {sorted(present & _DEVICE_SCALARS)}: "
                           "the profile needs DeviceShare (the sequential cycle)")
    rec["req"][:] = req
    nzc, nzm = nonzero_request(pod)
    rec["nz_cpu_m"], rec["nz_mem"] = nzc, nzm
    est = estimate_pod(pod, p.loadaware)
    rec["est_cpu"] = est.get(k8s.CPU, 0)
    rec["est_mem"] = est.get(k8s.MEMORY, 0)
    flags = 0
    if k8s.priority_class(pod) == k8s.PRIORITY_PROD:
        flags |= abi.POD_PROD
    if k8s.is_daemonset_pod(pod):
        flags |= abi.POD_DAEMONSET
    if req[abi.RES_CPU] or req[abi.RES_MEM] or req[abi.RES_EPH] or present:
        flags |= abi.POD_HAS_REQ
    if k8s.BATCH_CPU in present:
        flags |= abi.POD_REQ_BCPU
    if k8s.BATCH_MEMORY in present:
        flags |= abi.POD_REQ_BMEM
    # NodeNUMAResource PreFilter (plugin.go:210-260, AllowUseCPUSet util.go:48-55)
    allow = k8s.qos_class_raw(pod) in (k8s.QOS_LSE, k8s.QOS_LSR) and k8s.priority_class(pod) == k8s.PRIORITY_PROD
    zero = not (any(req) or present)
    try:
        nf, ncpus, pol = numa.prefilter_state(pod.annotations or {}, allow, int(req[abi.RES_CPU]), zero,
                                              p.numa.default_cpu_bind_policy)
    except numa.PreFilterError:
        nf, ncpus, pol = abi.POD_NUMA_ERROR, 0, 0
    from . import reservation as rv
    flags |= rv.pod_keys(pod)
    rec["flags"] = flags | nf | (abi.POD_CPUSET_QOS if allow else 0)
    rec["numa_cpus"] = ncpus
    rec["numa_policy"] = pol
    rec["resv_match"] = resv_index.pod_mask(pod) if resv_index is not None else 0
    rec["static_class"] = static_class_of(pod, profile, static_classes)
    if rv.is_reservation_operating_pod(pod) and not rv.is_reserve_pod(pod) and _uses(p, PLUGIN_RESERVATION):
        # the Reservation Filter's Aligned policy check (reservation/plugin.go:332-357)
        rec["flags"] = int(rec["flags"]) | abi.POD_RESV_OPERATING | (abi.RESV_POLICY_ALIGNED << abi.POD_RESERVE_POLICY_SHIFT)
    if rv.is_reserve_pod(pod) and _uses(p, PLUGIN_RESERVATION):
        if reservations is None:
            raise MarshalError(f"reserve pod {pod.key}: pass the reservations (name -> Reservation)")
        rv.reserve_pod_fields(rec, None, pod, reservations, {})
    return rec


def pod_records(pods: Iterable[k8s.Pod], profile: Profile, resv_index=None, static_classes=None,
                reservations=None) -> np.ndarray:
    pods = list(pods)
    arr = pod_array(len(pods))
    for i, p in enumerate(pods):
        pod_record(p, profile, arr[i], resv_index, static_classes, reservations)
    return arr


def static_classes_for(pods: Iterable[k8s.Pod], profile: Profile):
    """A StaticClasses registry holding the static classes of `pods` (the pods
    a snapshot will schedule), for build_table / pod_records."""
    from .nodefilters import StaticClasses
    sc = StaticClasses()
    if static_keyed(profile):
        for pod in pods:
            sc.classify(pod_static(pod, profile))
    return sc


# ---------------------------------------------------------------------------
# Node side

@dataclass
class AssignedPod:
    """podAssignCache entry (pod_assign_cache.go:40-43)."""
    pod: k8s.Pod
    timestamp: float


@dataclass
class ClusterState:
    """What the plugins read at a scheduling cycle: nodes, NodeMetrics, the pod
    lister, the NodeInfo pods and the LoadAware podAssignCache."""
    nodes: List[k8s.Node] = field(default_factory=list)
    node_metrics: Dict[str, k8s.NodeMetric] = field(default_factory=dict)
    pods: Dict[str, k8s.Pod] = field(default_factory=dict)            # lister, key ns/name
    node_pods: Dict[str, List[k8s.Pod]] = field(default_factory=dict)  # NodeInfo.Pods per node
    assigned: Dict[str, List[AssignedPod]] = field(default_factory=dict)
    devices: Dict[str, object] = field(default_factory=dict)          # Device CRs by node (deviceshare.Device)
    # PodTopologySpread: the registry of the pods to schedule (topologyspread.SpreadRegistry;
    # its topology keys are InterPodAffinity's too)
    spread: object = None
    # InterPodAffinity: the count entries (interpodaffinity.IpaRegistry over `spread`'s keys)
    ipa: object = None


def estimate_node(node: k8s.Node) -> k8s.ResourceList:
    """EstimateNode, default_estimator.go:110-129 (raw-allocatable override)."""
    raw = node.annotations.get(k8s.ANNOTATION_NODE_RAW_ALLOCATABLE)
    if raw is None:
        return node.allocatable
    try:
        parsed = {k: k8s.Quantity(v) for k, v in json.loads(raw).items()}
    except Exception:  # json error -> Allocatable
        return node.allocatable
    if not parsed:
        return node.allocatable
    out = dict(node.allocatable)
    out.update(parsed)
    return out


def is_node_metric_expired(nm: Optional[k8s.NodeMetric], expiration_s: int, now: float) -> bool:
    """isNodeMetricExpired, helper.go:36-41."""
    return nm is None or nm.update_time is None or (expiration_s > 0 and now - nm.update_time >= expiration_s)


def get_target_aggregated_usage(nm: k8s.NodeMetric, duration_s: Optional[float], agg_type: str):
    """getTargetAggregatedUsage, helper.go:58-90."""
    if not nm.node_metric_present or not nm.aggregated:
        return None
    if not duration_s:
        max_d, max_i = 0.0, 0
        for i, v in enumerate(nm.aggregated):
            if v.duration_s > max_d:
                max_d, max_i = v.duration_s, i
        usage = nm.aggregated[max_i].usage.get(agg_type)
        return usage if usage else None
    for v in nm.aggregated:
        if v.duration_s == duration_s:
            usage = v.usage.get(agg_type)
            if usage:
                return usage
    return None


@dataclass
class _FilterProfile:
    usage_thresholds: Dict[str, int]
    prod_usage_thresholds: Dict[str, int]
    aggregated: Optional[Tuple[Dict[str, int], str, float]]  # (thresholds, type, duration)


def usage_thresholds_filter_profile(node: k8s.Node, args: LoadAwareSchedulingArgs) -> _FilterProfile:
    """generateUsageThresholdsFilterProfile, helper.go:102-140 (+ GetCustomUsageThresholds load_aware.go:51-62)."""
    agg_args = args.aggregated
    filter_with_agg = agg_args is not None and len(agg_args.usage_thresholds) > 0 and agg_args.usage_aggregation_type != ""
    default_agg = ((dict(agg_args.usage_thresholds), agg_args.usage_aggregation_type,
                    agg_args.usage_aggregated_duration_s) if filter_with_agg else None)
    data = node.annotations.get(k8s.ANNOTATION_CUSTOM_USAGE_THRESHOLDS)
    custom = None
    if data is not None:
        try:
            custom = json.loads(data)
            if not isinstance(custom, dict):
                custom = None
        except Exception:
            custom = None
    if data is not None and custom is None:  # unmarshal error
        return _FilterProfile(dict(args.usage_thresholds), dict(args.prod_usage_thresholds), default_agg)
    custom = custom or {}
    ut = custom.get("usageThresholds") or {}
    pt = custom.get("prodUsageThresholds") or {}
    ag = custom.get("aggregatedUsage")
    if not ut:
        ut = dict(args.usage_thresholds)
    if not pt:
        pt = dict(args.prod_usage_thresholds)
    agg = None
    if ag is not None:
        at = ag.get("usageThresholds") or {}
        typ = ag.get("usageAggregationType") or ""
        if at and typ:
            agg = (dict(at), typ, _parse_duration(ag.get("usageAggregatedDuration")))
    if agg is None and filter_with_agg:
        agg = default_agg
    return _FilterProfile({k: int(v) for k, v in ut.items()}, {k: int(v) for k, v in pt.items()}, agg)


def _parse_duration(v) -> float:
    if v is None:
        return 0.0
    if isinstance(v, (int, float)):
        return float(v)
    import re
    total = 0.0
    for num, unit in re.findall(r"([0-9.]+)(ns|us|ms|s|m|h)", v):
        total += float(num) * {"ns": 1e-9, "us": 1e-6, "ms": 1e-3, "s": 1, "m": 60, "h": 3600}[unit]
    return total


def build_pod_metric_map(cluster: ClusterState, nm: k8s.NodeMetric, filter_prod: bool) -> Dict[str, k8s.ResourceList]:
    """buildPodMetricMap, helper.go:153-170."""
    out = {}
    for pm in nm.pods_metric:
        pod = cluster.pods.get(f"{pm.namespace}/{pm.name}")
        if pod is None:
            continue
        if filter_prod and k8s.priority_class(pod) != k8s.PRIORITY_PROD:
            continue
        out[f"{pm.namespace}/{pm.name}"] = pm.usage
    return out


def _sum_rl(dst: Dict[str, k8s.Quantity], src: k8s.ResourceList):
    for n, q in src.items():
        dst[n] = dst.get(n, k8s.Quantity(0)) + q


def estimated_assigned_pod_used(cluster: ClusterState, node_name: str, nm: k8s.NodeMetric, pod_metrics,
                                filter_prod: bool, args: LoadAwareSchedulingArgs, score_agg_nil: bool):
    """estimatedAssignedPodUsed, load_aware.go:337-376."""
    est_used: Dict[str, int] = {}
    est_pods: Set[str] = set()
    update_t = nm.update_time if nm.update_time is not None else float("-inf")
    interval = nm.report_interval_s if nm.report_interval_s is not None else DEFAULT_REPORT_INTERVAL_S
    for info in cluster.assigned.get(node_name, []):
        if filter_prod and k8s.priority_class(info.pod) != k8s.PRIORITY_PROD:
            continue
        name = info.pod.key
        usage = pod_metrics.get(name) or {}
        missed = info.timestamp > update_t                                         # helper.go:50-52
        in_interval = info.timestamp < update_t and (update_t - info.timestamp) < interval  # helper.go:54-56
        if not usage or missed or in_interval or score_agg_nil:
            est = estimate_pod(info.pod, args)
            for r, v in est.items():
                if r in usage:
                    u = k8s.resource_value(r, usage[r])
                    if u > v:
                        v = u
                est_used[r] = est_used.get(r, 0) + v
            est_pods.add(name)
    return est_used, est_pods


def node_row(table: NodeTable, i: int, node: k8s.Node, cluster: ClusterState, profile: Profile, now: float,
             static_classes=None, node_index: Optional[int] = None):
    """Fill row i of `table` from the objects (Fit accounting + LoadAware state,
    and the static_allow bits of `static_classes` when the profile enables the
    upstream static filters).  `node_index`: the node's row in the snapshot
    when `table` holds a subset of its rows (an update_nodes delta)."""
    p = profile.resolved()
    args = p.loadaware
    t = table.cols
    sf = static_filters_of(p)
    if sf:
        from .nodefilters import static_allow
        if static_classes is None:
            raise MarshalError("the profile enables static node filters: pass the snapshot's StaticClasses")
        t["static_allow"][i] = static_allow([node_static(node)], static_classes, sf)[0]
    else:
        t["static_allow"][i] = 0xFFFFFFFF
    if table.has_ext:
        ext_row(table, i, node, cluster, profile, static_classes, node_index)
    # ---- Fit: Allocatable / Requested / NonZeroRequested / len(Pods)
    alloc = node.allocatable
    t["alloc0"][i] = alloc[k8s.CPU].milli_value() if k8s.CPU in alloc else 0
    t["alloc1"][i] = alloc[k8s.MEMORY].value() if k8s.MEMORY in alloc else 0
    t["alloc2"][i] = alloc[k8s.EPHEMERAL].value() if k8s.EPHEMERAL in alloc else 0
    t["alloc3"][i] = alloc[k8s.BATCH_CPU].value() if k8s.BATCH_CPU in alloc else 0
    t["alloc4"][i] = alloc[k8s.BATCH_MEMORY].value() if k8s.BATCH_MEMORY in alloc else 0
    t["alloc_pods"][i] = alloc[k8s.PODS].value() if k8s.PODS in alloc else 0
    req = [0] * abi.NRES
    nzc = nzm = 0
    pods_on_node = cluster.node_pods.get(node.name, [])
    for pod in pods_on_node:
        r, _ = fit_request(pod)
        for k in range(abi.NRES):
            req[k] += r[k]
        a, b = nonzero_request(pod)
        nzc += a
        nzm += b
    for k in range(abi.NRES):
        t[f"requested{k}"][i] = req[k]
    t["nz_cpu_m"][i], t["nz_mem"][i] = nzc, nzm
    t["npods"][i] = len(pods_on_node)
    # ---- LoadAware
    est_alloc = estimate_node(node)
    t["la_alloc_cpu_m"][i] = est_alloc[k8s.CPU].milli_value() if k8s.CPU in est_alloc else 0
    t["la_alloc_mem"][i] = est_alloc[k8s.MEMORY].value() if k8s.MEMORY in est_alloc else 0
    t["laf_total_m0"][i] = t["la_alloc_cpu_m"][i]
    t["laf_total_m1"][i] = est_alloc[k8s.MEMORY].milli_value() if k8s.MEMORY in est_alloc else 0
    nm = cluster.node_metrics.get(node.name)
    flags = 0
    for c in ("la_used_cpu_m", "la_used_mem", "la_used_prod_cpu_m", "la_used_prod_mem", "laf_used_m0",
              "laf_used_m1", "laf_prod_used_m0", "laf_prod_used_m1", "laf_thr0", "laf_thr1",
              "laf_prod_thr0", "laf_prod_thr1"):
        t[c][i] = 0
    if nm is not None:
        flags |= abi.LA_HAS_METRIC
        expired = is_node_metric_expired(nm, args.node_metric_expiration_seconds, now)
        if args.filter_expired_node_metrics and args.node_metric_expiration_seconds is not None and expired:
            flags |= abi.LA_FILTER_SKIP
        if args.node_metric_expiration_seconds is not None and expired:
            flags |= abi.LA_SCORE_EXPIRED
        fp = usage_thresholds_filter_profile(node, args)
        thresholds = fp.aggregated[0] if fp.aggregated else fp.usage_thresholds
        _check_thr_keys(thresholds)
        _check_thr_keys(fp.prod_usage_thresholds)
        t["laf_thr0"][i] = thresholds.get(k8s.CPU, 0)
        t["laf_thr1"][i] = thresholds.get(k8s.MEMORY, 0)
        t["laf_prod_thr0"][i] = fp.prod_usage_thresholds.get(k8s.CPU, 0)
        t["laf_prod_thr1"][i] = fp.prod_usage_thresholds.get(k8s.MEMORY, 0)
        if fp.prod_usage_thresholds:
            flags |= abi.LA_PROD_MODE
        if nm.pods_metric:
            flags |= abi.LA_HAS_PODS_METRIC
        if nm.node_metric_present:
            if fp.aggregated:
                flags |= abi.LA_AGGREGATED
                usage = get_target_aggregated_usage(nm, fp.aggregated[2], fp.aggregated[1])
            else:
                usage = nm.node_usage if nm.node_usage is not None else {}
            if usage is not None:
                flags |= abi.LA_FILTER_USAGE
                t["laf_used_m0"][i] = usage[k8s.CPU].milli_value() if k8s.CPU in usage else 0
                t["laf_used_m1"][i] = usage[k8s.MEMORY].milli_value() if k8s.MEMORY in usage else 0
        # prod pods' usage for filterProdUsage (load_aware.go:232-233)
        prod_metrics = build_pod_metric_map(cluster, nm, True)
        prod_sum: Dict[str, k8s.Quantity] = {}
        for u in prod_metrics.values():
            _sum_rl(prod_sum, u)
        t["laf_prod_used_m0"][i] = prod_sum[k8s.CPU].milli_value() if k8s.CPU in prod_sum else 0
        t["laf_prod_used_m1"][i] = prod_sum[k8s.MEMORY].milli_value() if k8s.MEMORY in prod_sum else 0
        # ---- Score base, non-prod path (load_aware.go:292-327)
        agg = args.aggregated
        score_with_agg = agg is not None and agg.score_aggregation_type != ""
        score_usage = None
        if nm.node_metric_present:
            score_usage = (get_target_aggregated_usage(nm, agg.score_aggregated_duration_s, agg.score_aggregation_type)
                           if score_with_agg else (nm.node_usage if nm.node_usage is not None else {}))
        score_agg_nil = score_with_agg and score_usage is None
        for prod_path in (False, True):
            pm = build_pod_metric_map(cluster, nm, prod_path)
            est_used, est_pods = estimated_assigned_pod_used(cluster, node.name, nm, pm, prod_path, args, score_agg_nil)
            pod_usages: Dict[str, k8s.Quantity] = {}
            est_usages: Dict[str, k8s.Quantity] = {}
            for name, u in pm.items():
                _sum_rl(est_usages if name in est_pods else pod_usages, u)
            base = dict(est_used)
            if prod_path:
                for r, q in pod_usages.items():
                    base[r] = base.get(r, 0) + k8s.resource_value(r, q)
            elif nm.node_metric_present and score_usage is not None:
                for r, q in score_usage.items():
                    e = est_usages.get(r)
                    if e is not None and not e.is_zero() and q.cmp(e) >= 0:
                        q = q - e
                    base[r] = base.get(r, 0) + k8s.resource_value(r, q)
            pre = "la_used_prod_" if prod_path else "la_used_"
            t[pre + "cpu_m"][i] = base.get(k8s.CPU, 0)
            t[pre + "mem"][i] = base.get(k8s.MEMORY, 0)
    t["la_flags"][i] = flags


def ext_row(table: NodeTable, i: int, node: k8s.Node, cluster: ClusterState, profile: Profile, static_classes=None,
            node_index: Optional[int] = None):
    """Row i of the sequential cycle's columns: the node's Device CR and its
    pods' device allocations (dev_*), the extended scalars' Allocatable and
    Requested (xalloc / xrequested), the NodeAffinity / TaintToleration raw
    Scores per static class (static_score)."""
    from . import deviceshare as ds
    t = table.cols
    pods_on_node = cluster.node_pods.get(node.name, [])
    if table.dev_slots:
        ds.device_rows(table, i, cluster.devices.get(node.name),
                       [ds.parse_device_allocated(p.annotations) for p in pods_on_node])
    t["xalloc"][i] = 0
    t["xrequested"][i] = 0
    for n, q in node.allocatable.items():
        if n in ds.XRES_INDEX:
            t["xalloc"][i, ds.XRES_INDEX[n]] = q.value()
    for p in pods_on_node:
        for n, v in ds.fit_xreq(p).items():
            t["xrequested"][i, ds.XRES_INDEX[n]] += v
    if table.has_pts:
        pts_row(table, i, node, cluster, i if node_index is None else node_index)
    if table.has_ipa:
        ipa_row(table, i, node, cluster)
    t["static_score"][i] = 0
    if static_scores_of(profile):
        from .nodefilters import static_scores
        if static_classes is None:
            raise MarshalError("the profile enables NodeAffinity / TaintToleration Scores: pass the StaticClasses")
        t["static_score"][i] = static_scores([node_static(node)], static_classes)[0]


def pts_row(table: NodeTable, i: int, node: k8s.Node, cluster: ClusterState, node_index: int):
    """Row i of the PodTopologySpread columns: the node's domain per key (the
    snapshot's domain index; a value it does not hold needs a rebuild; the
    hostname domain is the node's snapshot row `node_index`), its matching pods
    per table constraint, its spread-class eligibility."""
    from . import topologyspread as ts
    reg = cluster.spread
    labels = node.labels or {}
    dom = table["pts_dom"][i]
    dom[:] = -1
    for k, key in enumerate(reg.keys):
        v = labels.get(key)
        if v is None:
            continue
        if key == ts.HOSTNAME:
            dom[k] = node_index
            continue
        d = reg.domains.values[k].get(v) if reg.domains is not None else None
        if d is None:
            raise NewTopologyValue(f"topology value {key}={v!r} is new to the snapshot: rebuild it")
        dom[k] = d
    cnt, elig = ts.node_pts(reg, node, cluster.node_pods.get(node.name, [])) if reg.cons or reg.classes else (0, 0)
    table["pts_cnt"][i] = cnt
    table["pts_elig"][i] = elig


def ipa_row(table: NodeTable, i: int, node: k8s.Node, cluster: ClusterState):
    """Row i of the InterPodAffinity count column.  A running pod carrying a
    term that a pod to schedule matches but the snapshot has no entry for
    needs a rebuild."""
    from .interpodaffinity import node_ipa
    reg = cluster.ipa
    pods_on_node = cluster.node_pods.get(node.name, [])
    before = len(reg.entries)
    for p in pods_on_node:
        reg.register_existing(p)
    if len(reg.entries) != before or (reg.frozen is not None and len(reg.entries) != reg.frozen):
        raise NewTopologyValue(f"node {node.name}: a running pod carries an affinity term new to the snapshot")
    table["ipa_cnt"][i] = node_ipa(reg, pods_on_node)


def pod_ext_records(pods, profile: Profile, spread=None, ipa=None, reservations=None, node_index=None) -> np.ndarray:
    """koordhip_pod_ext records: DeviceShare requests, extended scalars,
    (PodTopologySpread in the profile) the pods' spread constraints in the
    registry's tables, (InterPodAffinity) their count-entry masks and weights
    and (the Reservation plugin) a pinned reserve pod's node (`node_index`:
    node name -> snapshot row)."""
    from . import deviceshare as ds
    from .config import PLUGIN_PTS
    from .topologyspread import pod_pts_fields
    from .config import PLUGIN_IPA
    pods = list(pods)
    arr = ds.pod_ext_records(pods)
    if _uses(profile, PLUGIN_PTS):
        if spread is None:
            raise MarshalError("the profile enables PodTopologySpread: pass the snapshot's SpreadRegistry")
        for j, p in enumerate(pods):
            if not spread.covers(p):
                raise MarshalError(f"pod {p.key}: spread constraints first seen after the snapshot was built: rebuild it")
            pod_pts_fields(arr[j], p, spread)
    if _uses(profile, PLUGIN_IPA):
        if ipa is None:
            raise MarshalError("the profile enables InterPodAffinity: pass the snapshot's IpaRegistry")
        for j, p in enumerate(pods):
            if not ipa.covers(p):
                raise MarshalError(f"pod {p.key}: affinity terms first seen after the snapshot was built: rebuild it")
            ipa.pod_fields(arr[j], p)
    if _uses(profile, PLUGIN_RESERVATION):
        from . import reservation as rv
        for j, p in enumerate(pods):
            if rv.is_reserve_pod(p):
                if reservations is None or node_index is None:
                    raise MarshalError(f"reserve pod {p.key}: pass the reservations and the node index")
                scratch = pod_array(1)[0]
                rv.reserve_pod_fields(scratch, arr[j], p, reservations, node_index)
    return arr


def device_slots_of(cluster: ClusterState) -> int:
    """The table's dev_slots: the most devices of one type any Device CR lists (>= 1)."""
    m = 1
    for d in cluster.devices.values():
        per: Dict[str, int] = {}
        for x in d.devices:
            per[x.type] = per.get(x.type, 0) + 1
        m = max([m] + list(per.values()))
    if m > abi.DEV_SLOTS:
        raise MarshalError(f"a node lists more than {abi.DEV_SLOTS} devices of one type")
    return m


def _check_thr_keys(th: Dict[str, int]):
    for k in th:
        if k not in (k8s.CPU, k8s.MEMORY):
            raise MarshalError(f"usage threshold on {k!r} is not supported by the engine (cpu, memory only)")


def build_table(cluster: ClusterState, profile: Profile, now: float, static_classes=None) -> NodeTable:
    """The snapshot of `cluster`; with static filters enabled the node bits
    cover the classes `static_classes` holds now, which it then freezes (a pod
    of a later class needs a rebuilt snapshot)."""
    t = NodeTable.empty(len(cluster.nodes))
    t.names = [n.name for n in cluster.nodes]
    if sequential_profile(profile):
        from .config import PLUGIN_DEVICESHARE, PLUGIN_PTS
        t.enable_ext(device_slots_of(cluster) if PLUGIN_DEVICESHARE in profile.filters else 0)
        if PLUGIN_DEVICESHARE in profile.filters and _uses(profile, PLUGIN_RESERVATION):
            t.enable_resv_dev()     # reservations holding devices (reservation.device_reservation_row)
        from .config import PLUGIN_IPA
        reg = cluster.spread
        ipa = cluster.ipa if _uses(profile, PLUGIN_IPA) else None
        if ipa is not None:
            if ipa.topo is not reg:
                raise MarshalError("ClusterState.ipa must share ClusterState.spread's topology keys")
            for pods_on_node in cluster.node_pods.values():
                for p in pods_on_node:
                    ipa.register_existing(p)
        want = (_uses(profile, PLUGIN_PTS) and reg is not None and reg.keys) or (ipa is not None and ipa.entries)
        if want:
            from . import topologyspread as ts
            from .snapshot import IpaMeta, PtsMeta
            reg.domains = ts.DomainIndex(reg)
            reg.domains.build(cluster.nodes)
            ndom = [0 if key == ts.HOSTNAME else max(1, len(reg.domains.values[k])) for k, key in enumerate(reg.keys)]
            pts_on = _uses(profile, PLUGIN_PTS)
            t.enable_pts(PtsMeta(keys=len(reg.keys), hostname=sum(1 << k for k, key in enumerate(reg.keys)
                                                                  if key == ts.HOSTNAME),
                                 ndom=ndom + [0] * (abi.PTS_KEYS - len(ndom)),
                                 cons_key=[k for _, _, k in reg.cons] if pts_on else [],
                                 classes=len(reg.classes) if pts_on else 0))
            reg.freeze()
            if ipa is not None and ipa.entries:
                t.enable_ipa(IpaMeta(ent_key=ipa.ent_keys()))
                ipa.freeze()
    for i, node in enumerate(cluster.nodes):
        node_row(t, i, node, cluster, profile, now, static_classes)
    if static_classes is not None:
        static_classes.frozen = len(static_classes.specs)
    return t
