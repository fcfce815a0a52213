"""Minimal Kubernetes object model for the host side of the placement engine.

Only what the Filter/Score hot path reads: resource.Quantity arithmetic, Pod /
Node / NodeMetric fields, and the koordinator priority / QoS helpers.  The Go
host gets these from client-go; here they are plain dataclasses so the parity
tests can be written like the reference's own table tests.

Reference semantics restated:
  * resource.Quantity Value()/MilliValue() round up (k8s.io/apimachinery
    pkg/api/resource/quantity.go, upstream v0.24.15).
  * priority class:  apis/extension/priority.go:71-100, priority_utils.go:26-47
  * QoS class:       apis/extension/qos_utils.go:32-78 and (upstream)
    pkg/apis/core/v1/helper/qos GetPodQOS.
  * PodRequestsAndLimits: (upstream) pkg/api/v1/resource/helpers.go.
"""
from __future__ import annotations

import math
import re
from dataclasses import dataclass, field
from fractions import Fraction
from typing import Dict, List, Optional, Tuple

# ---------------------------------------------------------------------------
# resource names (corev1 + apis/extension/resource.go:25-30)
CPU = "cpu"
MEMORY = "memory"
EPHEMERAL = "ephemeral-storage"
PODS = "pods"
BATCH_CPU = "kubernetes.io/batch-cpu"
BATCH_MEMORY = "kubernetes.io/batch-memory"
MID_CPU = "kubernetes.io/mid-cpu"
MID_MEMORY = "kubernetes.io/mid-memory"

LABEL_POD_QOS = "koordinator.sh/qosClass"            # apis/extension/constants.go:31
LABEL_POD_PRIORITY_CLASS = "koordinator.sh/priority-class"
ANNOTATION_CUSTOM_USAGE_THRESHOLDS = "scheduling.koordinator.sh/usage-thresholds"  # load_aware.go:28
ANNOTATION_NODE_RAW_ALLOCATABLE = "node.koordinator.sh/raw-allocatable"           # node_resource_amplification.go:37

# ---------------------------------------------------------------------------
# resource.Quantity

_SUFFIX = {
    "": Fraction(1),
    "n": Fraction(1, 10**9), "u": Fraction(1, 10**6), "m": Fraction(1, 1000),
    "k": Fraction(10**3), "M": Fraction(10**6), "G": Fraction(10**9), "T": Fraction(10**12),
    "P": Fraction(10**15), "E": Fraction(10**18),
    "Ki": Fraction(2**10), "Mi": Fraction(2**20), "Gi": Fraction(2**30), "Ti": Fraction(2**40),
    "Pi": Fraction(2**50), "Ei": Fraction(2**60),
}
_QRE = re.compile(r"^([+-]?[0-9]*\.?[0-9]*)(?:([eE][+-]?[0-9]+)|(Ki|Mi|Gi|Ti|Pi|Ei|n|u|m|k|M|G|T|P|E)?)$")


class Quantity:
    """Exact decimal/binary quantity (resource.MustParse semantics)."""

    __slots__ = ("v",)

    def __init__(self, v):
        if isinstance(v, Quantity):
            self.v = v.v
        elif isinstance(v, str):
            self.v = _parse(v)
        else:
            self.v = Fraction(v)

    def value(self) -> int:
        """Quantity.Value(): rounds up to the next integer."""
        return math.ceil(self.v)

    def milli_value(self) -> int:
        """Quantity.MilliValue(): rounds up to the next milli unit."""
        return math.ceil(self.v * 1000)

    def is_zero(self) -> bool:
        return self.v == 0

    def cmp(self, other: "Quantity") -> int:
        o = other.v if isinstance(other, Quantity) else Fraction(other)
        return (self.v > o) - (self.v < o)

    def __add__(self, other):
        return Quantity(self.v + Quantity(other).v)

    def __sub__(self, other):
        return Quantity(self.v - Quantity(other).v)

    def __eq__(self, other):
        return isinstance(other, Quantity) and self.v == other.v

    def __hash__(self):
        return hash(self.v)

    def __repr__(self):
        return f"Quantity({self.v})"


def _parse(s: str) -> Fraction:
    m = _QRE.match(s.strip())
    if not m or m.group(1) in ("", "+", "-", "."):
        raise ValueError(f"quantities must match the regular expression: {s!r}")
    num = Fraction(m.group(1))
    if m.group(2):
        num *= Fraction(10) ** int(m.group(2)[1:])
    else:
        num *= _SUFFIX[m.group(3) or ""]
    return num


def Q(s) -> Quantity:
    return Quantity(s)


ResourceList = Dict[str, Quantity]


def rl(**kw) -> ResourceList:
    """rl(cpu="16", memory="32Gi", batch_cpu="4000") -> ResourceList."""
    names = {"cpu": CPU, "memory": MEMORY, "ephemeral_storage": EPHEMERAL, "pods": PODS,
             "batch_cpu": BATCH_CPU, "batch_memory": BATCH_MEMORY}
    return {names.get(k, k): Quantity(v) for k, v in kw.items()}


def resource_value(name: str, q: Quantity) -> int:
    """getResourceValue, loadaware/helper.go:146-151: cpu -> MilliValue, else Value."""
    return q.milli_value() if name == CPU else q.value()


# ---------------------------------------------------------------------------
# objects

@dataclass
class Container:
    name: str = "c"
    requests: ResourceList = field(default_factory=dict)
    limits: ResourceList = field(default_factory=dict)


@dataclass
class OwnerReference:
    """metav1.OwnerReference of a pod (reservation owner matching)."""
    kind: str = ""
    name: str = ""
    uid: str = ""
    api_version: str = ""
    controller: Optional[bool] = None


@dataclass
class Pod:
    namespace: str = "default"
    name: str = "pod"
    uid: str = ""
    labels: Dict[str, str] = field(default_factory=dict)
    annotations: Dict[str, str] = field(default_factory=dict)
    priority: Optional[int] = None
    containers: List[Container] = field(default_factory=list)
    init_containers: List[Container] = field(default_factory=list)
    overhead: Optional[ResourceList] = None
    owner_kinds: List[str] = field(default_factory=list)
    node_name: str = ""
    qos_status: str = ""          # Status.QOSClass
    phase: str = "Running"
    ready: bool = True            # the Ready condition (k8spodutil.IsPodReady)
    deleting: bool = False        # metadata.deletionTimestamp set
    owner_refs: List[OwnerReference] = field(default_factory=list)
    api_version: str = "v1"
    # what the upstream static filters read (nodefilters.py): spec.nodeSelector,
    # spec.affinity.nodeAffinity.requiredDuringScheduling... terms
    # (reservation.NodeSelectorTerm; None = unset), spec.tolerations
    # (nodefilters.Toleration)
    node_selector: Dict[str, str] = field(default_factory=dict)
    required_node_affinity: Optional[list] = None
    tolerations: list = field(default_factory=list)
    # spec.affinity.nodeAffinity.preferredDuringScheduling...: [(weight, NodeSelectorTerm)]
    preferred_node_affinity: list = field(default_factory=list)
    # spec.topologySpreadConstraints (topologyspread.TopologySpreadConstraint)
    topology_spread_constraints: list = field(default_factory=list)
    # spec.affinity.podAffinity / podAntiAffinity (interpodaffinity.PodAffinityTerm,
    # WeightedPodAffinityTerm): required... and preferredDuringSchedulingIgnoredDuringExecution
    pod_affinity_required: list = field(default_factory=list)
    pod_affinity_preferred: list = field(default_factory=list)
    pod_anti_affinity_required: list = field(default_factory=list)
    pod_anti_affinity_preferred: list = field(default_factory=list)

    @property
    def key(self) -> str:
        return f"{self.namespace}/{self.name}"


@dataclass
class Node:
    name: str
    allocatable: ResourceList = field(default_factory=dict)
    annotations: Dict[str, str] = field(default_factory=dict)
    labels: Dict[str, str] = field(default_factory=dict)
    taints: list = field(default_factory=list)      # spec.taints (nodefilters.Taint)
    unschedulable: bool = False                     # spec.unschedulable


@dataclass
class PodMetric:
    namespace: str
    name: str
    usage: ResourceList


@dataclass
class AggregatedUsage:
    duration_s: float
    usage: Dict[str, ResourceList]   # aggregation type ("p50","p90","p95","p99","avg") -> usage


@dataclass
class NodeMetric:
    """slo/v1alpha1 NodeMetric (apis/slo/v1alpha1/nodemetric_types.go:38-128)."""
    name: str
    update_time: Optional[float] = None          # Status.UpdateTime, seconds
    report_interval_s: Optional[float] = None    # Spec.CollectPolicy.ReportIntervalSeconds
    node_usage: Optional[ResourceList] = None    # Status.NodeMetric.NodeUsage; None => Status.NodeMetric == nil
    aggregated: List[AggregatedUsage] = field(default_factory=list)
    pods_metric: List[PodMetric] = field(default_factory=list)
    has_node_metric: Optional[bool] = None       # override: NodeMetric set even if node_usage is None

    @property
    def node_metric_present(self) -> bool:
        if self.has_node_metric is not None:
            return self.has_node_metric
        return self.node_usage is not None or bool(self.aggregated)


# ---------------------------------------------------------------------------
# priority / QoS (apis/extension)

PRIORITY_PROD, PRIORITY_MID, PRIORITY_BATCH, PRIORITY_FREE, PRIORITY_NONE = (
    "koord-prod", "koord-mid", "koord-batch", "koord-free", "")
QOS_LSE, QOS_LSR, QOS_LS, QOS_BE, QOS_SYSTEM, QOS_NONE = "LSE", "LSR", "LS", "BE", "SYSTEM", ""

PRIORITY_PROD_MAX, PRIORITY_PROD_MIN = 9999, 9000
PRIORITY_MID_MAX, PRIORITY_MID_MIN = 7999, 7000
PRIORITY_BATCH_MAX, PRIORITY_BATCH_MIN = 5999, 5000
PRIORITY_FREE_MAX, PRIORITY_FREE_MIN = 3999, 3000


def priority_class_raw(pod: Pod) -> str:
    """GetPodPriorityClassRaw, apis/extension/priority.go:71-100."""
    if LABEL_POD_PRIORITY_CLASS in pod.labels:
        p = pod.labels[LABEL_POD_PRIORITY_CLASS]
        return p if p in (PRIORITY_PROD, PRIORITY_MID, PRIORITY_BATCH, PRIORITY_FREE) else PRIORITY_NONE
    if pod.priority is None:
        return PRIORITY_NONE
    p = pod.priority
    if PRIORITY_PROD_MIN <= p <= PRIORITY_PROD_MAX:
        return PRIORITY_PROD
    if PRIORITY_MID_MIN <= p <= PRIORITY_MID_MAX:
        return PRIORITY_MID
    if PRIORITY_BATCH_MIN <= p <= PRIORITY_BATCH_MAX:
        return PRIORITY_BATCH
    if PRIORITY_FREE_MIN <= p <= PRIORITY_FREE_MAX:
        return PRIORITY_FREE
    return PRIORITY_NONE


def kube_qos(pod: Pod) -> str:
    """(upstream) v1qos.GetPodQOS (k8s v1.24), via GetKubeQosClass qos_utils.go:72-78."""
    if pod.qos_status:
        return pod.qos_status
    requests: Dict[str, Fraction] = {}
    limits: Dict[str, Fraction] = {}
    guaranteed = True
    for c in list(pod.containers) + list(pod.init_containers):
        for n, q in c.requests.items():
            if n in (CPU, MEMORY) and q.v > 0:
                requests[n] = requests.get(n, Fraction(0)) + q.v
        found = set()
        for n, q in c.limits.items():
            if n in (CPU, MEMORY) and q.v > 0:
                found.add(n)
                limits[n] = limits.get(n, Fraction(0)) + q.v
        if not {CPU, MEMORY} <= found:
            guaranteed = False
    if not requests and not limits:
        return "BestEffort"
    if guaranteed:
        for n, r in requests.items():
            if n not in limits or limits[n] != r:
                guaranteed = False
                break
    if guaranteed and len(requests) == len(limits):
        return "Guaranteed"
    return "Burstable"


def qos_class_raw(pod: Pod) -> str:
    """GetPodQoSClassRaw, qos_utils.go:57-70: the koordinator.sh/qosClass label only."""
    q = pod.labels.get(LABEL_POD_QOS) if pod.labels else None
    return q if q in (QOS_LSE, QOS_LSR, QOS_LS, QOS_BE, QOS_SYSTEM) else QOS_NONE


def qos_class(pod: Pod) -> str:
    """GetPodQoSClassWithDefault, qos_utils.go:32-62 (Guaranteed -> LSR)."""
    q = pod.labels.get(LABEL_POD_QOS) if pod.labels else None
    if q is not None:
        return q if q in (QOS_LSE, QOS_LSR, QOS_LS, QOS_BE, QOS_SYSTEM) else QOS_NONE
    k = kube_qos(pod)
    return {"Guaranteed": QOS_LSR, "Burstable": QOS_LS, "BestEffort": QOS_BE}.get(k, QOS_NONE)


def priority_class(pod: Pod) -> str:
    """GetPodPriorityClassWithDefault, priority_utils.go:26-47."""
    p = priority_class_raw(pod)
    if p != PRIORITY_NONE:
        return p
    q = qos_class(pod)
    if q in (QOS_SYSTEM, QOS_LSE, QOS_LSR, QOS_LS):
        return PRIORITY_PROD
    if q == QOS_BE:
        return PRIORITY_BATCH
    return PRIORITY_NONE


def translate_resource(priority: str, name: str) -> str:
    """TranslateResourceNameByPriorityClass, apis/extension/resource.go:50-58.
    Free-priority pods map to "" (no entry in ResourceNameMap)."""
    if priority in (PRIORITY_PROD, PRIORITY_NONE):
        return name
    table = {PRIORITY_BATCH: {CPU: BATCH_CPU, MEMORY: BATCH_MEMORY},
             PRIORITY_MID: {CPU: MID_CPU, MEMORY: MID_MEMORY}}
    return table.get(priority, {}).get(name, "")


def is_daemonset_pod(pod: Pod) -> bool:
    """isDaemonSetPod, loadaware/helper.go:188-196."""
    return any(k == "DaemonSet" for k in pod.owner_kinds)


def is_terminated(pod: Pod) -> bool:
    return pod.phase in ("Succeeded", "Failed")


# ---------------------------------------------------------------------------
# PodRequestsAndLimits (upstream pkg/api/v1/resource/helpers.go)

def _add(dst: Dict[str, Fraction], src: ResourceList):
    for n, q in src.items():
        dst[n] = dst.get(n, Fraction(0)) + q.v


def _max(dst: Dict[str, Fraction], src: ResourceList):
    for n, q in src.items():
        if n not in dst or q.v > dst[n]:
            dst[n] = q.v


def pod_requests_and_limits(pod: Pod) -> Tuple[ResourceList, ResourceList]:
    reqs: Dict[str, Fraction] = {}
    lims: Dict[str, Fraction] = {}
    for c in pod.containers:
        _add(reqs, c.requests)
        _add(lims, c.limits)
    for c in pod.init_containers:
        _max(reqs, c.requests)
        _max(lims, c.limits)
    if pod.overhead:
        _add(reqs, pod.overhead)
        for n, q in pod.overhead.items():
            if n in lims:
                lims[n] += q.v
    return ({k: Quantity(v) for k, v in reqs.items()}, {k: Quantity(v) for k, v in lims.items()})


def round_half_away(x: float) -> int:
    """Go math.Round for x >= 0 (half away from zero), exact: floor + compare."""
    f = math.floor(x)
    return int(f) + (1 if (x - f) >= 0.5 else 0) if x >= 0 else -round_half_away(-x)
