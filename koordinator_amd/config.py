"""Plugin arguments for the three hot-path plugins, with the reference's
defaults and validation, and their lowering to the C-ABI koordhip_config.

  LoadAwareSchedulingArgs  pkg/scheduler/apis/config/types.go:29-74
                           defaults v1beta2/defaults.go:32-96
                           validation validation/validation_pluginargs.go:31-95
  NodeNUMAResourceArgs     types.go:102-108, defaults v1beta2/defaults.go:98-121
  NodeResourcesFitArgs     (upstream) + config/manager/scheduler-config.yaml:17-31
  plugin score weights     config/manager/scheduler-config.yaml:82-91
"""
from __future__ import annotations

import copy
from dataclasses import dataclass, field
from typing import Dict, Optional

from . import k8s

FIT_RESOURCES = [k8s.CPU, k8s.MEMORY, k8s.EPHEMERAL, k8s.BATCH_CPU, k8s.BATCH_MEMORY]

PLUGIN_FIT = "NodeResourcesFit"
PLUGIN_LOADAWARE = "LoadAwareScheduling"
PLUGIN_NUMA = "NodeNUMAResource"
PLUGIN_RESERVATION = "Reservation"
# upstream default-profile plugins (k8s v1.24.15): three static node filters
# (resolved by the host into static_allow) and one score
PLUGIN_NODE_UNSCHEDULABLE = "NodeUnschedulable"
PLUGIN_NODE_AFFINITY = "NodeAffinity"
PLUGIN_TAINT_TOLERATION = "TaintToleration"
PLUGIN_BALANCED = "NodeResourcesBalancedAllocation"
PLUGIN_NODE_NAME = "NodeName"
STATIC_FILTERS = (PLUGIN_NODE_UNSCHEDULABLE, PLUGIN_NODE_NAME, PLUGIN_NODE_AFFINITY, PLUGIN_TAINT_TOLERATION)
PLUGIN_DEVICESHARE = "DeviceShare"
PLUGIN_PTS = "PodTopologySpread"
PLUGIN_IPA = "InterPodAffinity"
# Scores normalized over the pod's feasible nodes (DefaultNormalizeScore, or the
# plugin's own min-max normalization): the sequential cycle; NodeAffinity /
# TaintToleration in `scores` are their Scores
NORMALIZED_SCORES = (PLUGIN_DEVICESHARE, PLUGIN_NODE_AFFINITY, PLUGIN_TAINT_TOLERATION, PLUGIN_PTS, PLUGIN_IPA)


class ArgsError(ValueError):
    """field.ErrorList.ToAggregate() analogue."""


@dataclass
class LoadAwareSchedulingAggregatedArgs:
    usage_thresholds: Dict[str, int] = field(default_factory=dict)
    usage_aggregation_type: str = ""
    usage_aggregated_duration_s: float = 0.0
    score_aggregation_type: str = ""
    score_aggregated_duration_s: float = 0.0


@dataclass
class LoadAwareSchedulingArgs:
    filter_expired_node_metrics: Optional[bool] = None
    node_metric_expiration_seconds: Optional[int] = None
    resource_weights: Dict[str, int] = field(default_factory=dict)
    usage_thresholds: Dict[str, int] = field(default_factory=dict)
    prod_usage_thresholds: Dict[str, int] = field(default_factory=dict)
    score_according_prod_usage: bool = False
    estimated_scaling_factors: Optional[Dict[str, int]] = None
    aggregated: Optional[LoadAwareSchedulingAggregatedArgs] = None

    def with_defaults(self) -> "LoadAwareSchedulingArgs":
        """SetDefaults_LoadAwareSchedulingArgs, v1beta2/defaults.go:75-96."""
        a = copy.deepcopy(self)
        if a.filter_expired_node_metrics is None:
            a.filter_expired_node_metrics = True
        if a.node_metric_expiration_seconds is None:
            a.node_metric_expiration_seconds = 180
        if not a.resource_weights:
            a.resource_weights = {k8s.CPU: 1, k8s.MEMORY: 1}
        if not a.usage_thresholds:
            a.usage_thresholds = {k8s.CPU: 65, k8s.MEMORY: 95}
        if a.estimated_scaling_factors is None:
            a.estimated_scaling_factors = {k8s.CPU: 85, k8s.MEMORY: 70}
        else:
            for k, v in {k8s.CPU: 85, k8s.MEMORY: 70}.items():
                a.estimated_scaling_factors.setdefault(k, v)
        return a

    def validate(self):
        """ValidateLoadAwareSchedulingArgs, validation_pluginargs.go:31-95."""
        errs = []
        if self.node_metric_expiration_seconds is not None and self.node_metric_expiration_seconds <= 0:
            errs.append("nodeMetricExpiredSeconds should be a positive value")
        for r, w in self.resource_weights.items():
            if w <= 0 or w > 100:
                errs.append(f"resourceWeights: resource Weight of {r} out of range, got {w}")
                break
        for r, t in self.usage_thresholds.items():
            if t < 0 or t > 100:
                errs.append(f"usageThresholds: resource Threshold of {r} out of range, got {t}")
                break
        for r, f in (self.estimated_scaling_factors or {}).items():
            if f <= 0 or f > 100:
                errs.append(f"estimatedScalingFactors: estimated resource Threshold of {r} out of range, got {f}")
                break
        for r in self.resource_weights:
            if r not in (self.estimated_scaling_factors or {}):
                errs.append(f"estimatedScalingFactors: Not found: {r!r}")
                break
        # Engine restriction (documented in DESIGN.md): weighted resources are cpu/memory.
        for r in self.resource_weights:
            if r not in (k8s.CPU, k8s.MEMORY):
                errs.append(f"resourceWeights: {r!r} is not supported by the engine (cpu, memory only)")
        if errs:
            raise ArgsError("; ".join(errs))


@dataclass
class NodeResourcesFitArgs:
    """LeastAllocated scoring strategy only (the shipped profile)."""
    scoring_type: str = "LeastAllocated"
    resources: Dict[str, int] = field(default_factory=lambda: {k8s.CPU: 1, k8s.MEMORY: 1})

    def validate(self):
        if self.scoring_type != "LeastAllocated":
            raise ArgsError(f"scoringStrategy.type {self.scoring_type!r} not supported (LeastAllocated)")
        for r, w in self.resources.items():
            if r not in FIT_RESOURCES:
                raise ArgsError(f"scoringStrategy.resources: {r!r} not supported by the engine")
            if w < 1 or w > 100:
                raise ArgsError(f"scoringStrategy.resources: weight of {r} out of range, got {w}")


@dataclass
class NodeNUMAResourceArgs:
    default_cpu_bind_policy: str = "FullPCPUs"
    scoring_type: str = "LeastAllocated"
    resources: Dict[str, int] = field(default_factory=lambda: {k8s.CPU: 1, k8s.MEMORY: 1})

    @property
    def default_most_allocated(self) -> bool:
        """GetDefaultNUMAAllocateStrategy (nodenumaresource/util.go:25-32)."""
        return self.scoring_type != "LeastAllocated"

    def validate(self):
        """ValidateNodeNUMAResourceArgs + the engine's scope (Least/MostAllocated over cpu/memory)."""
        if self.default_cpu_bind_policy not in ("", "Default", "FullPCPUs", "SpreadByPCPUs", "ConstrainedBurst"):
            raise ArgsError(f"defaultCPUBindPolicy: unsupported value {self.default_cpu_bind_policy!r}")
        if self.scoring_type not in ("LeastAllocated", "MostAllocated"):
            raise ArgsError(f"NodeNUMAResource scoringStrategy.type {self.scoring_type!r}: LeastAllocated or "
                            "MostAllocated (scoring.go:35-53)")
        for r, w in self.resources.items():
            if r not in (k8s.CPU, k8s.MEMORY):
                raise ArgsError(f"NodeNUMAResource scoringStrategy.resources: {r} is not supported by this engine")
            if not (0 <= w <= 100):
                raise ArgsError(f"NodeNUMAResource scoringStrategy.resources: weight of {r} out of range, got {w}")


@dataclass
class DeviceShareArgs:
    """DeviceShareArgs (pkg/scheduler/apis/config/types.go), defaults
    v1beta2/defaults.go:168-189: LeastAllocated over gpu-memory-ratio, rdma, fpga."""
    scoring_type: str = "LeastAllocated"
    resources: Dict[str, int] = field(default_factory=lambda: {
        "koordinator.sh/gpu-memory-ratio": 1, "koordinator.sh/rdma": 1, "koordinator.sh/fpga": 1})

    SCORER_RESOURCES = ("koordinator.sh/gpu-core", "koordinator.sh/gpu-memory-ratio", "koordinator.sh/gpu-memory",
                        "koordinator.sh/rdma", "koordinator.sh/fpga")

    def validate(self):
        if self.scoring_type not in ("LeastAllocated", "MostAllocated"):
            raise ArgsError(f"DeviceShare scoringStrategy.type {self.scoring_type!r}: LeastAllocated or MostAllocated")
        for r, w in self.resources.items():
            if r not in self.SCORER_RESOURCES:
                raise ArgsError(f"DeviceShare scoringStrategy.resources: {r!r} is not a device resource")
            if not 0 <= w <= 100:
                raise ArgsError(f"DeviceShare scoringStrategy.resources: weight of {r} out of range, got {w}")


@dataclass
class InterPodAffinityArgs:
    """InterPodAffinityArgs (upstream k8s v1.24 config/types.go), defaults
    v1beta2 SetDefaults_InterPodAffinityArgs: HardPodAffinityWeight 1."""
    hard_pod_affinity_weight: int = 1

    def validate(self):
        """ValidateInterPodAffinityArgs: 0..100."""
        if not 0 <= self.hard_pod_affinity_weight <= 100:
            raise ArgsError(f"hardPodAffinityWeight: Invalid value: {self.hard_pod_affinity_weight}: not in valid "
                            "range [0-100]")


@dataclass
class Profile:
    """The scheduling profile restricted to the hot-path plugins."""
    filters: tuple = (PLUGIN_FIT, PLUGIN_LOADAWARE)
    scores: Dict[str, int] = field(default_factory=lambda: {PLUGIN_FIT: 1, PLUGIN_LOADAWARE: 1})
    fit: NodeResourcesFitArgs = field(default_factory=NodeResourcesFitArgs)
    loadaware: LoadAwareSchedulingArgs = field(default_factory=LoadAwareSchedulingArgs)
    numa: NodeNUMAResourceArgs = field(default_factory=NodeNUMAResourceArgs)
    deviceshare: DeviceShareArgs = field(default_factory=DeviceShareArgs)
    interpodaffinity: InterPodAffinityArgs = field(default_factory=InterPodAffinityArgs)
    batch_pods: int = 0

    def resolved(self) -> "Profile":
        p = copy.deepcopy(self)
        p.loadaware = p.loadaware.with_defaults()
        return p


def shipped_profile(numa: bool = False, reservation: bool = False) -> Profile:
    """config/manager/scheduler-config.yaml:17-46,82-91 restricted to Fit + LoadAware
    (+ NodeNUMAResource with default args and score weight 1 when `numa`; + the
    Reservation plugin, Filter and Score weight 5000 (:60-91), when `reservation`)."""
    la = LoadAwareSchedulingArgs(
        filter_expired_node_metrics=False,
        node_metric_expiration_seconds=300,
        resource_weights={k8s.CPU: 1, k8s.MEMORY: 1},
        usage_thresholds={k8s.CPU: 65, k8s.MEMORY: 95},
        estimated_scaling_factors={k8s.CPU: 85, k8s.MEMORY: 70},
    )
    fit = NodeResourcesFitArgs(resources={k8s.CPU: 1, k8s.MEMORY: 1, k8s.BATCH_CPU: 1, k8s.BATCH_MEMORY: 1})
    if reservation:
        filters = (PLUGIN_FIT, PLUGIN_LOADAWARE) + ((PLUGIN_NUMA,) if numa else ()) + (PLUGIN_RESERVATION,)
        scores = {PLUGIN_FIT: 1, PLUGIN_LOADAWARE: 1, PLUGIN_RESERVATION: 5000}
        if numa:
            scores[PLUGIN_NUMA] = 1
        return Profile(filters=filters, scores=scores, fit=fit, loadaware=la)
    if numa:
        return Profile(filters=(PLUGIN_FIT, PLUGIN_LOADAWARE, PLUGIN_NUMA),
                       scores={PLUGIN_FIT: 1, PLUGIN_LOADAWARE: 1, PLUGIN_NUMA: 1}, fit=fit, loadaware=la)
    return Profile(fit=fit, loadaware=la)


def with_upstream(profile: Profile, static_filters=STATIC_FILTERS, balanced_weight: int = 0) -> Profile:
    """The profile plus upstream default-profile plugins: the static node
    filters (Filter) and NodeResourcesBalancedAllocation (Score, weight
    `balanced_weight`; 0 = not enabled)."""
    p = copy.deepcopy(profile)
    p.filters = tuple(p.filters) + tuple(f for f in static_filters if f not in p.filters)
    if balanced_weight:
        p.scores = dict(p.scores)
        p.scores[PLUGIN_BALANCED] = balanced_weight
    return p


def with_deviceshare(profile: Profile, weight: int = 1) -> Profile:
    """The profile plus DeviceShare at Filter and Score (scheduler-config.yaml:62-105: weight 1)."""
    p = copy.deepcopy(profile)
    if PLUGIN_DEVICESHARE not in p.filters:
        p.filters = tuple(p.filters) + (PLUGIN_DEVICESHARE,)
    p.scores = dict(p.scores)
    p.scores[PLUGIN_DEVICESHARE] = weight
    return p


def with_normalized_scores(profile: Profile, affinity: int = 0, taint: int = 0) -> Profile:
    """The upstream NodeAffinity (preferred terms) / TaintToleration
    (PreferNoSchedule) Scores at the given weights (0 = off)."""
    p = copy.deepcopy(profile)
    p.scores = dict(p.scores)
    if affinity:
        p.scores[PLUGIN_NODE_AFFINITY] = affinity
    if taint:
        p.scores[PLUGIN_TAINT_TOLERATION] = taint
    return p


def with_topology_spread(profile: Profile, weight: int = 2, filter: bool = True) -> Profile:
    """The upstream PodTopologySpread plugin: Filter (DoNotSchedule constraints)
    and Score (ScheduleAnyway; the upstream default profile weighs it 2)."""
    p = copy.deepcopy(profile)
    if filter and PLUGIN_PTS not in p.filters:
        p.filters = tuple(p.filters) + (PLUGIN_PTS,)
    if weight:
        p.scores = dict(p.scores)
        p.scores[PLUGIN_PTS] = weight
    return p


def with_interpod_affinity(profile: Profile, weight: int = 1, filter: bool = True,
                           hard_pod_affinity_weight: int = 1) -> Profile:
    """The upstream InterPodAffinity plugin: Filter (required affinity /
    anti-affinity) and Score (the upstream default profile weighs it 1)."""
    p = copy.deepcopy(profile)
    if filter and PLUGIN_IPA not in p.filters:
        p.filters = tuple(p.filters) + (PLUGIN_IPA,)
    if weight:
        p.scores = dict(p.scores)
        p.scores[PLUGIN_IPA] = weight
    p.interpodaffinity = InterPodAffinityArgs(hard_pod_affinity_weight)
    return p


def to_c_config(profile: Profile, device: int = -1):
    """Lower a resolved profile to the koordhip_config ctypes struct."""
    from .abi import (KOORDHIP_ABI_VERSION, PLUGIN_BITS, KoordhipConfig)

    p = profile.resolved()
    p.loadaware.validate()
    p.fit.validate()
    if PLUGIN_NUMA in p.filters or PLUGIN_NUMA in p.scores:
        p.numa.validate()
    cfg = KoordhipConfig()
    cfg.abi_version = KOORDHIP_ABI_VERSION
    from . import abi
    score_bits = {PLUGIN_NODE_AFFINITY: abi.PLUGIN_AFFINITY_SCORE, PLUGIN_TAINT_TOLERATION: abi.PLUGIN_TAINT_SCORE,
                  PLUGIN_DEVICESHARE: abi.PLUGIN_DEVICESHARE, PLUGIN_PTS: abi.PLUGIN_PTS, PLUGIN_IPA: abi.PLUGIN_IPA}
    own_filter_bits = {PLUGIN_DEVICESHARE: abi.PLUGIN_DEVICESHARE, PLUGIN_PTS: abi.PLUGIN_PTS,
                       PLUGIN_IPA: abi.PLUGIN_IPA}
    cfg.filter_plugins = 0
    for x in p.filters:  # (the three static filters share one bit)
        cfg.filter_plugins |= own_filter_bits[x] if x in own_filter_bits else PLUGIN_BITS[x]
    cfg.score_plugins = 0
    for x in p.scores:
        cfg.score_plugins |= score_bits[x] if x in score_bits else PLUGIN_BITS[x]
    cfg.device = device
    for name in p.scores:
        if name in STATIC_FILTERS and name not in NORMALIZED_SCORES:
            raise ArgsError(f"the Score of {name} is not supported (Filter only)")
    for e, name in enumerate(NORMALIZED_SCORES):
        if name in p.scores:
            w = p.scores[name]
            if not 1 <= w <= 100:
                raise ArgsError(f"score weight of {name} out of range, got {w}")
            cfg.ext_weight[e] = w
    if PLUGIN_DEVICESHARE in p.filters or PLUGIN_DEVICESHARE in p.scores:
        p.deviceshare.validate()
    p.interpodaffinity.validate()
    cfg.dev_most_allocated = 1 if p.deviceshare.scoring_type == "MostAllocated" else 0
    for k, r in enumerate(DeviceShareArgs.SCORER_RESOURCES):
        cfg.dev_res_weight[k] = p.deviceshare.resources.get(r, 0)
    order = [PLUGIN_FIT, PLUGIN_LOADAWARE, PLUGIN_NUMA, PLUGIN_BALANCED]
    for i, name in enumerate(order):
        w = p.scores.get(name, 0)
        if name in p.scores and not (1 <= w <= 100):
            raise ArgsError(f"score weight of {name} out of range, got {w}")
        cfg.plugin_weight[i] = w
    if PLUGIN_RESERVATION in p.scores:
        w = p.scores[PLUGIN_RESERVATION]
        bmax = 100 * sum(p.scores.get(x, 0) for x in order + list(NORMALIZED_SCORES))
        if not (1 <= w <= 1000000):
            raise ArgsError(f"score weight of {PLUGIN_RESERVATION} out of range, got {w}")
        if w <= bmax:
            # the engine ranks by (normalized reservation score, other plugins' total): exact only
            # when one unit of the former outweighs the latter (Reservation key)
            raise ArgsError(f"Reservation weight {w} must exceed 100 x the other score weights ({bmax})")
        cfg.reservation_weight = w
    for i, r in enumerate(FIT_RESOURCES):
        cfg.fit_weight[i] = p.fit.resources.get(r, 0)
    cfg.la_weight_cpu = p.loadaware.resource_weights.get(k8s.CPU, 0)
    cfg.la_weight_mem = p.loadaware.resource_weights.get(k8s.MEMORY, 0)
    cfg.la_score_according_prod_usage = 1 if p.loadaware.score_according_prod_usage else 0
    cfg.batch_pods = p.batch_pods
    cfg.numa_weight_cpu = p.numa.resources.get(k8s.CPU, 0)
    cfg.numa_weight_mem = p.numa.resources.get(k8s.MEMORY, 0)
    cfg.numa_most_allocated = 1 if p.numa.scoring_type == "MostAllocated" else 0
    return cfg
