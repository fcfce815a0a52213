"""Host side of the Reservation plugin: the Reservation object model, owner
matching and the per-node reservation columns of koordhip_node_soa.

Restated from the reference:
  * ReservationInfo           pkg/scheduler/frameworkext/reservation_info.go:36-126
    (Allocatable = ReservationRequests, ResourceNames = its keys, Allocated
    masked to them, AssignedPods)
  * IsAvailable / ReservationRequests   pkg/util/reservation/reservation.go:213-215, 334-345
  * owner matchers            reservation.go:357-442 (ObjectReference, controller
    reference, label selector; DNF over the owners list)
  * IsAllocateOnce            apis/extension/reservation.go:98-100 (default true)
  * IsUnschedulable           reservation_info.go:248-255
  * reservation order label   reservation/scoring.go:156-175 (strconv.ParseInt, 0 = none)
  * reserve pod non-zero request: calculateResource, reservation/transformer.go:302-333

The device evaluates owner matching as bit tests: every distinct owner spec
(x the results of the registered reservation affinities) of the snapshot's
reservations is a group g (<= 64), a reservation carries its group, a pod
carries the bit mask of the groups it matches and KOORDHIP_POD_RESV_AFFINITY
when it has a required reservation affinity (reservation.go:444-487: no
matched reservation on a node -> UnschedulableAndUnresolvable, plugin.go:
378-381).  Reserve pods are not streamed by this engine (MarshalError).
"""
from __future__ import annotations

import json
import re
from dataclasses import dataclass, field
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np

from . import abi, k8s
from .snapshot import RESV_COLS as RESV_COLUMNS, NodeTable, slot_col

LABEL_RESERVATION_ORDER = "scheduling.koordinator.sh/reservation-order"   # apis/extension/reservation.go
ANNOTATION_RESERVATION_AFFINITY = "scheduling.koordinator.sh/reservation-affinity"
ANNOTATION_RESERVE_POD = "scheduling.koordinator.sh/reserve-pod"

POLICY_DEFAULT, POLICY_ALIGNED, POLICY_RESTRICTED = "", "Aligned", "Restricted"
_POLICY_CODE = {POLICY_DEFAULT: abi.RESV_POLICY_DEFAULT, POLICY_ALIGNED: abi.RESV_POLICY_ALIGNED,
                POLICY_RESTRICTED: abi.RESV_POLICY_RESTRICTED}


class ReservationError(ValueError):
    pass


OwnerReference = k8s.OwnerReference


@dataclass
class LabelSelectorRequirement:
    key: str
    operator: str                 # In, NotIn, Exists, DoesNotExist
    values: List[str] = field(default_factory=list)


@dataclass
class LabelSelector:
    match_labels: Dict[str, str] = field(default_factory=dict)
    match_expressions: List[LabelSelectorRequirement] = field(default_factory=list)

    def validate(self):
        """metav1.LabelSelectorAsSelector's validation (the owner's ParseError)."""
        for r in self.match_expressions:
            if r.operator in ("In", "NotIn"):
                if not r.values:
                    raise ReservationError(f"values must be non-empty for operator {r.operator}")
            elif r.operator in ("Exists", "DoesNotExist"):
                if r.values:
                    raise ReservationError(f"values must be empty for operator {r.operator}")
            else:
                raise ReservationError(f"{r.operator!r} is not a valid label selector operator")

    def matches(self, labels: Dict[str, str]) -> bool:
        for k, v in self.match_labels.items():
            if labels.get(k) != v:
                return False
        for r in self.match_expressions:
            has = r.key in labels
            if r.operator == "In" and not (has and labels[r.key] in r.values):
                return False
            if r.operator == "NotIn" and has and labels[r.key] in r.values:
                return False
            if r.operator == "Exists" and not has:
                return False
            if r.operator == "DoesNotExist" and has:
                return False
        return True


@dataclass
class ObjectRef:
    """corev1.ObjectReference of ReservationOwner.Object."""
    uid: str = ""
    name: str = ""
    namespace: str = ""
    api_version: str = ""


@dataclass
class ControllerRef:
    """ReservationControllerReference."""
    kind: str = ""
    name: str = ""
    uid: str = ""
    api_version: str = ""
    namespace: str = ""
    controller: Optional[bool] = None


@dataclass
class ReservationOwner:
    object: Optional[ObjectRef] = None
    controller: Optional[ControllerRef] = None
    label_selector: Optional[LabelSelector] = None

    def key(self) -> str:
        """Canonical form (owner groups are distinct owner lists)."""
        def enc(x):
            if x is None:
                return None
            if isinstance(x, LabelSelector):
                return {"l": sorted(x.match_labels.items()),
                        "e": [(r.key, r.operator, sorted(r.values)) for r in x.match_expressions]}
            return sorted(vars(x).items())
        return json.dumps([enc(self.object), enc(self.controller), enc(self.label_selector)], sort_keys=True)


def match_object_ref(pod: k8s.Pod, ref: Optional[ObjectRef]) -> bool:
    """MatchObjectRef, reservation.go:412-420."""
    if ref is None:
        return True
    return ((not ref.uid or pod.uid == ref.uid) and (not ref.name or pod.name == ref.name)
            and (not ref.namespace or pod.namespace == ref.namespace)
            and (not ref.api_version or pod.api_version == ref.api_version))


def match_controller_ref(pod: k8s.Pod, ref: Optional[ControllerRef]) -> bool:
    """MatchReservationControllerReference, reservation.go:422-442."""
    if ref is None:
        return True
    if ref.namespace and ref.namespace != pod.namespace:
        return False
    for o in pod.owner_refs:
        if ((ref.controller is None or (o.controller is not None and ref.controller == o.controller))
                and (not ref.uid or ref.uid == o.uid) and (not ref.name or ref.name == o.name)
                and (not ref.kind or ref.kind == o.kind) and (not ref.api_version or ref.api_version == o.api_version)):
            return True
    return False


def match_owners(pod: k8s.Pod, owners: Sequence[ReservationOwner]) -> bool:
    """MatchReservationOwners (reservation.go:389-410): owners == [] matches nothing."""
    for m in owners:
        if (match_object_ref(pod, m.object) and match_controller_ref(pod, m.controller)
                and (m.label_selector is None or m.label_selector.matches(pod.labels))):
            return True
    return False


@dataclass
class NodeSelectorRequirement:
    key: str
    operator: str                 # In, NotIn, Exists, DoesNotExist, Gt, Lt
    values: List[str] = field(default_factory=list)


@dataclass
class NodeSelectorTerm:
    match_expressions: List[NodeSelectorRequirement] = field(default_factory=list)
    match_fields: List[NodeSelectorRequirement] = field(default_factory=list)


def _req_matches(r: NodeSelectorRequirement, labels: Dict[str, str]) -> bool:
    """(upstream) component-helpers nodeaffinity / labels.Requirement.Matches."""
    has = r.key in labels
    if r.operator == "In":
        return has and labels[r.key] in r.values
    if r.operator == "NotIn":
        return not has or labels[r.key] not in r.values
    if r.operator == "Exists":
        return has
    if r.operator == "DoesNotExist":
        return not has
    if r.operator in ("Gt", "Lt"):
        if not has:
            return False
        try:
            a, b = int(labels[r.key]), int(r.values[0])
        except (ValueError, IndexError):
            return False
        return a > b if r.operator == "Gt" else a < b
    return False


@dataclass
class ReservationAffinity:
    """apis/extension ReservationAffinity as GetRequiredReservationAffinity reads it
    (pkg/util/reservation/reservation.go:444-487): a label set the reservation
    must carry and node-selector terms over a fake node whose labels are the
    node's overlaid with the reservation's and whose name is the reservation's
    (reservation/transformer.go:335-359)."""
    selector: Dict[str, str] = field(default_factory=dict)
    terms: Optional[List[NodeSelectorTerm]] = None

    def key(self) -> str:
        return json.dumps([sorted(self.selector.items()),
                           None if self.terms is None else
                           [[[(r.key, r.operator, sorted(r.values)) for r in t.match_expressions],
                             [(r.key, r.operator, sorted(r.values)) for r in t.match_fields]] for t in self.terms]])

    def matches(self, node_labels: Dict[str, str], resv: "Reservation") -> bool:
        labels = dict(node_labels or {})
        labels.update(resv.labels or {})
        for k, v in self.selector.items():
            if labels.get(k) != v:
                return False
        if self.terms is None:
            return True
        for t in self.terms:                          # NodeSelector: terms ORed, a term's parts ANDed
            if not t.match_expressions and not t.match_fields:
                continue
            ok = all(_req_matches(r, labels) for r in t.match_expressions)
            ok = ok and all(_req_matches(r, {"metadata.name": resv.name}) for r in t.match_fields)
            if ok:
                return True
        return False


_NODE_SELECTOR_OPS = {"In", "NotIn", "Exists", "DoesNotExist", "Gt", "Lt"}


def parse_reservation_affinity(annotations: Dict[str, str]) -> Optional[ReservationAffinity]:
    """GetRequiredReservationAffinity: None without a selector or required terms;
    ReservationError on a malformed annotation / selector (the reference's
    BeforePreFilter error)."""
    raw = (annotations or {}).get(ANNOTATION_RESERVATION_AFFINITY, "")
    if not raw:
        return None
    try:
        a = json.loads(raw)
    except ValueError as e:
        raise ReservationError(f"reservation affinity: {e}") from e
    sel = a.get("reservationSelector") or {}
    req = a.get("requiredDuringSchedulingIgnoredDuringExecution")
    if not sel and req is None:
        return None
    terms = None
    if req is not None:
        terms = []
        for t in req.get("reservationSelectorTerms") or []:
            def reqs(xs, fields=False):
                out = []
                for x in xs or []:
                    op = x.get("operator", "")
                    vals = list(x.get("values") or [])
                    if op not in _NODE_SELECTOR_OPS or (fields and (x.get("key") != "metadata.name" or op not in ("In", "NotIn"))):
                        raise ReservationError(f"reservation affinity: unsupported requirement {x}")
                    if op in ("In", "NotIn") and not vals or op in ("Exists", "DoesNotExist") and vals \
                            or op in ("Gt", "Lt") and len(vals) != 1:
                        raise ReservationError(f"reservation affinity: invalid requirement {x}")
                    out.append(NodeSelectorRequirement(x.get("key", ""), op, vals))
                return out
            terms.append(NodeSelectorTerm(reqs(t.get("matchExpressions")), reqs(t.get("matchFields"), True)))
    return ReservationAffinity(dict(sel), terms)


@dataclass
class Reservation:
    """A scheduling.koordinator.sh/v1alpha1 Reservation as the scheduler cache holds it."""
    name: str
    node_name: str = ""                      # Status.NodeName
    phase: str = "Available"
    uid: str = ""
    labels: Dict[str, str] = field(default_factory=dict)
    owners: List[ReservationOwner] = field(default_factory=list)
    allocatable: k8s.ResourceList = field(default_factory=dict)   # Status.Allocatable (Available)
    template: List[k8s.Container] = field(default_factory=list)    # Spec.Template containers (the reserve pod)
    allocated: k8s.ResourceList = field(default_factory=dict)      # ReservationInfo.Allocated
    assigned: int = 0                                              # len(AssignedPods)
    allocate_once: Optional[bool] = None                           # Spec.AllocateOnce (nil -> true)
    allocate_policy: str = POLICY_DEFAULT
    unschedulable: bool = False
    deleting: bool = False                                         # DeletionTimestamp set
    # NodeNUMAResource: the reserve pod's cpuset allocation (its resource-status
    # annotation, held in NodeAllocation under the reservation's UID) and the
    # union of its AssignedPods' cpusets (RestoreReservation,
    # nodenumaresource/reservation.go:84-104)
    cpus: List[int] = field(default_factory=list)
    assigned_cpus: List[int] = field(default_factory=list)
    cpu_exclusive: str = ""                                        # the reserve pod's preferredCPUExclusivePolicy
    spec_node_name: str = ""                                       # Spec.Template.Spec.NodeName (a pinned reservation)
    # a bound pod in the reservation operating mode (operating_pod_reservation):
    # the pod is its own reserve pod; parse_error: its owners annotation did not
    # parse (ReservationInfo.ParseError: it matches no pod)
    pod: Optional[k8s.Pod] = None
    parse_error: bool = False
    # metadata.annotations: NewReservePod copies them onto the reserve pod
    # (util/reservation/reservation.go:75-80), so the device-allocated one is the
    # reserve pod's DeviceShare allocation (deviceshare/reservation.go:139-141)
    annotations: Dict[str, str] = field(default_factory=dict)
    # each AssignedPod's device allocation on the node (its device-allocated
    # annotation: nd.getUsed of the assigned pod, reservation.go:145-151)
    assigned_devices: List[dict] = field(default_factory=list)

    def reserved_cpus(self) -> List[int]:
        """RestoreReservation's reservedCPUs of this reservation: its allocated
        CPUs less its assigned pods' (reservation.go:84-104)."""
        taken = set(self.assigned_cpus)
        return sorted(c for c in set(self.cpus) if c not in taken)

    def is_available(self) -> bool:
        return bool(self.node_name) and self.phase == "Available"

    def reserve_pod(self) -> k8s.Pod:
        if self.pod is not None:
            return self.pod
        return k8s.Pod(name=f"reserve-{self.name}", uid=self.uid, annotations=dict(self.annotations or {}),
                       labels=dict(self.labels or {}), node_name=self.node_name,
                       containers=list(self.template) or [k8s.Container(requests=dict(self.allocatable))])

    def device_allocation(self) -> dict:
        """The reserve pod's DeviceShare allocation {type: [(minor, {resource: value})]}
        (its device-allocated annotation; an operating-mode pod's own)."""
        from .deviceshare import parse_device_allocated
        return parse_device_allocated(self.pod.annotations if self.pod is not None else self.annotations)


ANNOTATION_RESERVATION_NAME = "scheduling.koordinator.sh/reservation-name"
ANNOTATION_RESERVATION_NODE = "scheduling.koordinator.sh/reservation-node"


def is_reserve_pod(pod: k8s.Pod) -> bool:
    """IsReservePod, util/reservation/reservation.go:172-174."""
    return (pod.annotations or {}).get(ANNOTATION_RESERVE_POD) == "true"


def new_reserve_pod(r: Reservation) -> k8s.Pod:
    """NewReservePod (util/reservation/reservation.go:53-110) of a pending
    reservation: the template's containers, the reservation's labels, the
    reserve-pod / reservation-name annotations and, for a pinned reservation,
    the reservation-node annotation (spec.nodeName cleared); priority 0 when
    unset."""
    ann = dict(r.annotations or {})
    ann.update({ANNOTATION_RESERVE_POD: "true", ANNOTATION_RESERVATION_NAME: r.name})
    if r.spec_node_name:
        ann[ANNOTATION_RESERVATION_NODE] = r.spec_node_name
    return k8s.Pod(name=reservation_key(r), uid=r.uid, labels=dict(r.labels), annotations=ann, priority=0,
                   containers=list(r.template) or [k8s.Container(requests=dict(r.allocatable))])


def reservation_key(r: Reservation) -> str:
    """GetReservationKey: the UID when set, else the name."""
    return r.uid or r.name


def reserve_pod_fields(rec, ext_rec, pod: k8s.Pod, reservations: Dict[str, Reservation],
                       node_index: Dict[str, int]) -> None:
    """Mark a reserve pod's koordhip_pod record (KOORDHIP_POD_RESERVE, its
    reservation's AllocatePolicy; no reservation matches it, transformer.go:60,96)
    and its koordhip_pod_ext.reserve_node (the node its reservation names,
    plugin.go:335-339; ext_rec None: the pod may not name one)."""
    name = (pod.annotations or {}).get(ANNOTATION_RESERVATION_NAME, "")
    r = reservations.get(name)
    if r is None:                                    # rLister.Get fails: framework.Error (plugin.go:341-344)
        raise ReservationError(f"reserve pod {pod.key}: reservation {name!r} not found")
    if r.allocate_policy not in _POLICY_CODE:
        raise ReservationError(f"reservation {r.name}: unknown allocate policy {r.allocate_policy!r}")
    rec["flags"] = int(rec["flags"]) | abi.POD_RESERVE | (_POLICY_CODE[r.allocate_policy] << abi.POD_RESERVE_POLICY_SHIFT)
    rec["flags"] = int(rec["flags"]) & ~abi.POD_RESV_AFFINITY
    rec["resv_match"] = 0
    node = (pod.annotations or {}).get(ANNOTATION_RESERVATION_NODE, "")
    if node and ext_rec is not None:
        if node not in node_index:       # (the reference finds no node; the record cannot say "none")
            raise ReservationError(f"reserve pod {pod.key}: node {node!r} is not in the snapshot")
        ext_rec["reserve_node"] = node_index[node] + 1


LABEL_POD_OPERATING_MODE = "scheduling.koordinator.sh/operating-mode"


def is_reservation_operating_pod(pod: k8s.Pod) -> bool:
    """IsReservationOperatingMode, apis/extension/operating_pod.go:51-53."""
    return (pod.labels or {}).get(LABEL_POD_OPERATING_MODE) == "Reservation"


ANNOTATION_RESERVATION_ALLOCATED = "scheduling.koordinator.sh/reservation-allocated"   # apis/extension/reservation.go:37
ANNOTATION_RESERVATION_OWNERS = "scheduling.koordinator.sh/reservation-owners"
ANNOTATION_RESERVATION_CURRENT_OWNER = "scheduling.koordinator.sh/reservation-current-owner"


def _owner_from_json(o: dict) -> ReservationOwner:
    def ref(d, cls, keys):
        if d is None:
            return None
        return cls(**{k: d.get(j, "") for k, j in keys})
    obj = ref(o.get("object"), ObjectRef, [("uid", "uid"), ("name", "name"), ("namespace", "namespace"),
                                           ("api_version", "apiVersion")])
    ctl = o.get("controller")
    ctrl = None if ctl is None else ControllerRef(kind=ctl.get("kind", ""), name=ctl.get("name", ""),
                                                  uid=ctl.get("uid", ""), api_version=ctl.get("apiVersion", ""),
                                                  namespace=ctl.get("namespace", ""), controller=ctl.get("controller"))
    ls = o.get("labelSelector")
    sel = None
    if ls is not None:
        sel = LabelSelector(match_labels=dict(ls.get("matchLabels") or {}),
                            match_expressions=[LabelSelectorRequirement(x.get("key", ""), x.get("operator", ""),
                                                                        list(x.get("values") or []))
                                               for x in ls.get("matchExpressions") or []])
    return ReservationOwner(object=obj, controller=ctrl, label_selector=sel)


def reservation_allocated(pod: k8s.Pod) -> Optional[Tuple[str, str]]:
    """GetReservationAllocated: the (uid, name) of the reservation a pod was
    assumed into (its reservation-allocated annotation), None without one or on
    a parse error."""
    raw = (pod.annotations or {}).get(ANNOTATION_RESERVATION_ALLOCATED, "")
    if not raw:
        return None
    try:
        a = json.loads(raw)
        return str(a.get("uid", "") or ""), str(a.get("name", "") or "")
    except (ValueError, TypeError, AttributeError):
        return None


def current_owner(pod: k8s.Pod) -> Optional[Tuple[str, str, str]]:
    """GetReservationCurrentOwner: (namespace, name, uid) of the pod the
    operating-mode pod serves, None without one or on a parse error."""
    raw = (pod.annotations or {}).get(ANNOTATION_RESERVATION_CURRENT_OWNER, "")
    if not raw:
        return None
    try:
        o = json.loads(raw)
        return str(o.get("namespace", "") or ""), str(o.get("name", "") or ""), str(o.get("uid", "") or "")
    except (ValueError, TypeError, AttributeError):
        return None


def operating_reservation_name(pod: k8s.Pod) -> str:
    return f"operating-pod/{pod.namespace}/{pod.name}"


def operating_pod_reservation(pod: k8s.Pod) -> Optional[Reservation]:
    """The reservation cache's entry for a bound pod in the reservation
    operating mode (pod_eventhandler.go:104-124 -> cache.go:139-161,
    NewReservationInfoFromPod, frameworkext/reservation_info.go:101-126):
    Allocatable / ResourceNames = its PodRequestsAndLimits requests, owners from
    its reservation-owners annotation (a parse error: it matches no pod), always
    AllocateOnce (reservation_info.go:185-194), AllocatePolicy Aligned
    (:196-204), Available while the pod runs and is Ready (:238-246),
    unschedulable while terminating (:248-255), and its reservation-current-
    owner annotation as an assigned pod (cache.go:152-160; with AllocateOnce
    that takes it out of matching).  The pod itself is its reserve pod (a
    NodeInfo pod already).  None for any other pod."""
    if not is_reservation_operating_pod(pod) or not pod.node_name:
        return None
    reqs, _ = k8s.pod_requests_and_limits(pod)
    ann = pod.annotations or {}
    owners, perr = [], False
    raw = ann.get(ANNOTATION_RESERVATION_OWNERS, "")
    if raw:
        try:
            owners = [_owner_from_json(o) for o in json.loads(raw)]
        except (ValueError, TypeError, AttributeError):
            owners, perr = [], True
    assigned = 0
    cur = ann.get(ANNOTATION_RESERVATION_CURRENT_OWNER, "")
    if cur:
        try:
            json.loads(cur)
            assigned = 1
        except ValueError:
            assigned = 0              # (logged by the reference; no owner added)
    return Reservation(name=operating_reservation_name(pod), node_name=pod.node_name,
                       phase="Available" if (pod.phase == "Running" and pod.ready) else "Pending",
                       uid=pod.uid, labels=dict(pod.labels or {}), owners=owners, allocatable=dict(reqs),
                       allocated={}, assigned=assigned, allocate_once=True, allocate_policy=POLICY_ALIGNED,
                       deleting=pod.deleting, pod=pod, parse_error=perr)


def parse_order(labels: Dict[str, str]) -> int:
    """findMostPreferredReservationByOrder's label parse (scoring.go:160-167): 0 = unordered."""
    s = labels.get(LABEL_RESERVATION_ORDER, "")
    if not re.fullmatch(r"[+-]?[0-9]+", s):
        return 0
    v = int(s)
    if not (-(1 << 63) <= v < (1 << 63)):
        return 0                              # ParseInt range error
    return v


@dataclass
class ReservationIndex:
    """Owner groups of a snapshot's reservations (pods are matched against them).

    A group is a distinct (owner spec, results of the registered reservation
    affinities on the reservation) pair: a pod's bit g is MatchReservationOwners
    against the group's owners AND, for a pod with a required reservation
    affinity, that affinity's result on the group's reservations
    (matchReservation, reservation/transformer.go:335-359).  Affinities must be
    registered before the columns are built (register_affinities); a new one
    regroups every reservation (the columns and earlier pod masks are stale)."""
    groups: List[List[ReservationOwner]] = field(default_factory=list)
    group_of: Dict[str, int] = field(default_factory=dict)
    affinities: List[ReservationAffinity] = field(default_factory=list)
    group_aff: List[Tuple[bool, ...]] = field(default_factory=list)

    def register_affinities(self, pods) -> bool:
        """Register the required reservation affinities of `pods`; True when any
        was new (then rebuild the reservation columns and the pod masks)."""
        known = {a.key() for a in self.affinities}
        new = False
        for p in pods:
            a = parse_reservation_affinity(p.annotations or {})
            if a is not None and a.key() not in known:
                self.affinities.append(a)
                known.add(a.key())
                new = True
        if new:
            self.groups, self.group_of, self.group_aff = [], {}, []
        return new

    def group(self, owners: List[ReservationOwner], node_labels: Optional[Dict[str, str]] = None,
              resv: Optional["Reservation"] = None) -> int:
        res = tuple(a.matches(node_labels or {}, resv) if resv is not None else False for a in self.affinities)
        key = json.dumps([[o.key() for o in owners], res])
        g = self.group_of.get(key)
        if g is None:
            if len(self.groups) >= abi.RESV_MAX_GROUPS:
                raise ReservationError(f"more than {abi.RESV_MAX_GROUPS} distinct reservation owner / affinity groups")
            g = len(self.groups)
            self.groups.append(list(owners))
            self.group_aff.append(res)
            self.group_of[key] = g
        return g

    def pod_mask(self, pod: k8s.Pod) -> int:
        """koordhip_pod.resv_match: bit g set iff the pod matches group g."""
        if (pod.annotations or {}).get(ANNOTATION_RESERVE_POD) == "true":
            return 0                # a reserve pod matches no reservation (transformer.go:60,96)
        aff = parse_reservation_affinity(pod.annotations or {})
        ai = None
        if aff is not None:
            keys = [a.key() for a in self.affinities]
            if aff.key() not in keys:
                raise ReservationError("a reservation affinity not registered with this snapshot's index")
            ai = keys.index(aff.key())
        m = 0
        for g, owners in enumerate(self.groups):
            if match_owners(pod, owners) and (ai is None or self.group_aff[g][ai]):
                m |= 1 << g
        return m


def _q2(rl: k8s.ResourceList, name: str) -> int:
    q = rl.get(name)
    if q is None:
        return 0
    return q.milli_value() if name == k8s.CPU else q.value()


def available_by_node(node_index: Dict[str, int], reservations: Sequence[Reservation],
                      overflow: Optional[list] = None) -> Dict[int, List[Reservation]]:
    """The reservation cache's Available reservations by node row (cache.go:236-252),
    each node's in the given order: its reservation slots.  The reference keeps
    them in a map and breaks nomination ties by its iteration order; here the
    lowest slot wins (include/koordhip.h KOORDHIP_RESV_SLOTS).  More than
    RESV_SLOTS_MAX on a node raise -- except, with `overflow` given, bound
    operating-mode pods past the limit, which stay plain NodeInfo pods and are
    appended to `overflow` (outside the engine's envelope, counted by the caller)."""
    placed: Dict[int, List[Reservation]] = {}
    for r in reservations:
        if not r.is_available() or r.node_name not in node_index:
            continue
        rs = placed.setdefault(node_index[r.node_name], [])
        if len(rs) >= abi.RESV_SLOTS_MAX:
            if overflow is not None and r.pod is not None:
                overflow.append(r)
                continue
            raise ReservationError(f"node {r.node_name}: more than {abi.RESV_SLOTS_MAX} Available reservations")
        rs.append(r)
    return placed


def reservation_unsupported(r: Reservation, devices: bool) -> Optional[str]:
    """Why the engine cannot hold `r` as a reservation slot (None: it can):
    Allocatable keys other than cpu / memory and -- with DeviceShare's device
    columns (`devices`) -- the device scalars."""
    from .deviceshare import XRES_INDEX
    allowed = {k8s.CPU, k8s.MEMORY} | (set(XRES_INDEX) if devices else set())
    extra = set(r.allocatable) - allowed
    if extra:
        return f"resources {sorted(extra)}"
    if any(r.allocatable[n].value() <= 0 for n in set(r.allocatable) & set(XRES_INDEX)):
        return "a zero-valued extended resource"
    return None


def slots_needed(placed: Dict[int, List[Reservation]]) -> int:
    return max([1] + [len(rs) for rs in placed.values()])


def order_ranks(reservations: Iterable) -> Dict[int, int]:
    """Rank of every distinct non-zero reservation-order label value (ascending)
    (reservations: Reservation objects or per-node lists of them)."""
    flat = [x for r in reservations for x in (r if isinstance(r, list) else [r])]
    orders = sorted({parse_order(r.labels) for r in flat} - {0})
    if len(orders) > abi.RESV_MAX_ORDERS:
        raise ReservationError(f"more than {abi.RESV_MAX_ORDERS} distinct reservation orders")
    return {v: k for k, v in enumerate(orders)}


def clear_reservation_row(table: NodeTable, i):
    for q in range(table.resv_slots):
        for c in RESV_COLUMNS:
            table[slot_col(c, q)][i] = 0
    if table.has_resv_dev:
        table["resv_dev_slot"][i] = -1
        for c in ("resv_dev", "resv_xalloc", "resv_xallocated"):
            table[c][i] = 0


def reservation_row(table: NodeTable, i: int, r, index: "ReservationIndex", rank: Dict[int, int],
                    node_labels: Optional[Dict[str, str]] = None):
    """Row i of the resv_* columns for node i's Available reservations r (one
    Reservation or a list, one per slot; node_labels: what reservation
    affinities see of the node)."""
    rs = r if isinstance(r, list) else [r]
    if len(rs) > table.resv_slots:
        raise ReservationError(f"{len(rs)} reservations on a node of a table with {table.resv_slots} slots")
    clear_reservation_row(table, i)
    for q, x in enumerate(rs):
        _reservation_slot(table, i, q, x, index, rank, node_labels)
    device_reservation_row(table, i, rs)


def device_reservation_row(table: NodeTable, i: int, rs: List[Reservation]):
    """Row i of the device-holding reservation columns (resv_dev_slot, resv_dev,
    resv_xalloc, resv_xallocated) for node i's reservations `rs` in slot order:
    DeviceShare's RestoreReservation state (deviceshare/reservation.go:119-170)
    -- the reserve pod's device allocation as the reservation's allocatable, its
    AssignedPods' allocations on those minors as its allocated
    (appendAllocatedByHints) -- and the reservation's NodeResourcesFit extended
    scalars (Allocatable; Allocated masked to its keys).  The engine holds one
    such reservation per node; a reservation listing extended scalars must hold
    devices (its scalars ride on that slot)."""
    from .deviceshare import TYPE_INDEX, TYPE_RESOURCES, XRES_INDEX
    held = [(q, r) for q, r in enumerate(rs) if r.device_allocation() or set(r.allocatable) & set(XRES_INDEX)]
    if not table.has_resv_dev:
        if held:
            raise ReservationError(f"reservation {held[0][1].name}: a reservation holding devices needs the "
                                   "device-holding reservation columns (DeviceShare with devices; NodeTable.enable_resv_dev)")
        return
    table["resv_dev_slot"][i] = -1
    table["resv_dev"][i] = 0
    table["resv_xalloc"][i] = 0
    table["resv_xallocated"][i] = 0
    if not held:
        return
    if len(held) > 1:
        raise ReservationError(f"node {i}: more than one reservation holding devices (the engine holds one per node)")
    q, r = held[0]
    alloc = r.device_allocation()
    if not alloc:
        raise ReservationError(f"reservation {r.name}: extended resources in its Allocatable but no device allocation")
    slot_of = {(typ, int(table["dev_minor"][i, t, s])): s for typ, t in TYPE_INDEX.items()
               for s in range(table.dev_slots) if table["dev_minor"][i, t, s] >= 0}
    A = table["resv_dev"][i, 0]
    D = table["resv_dev"][i, 1]
    for typ, items in alloc.items():
        for minor, res in items:
            s = slot_of.get((typ, minor))
            if s is None:
                raise ReservationError(f"reservation {r.name}: device {typ}/{minor} is not on its node")
            for k, n in enumerate(TYPE_RESOURCES[typ]):
                A[TYPE_INDEX[typ], s, k] += res.get(n, 0)
    for pa in r.assigned_devices:         # appendAllocatedByHints: only the reservation's minors
        for typ, items in pa.items():
            for minor, res in items:
                s = slot_of.get((typ, minor))
                if s is None or not A[TYPE_INDEX[typ], s].any():
                    continue
                for k, n in enumerate(TYPE_RESOURCES[typ]):
                    D[TYPE_INDEX[typ], s, k] += res.get(n, 0)
    if not A.any():
        raise ReservationError(f"reservation {r.name}: its device allocation holds no resources")
    table["resv_dev_slot"][i] = q
    for n in set(r.allocatable) & set(XRES_INDEX):
        j = XRES_INDEX[n]
        table["resv_xalloc"][i, j] = r.allocatable[n].value()
        table["resv_xallocated"][i, j] = r.allocated[n].value() if n in r.allocated else 0


def _reservation_slot(table: NodeTable, i: int, q: int, r: Reservation, index: "ReservationIndex",
                      rank: Dict[int, int], node_labels: Optional[Dict[str, str]]):
    from .marshal import nonzero_request, fit_request

    from .deviceshare import XRES_INDEX, fit_xreq
    col = lambda c: table[slot_col(c, q)]
    names = set(r.allocatable)
    xnames = names & set(XRES_INDEX)
    extra = names - {k8s.CPU, k8s.MEMORY} - xnames
    if extra:
        raise ReservationError(f"reservation {r.name}: resources {sorted(extra)} are not supported")
    for n in sorted(xnames):
        if r.allocatable[n].value() <= 0:     # (a zero-valued key: Restricted's LessThanOrEqual still reads it)
            raise ReservationError(f"reservation {r.name}: a zero-valued extended resource {n!r} in its Allocatable")
    parse_ok = not r.parse_error
    try:
        for o in r.owners:
            if o.label_selector is not None:
                o.label_selector.validate()
    except ReservationError:
        parse_ok = False                                  # ReservationInfo.ParseError
    pod = r.reserve_pod()
    req, present = fit_request(pod)
    if present - {k8s.CPU, k8s.MEMORY} - set(XRES_INDEX) or \
            any(req[k] for k in range(abi.NRES) if k not in (abi.RES_CPU, abi.RES_MEM)):
        raise ReservationError(f"reservation {r.name}: the reserve pod requests resources other than cpu, memory and "
                               "device scalars")
    if req[abi.RES_CPU] != _q2(r.allocatable, k8s.CPU) or req[abi.RES_MEM] != _q2(r.allocatable, k8s.MEMORY) or \
            fit_xreq(pod) != {n: r.allocatable[n].value() for n in xnames}:
        raise ReservationError(f"reservation {r.name}: allocatable differs from the reserve pod's requests")
    f = abi.RESV_PRESENT if parse_ok else 0
    if r.allocate_once is None or r.allocate_once:
        f |= abi.RESV_ALLOCATE_ONCE
    if r.unschedulable or r.deleting:
        f |= abi.RESV_UNSCHEDULABLE
    order = parse_order(r.labels)
    if order != 0:
        if order not in rank:
            raise ReservationError(f"reservation {r.name}: order {order} has no rank in this snapshot")
        f |= abi.RESV_ORDERED
        col("resv_order_rank")[i] = rank[order]
    if k8s.CPU in names:
        f |= abi.RESV_KEY_CPU
    if k8s.MEMORY in names:
        f |= abi.RESV_KEY_MEM
    if r.allocate_policy not in _POLICY_CODE:
        raise ReservationError(f"reservation {r.name}: unknown allocate policy {r.allocate_policy!r}")
    f |= _POLICY_CODE[r.allocate_policy] << abi.RESV_POLICY_SHIFT
    f |= index.group(r.owners, node_labels, r) << abi.RESV_GROUP_SHIFT
    col("resv_flags")[i] = f
    col("resv_alloc0")[i] = _q2(r.allocatable, k8s.CPU)
    col("resv_alloc1")[i] = _q2(r.allocatable, k8s.MEMORY)
    nzc, nzm = nonzero_request(pod)
    col("resv_nz0")[i] = nzc
    col("resv_nz1")[i] = nzm
    # Allocated masked to ResourceNames (reservation_info.go:286, 303)
    col("resv_allocated0")[i] = _q2(r.allocated, k8s.CPU) if k8s.CPU in names else 0
    col("resv_allocated1")[i] = _q2(r.allocated, k8s.MEMORY) if k8s.MEMORY in names else 0
    col("resv_assigned")[i] = r.assigned
    m = reserved_cpu_mask(table, i, r)
    for w in range(abi.NUMA_WORDS):
        col(f"resv_cpus{w}")[i] = m[w]


def reserved_cpu_mask(table: NodeTable, i: int, r: Reservation) -> List[int]:
    """The resv_cpus words of reservation r on node i: its reserved CPUs as
    core-major positions of the node's topology class.  A node without a (valid)
    CPU topology holds no allocation (resourceManager.Update skips it,
    resource_manager.go:328-339), so nothing is reserved there."""
    words = [0] * abi.NUMA_WORDS
    cpus = r.reserved_cpus()
    cls = int(table["numa_class"][i])
    if not cpus or cls < 0 or cls >= len(table.numa_classes):
        return words
    rec = table.numa_classes[cls]
    pos_of = {int(rec["cpu_id"][p]): p for p in range(int(rec["num_cpus"]))}
    for c in cpus:
        p = pos_of.get(c)
        if p is None:
            raise ReservationError(f"reservation {r.name}: CPU {c} is not in node {i}'s topology")
        words[p >> 6] |= 1 << (p & 63)
    for w in range(abi.NUMA_WORDS):
        if words[w] & int(table[f"numa_free{w}"][i]):
            raise ReservationError(f"reservation {r.name}: its CPUs must be allocated on node {i} (NodeAllocation "
                                   "holds the reserve pod's cpuset)")
    return words


def reservation_columns(table: NodeTable, node_index: Dict[str, int], reservations: Sequence[Reservation],
                        index: Optional[ReservationIndex] = None,
                        node_labels: Optional[Dict[str, Dict[str, str]]] = None,
                        overflow: Optional[list] = None) -> ReservationIndex:
    """Fill the resv_* columns of `table` (the reservation cache's view,
    cache.go:236-252) and return the owner groups for the pod masks
    (node_labels: node name -> labels, for reservation affinities)."""
    index = index or ReservationIndex()
    placed = available_by_node(node_index, reservations, overflow)
    table.set_resv_slots(max(table.resv_slots, slots_needed(placed)))
    clear_reservation_row(table, slice(None))
    rank = order_ranks(placed.values())
    for i, rs in placed.items():
        reservation_row(table, i, rs, index, rank, (node_labels or {}).get(rs[0].node_name))
    return index


def pod_keys(pod: k8s.Pod) -> int:
    """KOORDHIP_POD_KEY_* bits: the cpu / memory keys of PodRequestsAndLimits,
    and KOORDHIP_POD_RESV_AFFINITY for a required reservation affinity."""
    reqs, _ = k8s.pod_requests_and_limits(pod)
    f = (abi.POD_KEY_CPU if k8s.CPU in reqs else 0) | (abi.POD_KEY_MEM if k8s.MEMORY in reqs else 0)
    if parse_reservation_affinity(pod.annotations or {}) is not None:
        f |= abi.POD_RESV_AFFINITY
    return f
