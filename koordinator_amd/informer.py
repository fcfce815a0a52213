"""Event-driven marshaller: the scheduler's informer handlers kept as a
ClusterState, turned into row deltas for ``koordhip_update_nodes``.

The reference keeps its plugin state current with informer callbacks:
LoadAwareScheduling's podAssignCache (loadaware/pod_assign_cache.go:53-117),
the scheduler cache's NodeInfo (upstream: assigned, non-terminated pods),
the pod lister that buildPodMetricMap consults (loadaware/helper.go:153-170)
and the NodeMetric lister (load_aware.go:123-133, 269-287).  Every Filter /
Score call then reads that state.  Here each event updates the same
ClusterState that ``marshal.build_table`` reads and marks the node rows it can
change dirty; ``flush`` recomputes only those rows (``marshal.node_row``) and
hands them to the engine in one ``update_nodes`` call.  A flush also
re-derives the rows whose NodeMetric crossed its expiry since the previous
flush (the only input that changes with time alone).

The node SET is positional on the device: adding or deleting a node needs a
new snapshot (``flush`` returns ``needs_reload``; ``table()`` builds it).
NodeNUMAResource columns come from NodeResourceTopology events (the NRT
handler, nodenumaresource/topology_eventhandler.go:62-113: TopologyOptions per
node) and from the pods' resource-status annotations (the NUMA pod handler,
pod_eventhandler.go:94-144: NodeAllocation per node, applied in event order --
an allocation that arrives while its node has no CPU topology is dropped, like
resourceManager.Update).  A table loaded without NRT objects keeps its NUMA
columns, carried over by node name across a reload.  Topology classes are
fixed at load_snapshot: an NRT with a new CPU topology shape needs a reload.

Reservations (the Reservation plugin's reservationCache, reservation/cache.go:
117-252, fed by the reservation informer) are kept by name; an add / update /
delete re-derives the resv_* columns of the nodes it leaves and enters.  Owner
groups are append-only (``resv_index``): pod masks made earlier stay valid.  A
reservation-order value the snapshot has no rank for needs a reload (ranks are
snapshot-wide).  Every reload rebuilds the owner groups from the live
reservations (pod masks made before it are stale); a new group past
RESV_MAX_GROUPS, or reserved CPUs on a snapshot loaded without the resv_cpus
columns, asks for a reload too.  ``register_pods`` registers the pods to
schedule (their reservation affinities and upstream static-filter classes)
before ``pod_records``; one the snapshot does not cover asks for a reload.

``flush`` hands the rows to the engine first and adopts them into the
informer's table image only when ``update_nodes`` succeeded, so a failed call
leaves the rows dirty for the next flush.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Set

import numpy as np

from . import abi, k8s
from .config import Profile
from . import numa as nm
from . import reservation as rv
from .marshal import AssignedPod, ClusterState, NewTopologyValue, build_table, is_node_metric_expired, node_row
from .snapshot import NodeTable


class PodAssignCache:
    """podAssignCache (loadaware/pod_assign_cache.go:35-117): node name ->
    pod UID -> (pod, assign timestamp)."""

    def __init__(self):
        self.items: Dict[str, Dict[str, AssignedPod]] = {}

    def assign(self, node_name: str, pod: k8s.Pod, now: float):
        """:53-68 -- pods without a node or terminated are not cached."""
        if node_name == "" or k8s.is_terminated(pod):
            return
        self.items.setdefault(node_name, {})[pod.uid] = AssignedPod(pod, now)

    def unassign(self, node_name: str, pod: k8s.Pod):
        """:70-80 -- the node's map goes away with its last pod."""
        if node_name == "":
            return
        m = self.items.get(node_name)
        if m is None:
            return
        m.pop(pod.uid, None)
        if not m:
            del self.items[node_name]

    def on_add(self, pod: k8s.Pod, now: float):
        self.assign(pod.node_name, pod, now)

    def on_update(self, old: Optional[k8s.Pod], new: k8s.Pod, now: float):
        """:91-101 -- a terminated pod leaves the cache, any other is (re)assigned."""
        if k8s.is_terminated(new):
            self.unassign(new.node_name, new)
        else:
            self.assign(new.node_name, new, now)

    def on_delete(self, pod: k8s.Pod):
        self.unassign(pod.node_name, pod)

    def node_list(self, node_name: str) -> List[AssignedPod]:
        return list(self.items.get(node_name, {}).values())


@dataclass
class FlushResult:
    rows: int = 0                 # rows handed to update_nodes
    needs_reload: bool = False    # the node set changed: load a new snapshot (table())
    expired_flips: int = 0        # rows re-derived because a NodeMetric crossed its expiry


class Informer:
    """Node / Pod / NodeMetric event handlers over one ClusterState."""

    def __init__(self, profile: Profile, nodes: List[k8s.Node] = (), now: float = 0.0):
        self.profile = profile
        self.cluster = ClusterState(nodes=list(nodes))
        self.assign_cache = PodAssignCache()
        self._index: Dict[str, int] = {n.name: i for i, n in enumerate(self.cluster.nodes)}
        self._pods_by_uid: Dict[str, k8s.Pod] = {}
        self._pod_node: Dict[str, str] = {}           # pod UID -> the node whose NodeInfo holds it
        self._metric_refs: Dict[str, Set[str]] = {}   # pod key -> nodes whose NodeMetric lists it
        self._dirty: Set[str] = set()
        self._reload = False
        self._expired: Dict[str, bool] = {}
        self._table: Optional[NodeTable] = None
        self._now = now
        self.reservations: Dict[str, rv.Reservation] = {}
        self.nrts: Dict[str, nm.NodeResourceTopology] = {}
        self._topo: Dict[str, nm.TopologyOptions] = {}      # topologyManager.topologyOptions
        self._alloc: Dict[str, nm.NodeAllocation] = {}      # resourceManager.nodeAllocations
        self._pod_alloc_node: Dict[str, str] = {}           # pod UID -> node whose NodeAllocation holds it
        self._classes: Optional[nm.ClassTable] = None
        self.resv_index = rv.ReservationIndex()
        self._resv_rank: Dict[int, int] = {}
        self._resv_cpus_loaded = False                      # the snapshot carried resv_cpus columns
        # NodeInfo's reserve pods of the Available reservations (the scheduler
        # cache holds them, frameworkext/eventhandlers/reservation_handler.go:
        # 250-281): reservation name -> the pod in cluster.node_pods
        self._resv_pods: Dict[str, k8s.Pod] = {}
        # AssignedPods from the pods' reservation-allocated annotation
        # (reservation/pod_eventhandler.go:95-131): reservation uid or name -> pod uid -> pod
        self._assigned: Dict[str, Dict[str, k8s.Pod]] = {}
        self._assigned_of: Dict[str, str] = {}              # pod uid -> the key it is assigned under
        # operating-mode pods: the reservation cache keeps their ReservationInfo
        # across updates (cache.go:139-161: UpdatePod refreshes the Allocatable
        # only; AddAssignedPod is cumulative): pod uid -> (owners, parse error,
        # the current owners seen: key -> (namespace, name, uid))
        self._op_state: Dict[str, tuple] = {}
        # bound operating-mode pods the engine cannot hold as a reservation slot
        # (unsupported resources, more than RESV_SLOTS_MAX on a node): they stay
        # plain NodeInfo pods; pod key -> reason
        self.outside_envelope: Dict[str, str] = {}
        from .nodefilters import StaticClasses
        from .topologyspread import SpreadRegistry
        self.static_classes = StaticClasses()
        self.cluster.spread = SpreadRegistry()
        from .interpodaffinity import IpaRegistry
        self.cluster.ipa = IpaRegistry(self.cluster.spread,
                                       hard_weight=profile.interpodaffinity.hard_pod_affinity_weight)

    # ---- full snapshot --------------------------------------------------------
    def table(self, now: float) -> NodeTable:
        """A full snapshot of the current state (initial load, or after the node set changed)."""
        self._sync_assigned()
        t = build_table(self.cluster, self.profile, now, self.static_classes)
        if self.nrts:
            self._classes = nm.ClassTable()
            for i, node in enumerate(self.cluster.nodes):
                self._numa_row(t, i, node, frozen=False)
            t.numa_classes = self._classes.records()
        elif self._table is not None:
            _keep_numa(t, self._table)
        live = self._live_reservations()
        self._resv_rank = rv.order_ranks(rv.available_by_node(self._index, live, []).values())
        # owner groups from the live reservations only (the registered affinities stay)
        self.resv_index = rv.ReservationIndex(affinities=list(self.resv_index.affinities))
        over: list = []
        rv.reservation_columns(t, self._index, live, self.resv_index, self._node_labels(), over)
        self._note_overflow(over)
        self._resv_cpus_loaded = _has_resv_cpus(t)
        self._table = t
        self._dirty.clear()
        self._reload = False
        self._expired = self._expiry_states(now)
        self._now = now
        return t

    def attach(self, table: NodeTable, now: float):
        """Adopt `table` (already loaded into the engine) as the current image."""
        if table.names != [n.name for n in self.cluster.nodes]:
            raise ValueError("table rows do not match the informer's node set")
        self._table = table
        self._resv_cpus_loaded = _has_resv_cpus(table)
        self._expired = self._expiry_states(now)
        self._now = now

    def _node_labels(self) -> Dict[str, Dict[str, str]]:
        """What reservation affinities see of each node (reservation/transformer.go:335-359)."""
        return {n.name: dict(n.labels or {}) for n in self.cluster.nodes}

    # ---- node events -------------------------------------------------------------
    def on_node_add(self, node: k8s.Node):
        if node.name in self._index:
            return self.on_node_update(None, node)
        self._index[node.name] = len(self.cluster.nodes)
        self.cluster.nodes.append(node)
        self._reload = True

    def on_node_update(self, old: Optional[k8s.Node], node: k8s.Node):
        i = self._index.get(node.name)
        if i is None:
            return self.on_node_add(node)
        self.cluster.nodes[i] = node
        self._dirty.add(node.name)

    def on_node_delete(self, node: k8s.Node):
        i = self._index.pop(node.name, None)
        if i is None:
            return
        del self.cluster.nodes[i]
        self._index = {n.name: j for j, n in enumerate(self.cluster.nodes)}
        self.cluster.node_metrics.pop(node.name, None)
        self._reload = True

    # ---- pod events ----------------------------------------------------------------
    def _node_pods_set(self, pod: k8s.Pod, present: bool):
        """NodeInfo.Pods: assigned, non-terminated pods (upstream scheduler cache)."""
        nn = self._pod_node.pop(pod.uid, None)
        if nn is not None:
            self.cluster.node_pods[nn] = [p for p in self.cluster.node_pods.get(nn, []) if p.uid != pod.uid]
            self._dirty.add(nn)
        if present and pod.node_name and not k8s.is_terminated(pod):
            self.cluster.node_pods.setdefault(pod.node_name, []).append(pod)
            self._pod_node[pod.uid] = pod.node_name
            self._dirty.add(pod.node_name)

    def _touch_metric_refs(self, pod: k8s.Pod):
        for nn in self._metric_refs.get(pod.key, ()):
            self._dirty.add(nn)

    def on_pod_add(self, pod: k8s.Pod, now: float):
        old = self._pods_by_uid.get(pod.uid)
        if old is not None:
            return self.on_pod_update(old, pod, now)
        self._pods_by_uid[pod.uid] = pod
        self.cluster.pods[pod.key] = pod
        self._node_pods_set(pod, True)
        self._numa_pod(pod, True)
        self.assign_cache.on_add(pod, now)
        if pod.node_name:
            self._dirty.add(pod.node_name)
        self._touch_metric_refs(pod)
        self._track_assigned(pod, True)
        self._operating_pod(None, pod)

    def on_pod_update(self, old: Optional[k8s.Pod], pod: k8s.Pod, now: float):
        prev = self._pods_by_uid.get(pod.uid)
        if prev is not None and prev.key != pod.key:
            self.cluster.pods.pop(prev.key, None)
            self._touch_metric_refs(prev)
        self._pods_by_uid[pod.uid] = pod
        self.cluster.pods[pod.key] = pod
        self._node_pods_set(pod, True)
        self._numa_pod(pod, True)
        if prev is not None and prev.node_name and prev.node_name != pod.node_name:
            # the assign cache is keyed by the pod's current node (pod_assign_cache.go:91-101)
            self.assign_cache.unassign(prev.node_name, prev)
            self._dirty.add(prev.node_name)
        self.assign_cache.on_update(old, pod, now)
        if pod.node_name:
            self._dirty.add(pod.node_name)
        self._touch_metric_refs(pod)
        self._track_assigned(pod, True)
        self._operating_pod(prev, pod)

    def on_pod_delete(self, pod: k8s.Pod):
        prev = self._pods_by_uid.pop(pod.uid, pod)
        self.cluster.pods.pop(prev.key, None)
        self._node_pods_set(prev, False)
        self._numa_pod(prev, False)
        self.assign_cache.on_delete(prev)
        if prev.node_name:
            self._dirty.add(prev.node_name)
        self._touch_metric_refs(prev)
        self._track_assigned(prev, False)
        self._operating_pod(prev, None)

    def _track_assigned(self, pod: k8s.Pod, present: bool):
        """The reservation cache's AssignedPods (reservation/pod_eventhandler.go:
        95-131, cache.go:201-232): a bound, non-terminated pod whose
        reservation-allocated annotation names a reservation is one of its
        assigned pods; terminated or deleted, it leaves."""
        old = self._assigned_of.pop(pod.uid, None)
        if old is not None:
            m = self._assigned.get(old, {})
            m.pop(pod.uid, None)
            if not m:
                self._assigned.pop(old, None)
            self._dirty_reservation(old)
        ra = rv.reservation_allocated(pod) if present else None
        if ra is None or not pod.node_name or k8s.is_terminated(pod):
            return
        key = ra[0] or ra[1]
        if not key:
            return
        self._assigned.setdefault(key, {})[pod.uid] = pod
        self._assigned_of[pod.uid] = key
        self._dirty_reservation(key)

    def _dirty_reservation(self, key: str):
        for r in self.reservations.values():
            if key in (r.uid, r.name) and r.node_name:
                self._dirty.add(r.node_name)

    def _devices_on(self) -> bool:
        from .config import PLUGIN_DEVICESHARE
        return PLUGIN_DEVICESHARE in self.profile.filters or PLUGIN_DEVICESHARE in self.profile.scores

    def _operating_pod(self, prev: Optional[k8s.Pod], pod: Optional[k8s.Pod]):
        """A bound pod in the reservation operating mode is also an Available
        reservation on its node (the reservation cache, pod_eventhandler.go:104-124,
        cache.go:139-168): reservation_columns gives it a slot like a
        Reservation's (rv.operating_pod_reservation).  Its ReservationInfo
        outlives updates (cache.go:139-161): the owners parsed when it was first
        added stay, its current owners accumulate as assigned pods; a terminated
        or deleted pod removes it (pod_eventhandler.go:91-93, 136-141).  One the
        engine cannot hold (resources outside the envelope) stays a plain pod,
        counted in `outside_envelope`."""
        gone = pod is None or k8s.is_terminated(pod)
        r = rv.operating_pod_reservation(pod) if not gone else None
        if prev is not None and rv.is_reservation_operating_pod(prev):
            old = rv.operating_reservation_name(prev)
            if r is None or r.name != old:
                if old in self.reservations:
                    self.on_reservation_delete(old)
        if r is None:
            if prev is not None:
                self._op_state.pop(prev.uid, None)
                self.outside_envelope.pop(prev.key, None)
            if pod is not None:
                self._op_state.pop(pod.uid, None)
            return
        st = self._op_state.get(pod.uid)
        if st is None:
            st = (r.owners, r.parse_error, {})
            self._op_state[pod.uid] = st
        owners, perr, seen = st
        cur = rv.current_owner(pod)
        if cur is not None:
            seen.setdefault(cur[2] or f"{cur[0]}/{cur[1]}", cur)   # AddAssignedPod (a repeated UID is skipped)
        r.owners, r.parse_error, r.assigned = owners, perr, len(seen)
        why = rv.reservation_unsupported(r, self._devices_on())
        if why is not None:
            self.outside_envelope[pod.key] = why
            if r.name in self.reservations:
                self.on_reservation_delete(r.name)
            return
        self.outside_envelope.pop(pod.key, None)
        self.on_reservation(r)

    def _note_overflow(self, over: list):
        for r in over:
            if r.pod is not None:
                self.outside_envelope[r.pod.key] = f"more than {abi.RESV_SLOTS_MAX} reservations on node {r.node_name}"

    def _pod_named(self, namespace: str, name: str) -> Optional[k8s.Pod]:
        return self.cluster.pods.get(f"{namespace or 'default'}/{name}") or self.cluster.pods.get(f"{namespace}/{name}")

    def _live_reservations(self) -> List[rv.Reservation]:
        """The reservations as the reservation cache holds them now: a
        Reservation with pods assigned through their reservation-allocated
        annotation takes its assigned count, Allocated (their requests masked to
        its ResourceNames, reservation_info.go:297-306), their cpusets and device
        allocations from those pods; an operating-mode pod's current owners
        supply their cpusets and device allocations (nd.getUsed / the
        NodeAllocation of the owner, when it is a pod of the cluster).  Otherwise
        the Reservation's own fields stand."""
        import dataclasses
        from . import deviceshare as ds
        out = []
        for r in self.reservations.values():
            pods = []
            if r.pod is not None:
                st = self._op_state.get(r.pod.uid)
                for (ns, nmn, _uid) in (st[2].values() if st else ()):
                    q = self._pod_named(ns, nmn)
                    if q is not None and q.node_name == r.node_name:
                        pods.append(q)
                cpus = (nm.pod_allocation(r.pod.annotations or {}) or ([], "", []))[0]
                r = dataclasses.replace(r, cpus=list(cpus))
            else:
                pods = list(self._assigned.get(r.uid, {}).values()) + \
                    ([] if r.uid else list(self._assigned.get(r.name, {}).values()))
                if not pods:
                    out.append(r)
                    continue
                names = set(r.allocatable)
                alloc: k8s.ResourceList = {}
                for q in pods:
                    reqs, _ = k8s.pod_requests_and_limits(q)
                    for n, v in reqs.items():
                        if n in names:
                            alloc[n] = alloc[n] + v if n in alloc else v
                r = dataclasses.replace(r, assigned=len(pods), allocated=alloc)
            acpus, adev = [], []
            for q in pods:
                a = nm.pod_allocation(q.annotations or {})
                if a is not None:
                    acpus.extend(a[0])
                d = ds.parse_device_allocated(q.annotations or {})
                if d:
                    adev.append(d)
            out.append(dataclasses.replace(r, assigned_cpus=sorted(set(acpus)) or list(r.assigned_cpus),
                                           assigned_devices=adev or list(r.assigned_devices)))
        return out

    # ---- NodeMetric events -------------------------------------------------------------
    def on_node_metric(self, nm: k8s.NodeMetric):
        """Add or update."""
        old = self.cluster.node_metrics.get(nm.name)
        if old is not None:
            for pm in old.pods_metric:
                self._metric_refs.get(f"{pm.namespace}/{pm.name}", set()).discard(nm.name)
        self.cluster.node_metrics[nm.name] = nm
        for pm in nm.pods_metric:
            self._metric_refs.setdefault(f"{pm.namespace}/{pm.name}", set()).add(nm.name)
        self._dirty.add(nm.name)

    def on_node_metric_delete(self, name: str):
        old = self.cluster.node_metrics.pop(name, None)
        if old is not None:
            for pm in old.pods_metric:
                self._metric_refs.get(f"{pm.namespace}/{pm.name}", set()).discard(name)
        self._dirty.add(name)

    # ---- NodeResourceTopology events (topology_eventhandler.go:62-113) ------------------------------
    def on_nrt(self, nrt: nm.NodeResourceTopology):
        """Add or update: the node's TopologyOptions are replaced (its NodeAllocation stays)."""
        self.nrts[nrt.name] = nrt
        self._topo[nrt.name] = nm.topology_options(nrt)
        self._dirty.add(nrt.name)

    def on_nrt_delete(self, name: str):
        self.nrts.pop(name, None)
        self._topo.pop(name, None)
        self._dirty.add(name)

    # ---- Device events (deviceshare/device_handler.go: the nodeDevice of the node) -----------------
    def on_device(self, dev):
        """Add or update a Device CR (deviceshare.Device, named after its node).
        More devices of one type than the loaded snapshot's dev_slots: reload."""
        self.cluster.devices[dev.name] = dev
        self._dirty.add(dev.name)
        if self._table is not None and self._table.has_ext:
            per = {}
            for d in dev.devices:
                per[d.type] = per.get(d.type, 0) + 1
            if max(per.values(), default=0) > self._table.dev_slots:
                self._reload = True

    def on_device_delete(self, name: str):
        if self.cluster.devices.pop(name, None) is not None:
            self._dirty.add(name)

    def _numa_pod(self, pod: k8s.Pod, present: bool):
        """podEventHandler.updatePod / deletePod (pod_eventhandler.go:94-144)."""
        if not pod.node_name:
            return
        if not present or k8s.is_terminated(pod):
            self._alloc.setdefault(pod.node_name, nm.NodeAllocation()).release(pod.uid)
            self._dirty.add(pod.node_name)
            return
        a = nm.pod_allocation(pod.annotations or {})
        if a is None:
            return
        opts = self._topo.get(pod.node_name)
        if opts is None or opts.topology is None:     # resourceManager.Update: no valid CPU topology
            return
        self._alloc.setdefault(pod.node_name, nm.NodeAllocation()).update(pod.uid, *a)
        self._dirty.add(pod.node_name)

    def _numa_row(self, table, j: int, node: k8s.Node, frozen: bool):
        prof = self.profile.resolved()
        nm.numa_row(table, j, self._topo.get(node.name), self._alloc.get(node.name), self._classes,
                    node.labels or {}, prof.numa.default_most_allocated, frozen=frozen)

    # ---- Reservation events (reservation/cache.go:117-252) ------------------------------------------
    def _numa_reservation(self, r: rv.Reservation, present: bool):
        """The reserve pod's cpuset in NodeAllocation (ReservationToPodEventHandler ->
        podEventHandler, nodenumaresource/pod_eventhandler.go:40-50,94-144)."""
        uid = r.uid or f"reservation/{r.name}"
        if not r.node_name or r.pod is not None:  # (an operating-mode pod's cpuset is its own: _numa_pod)
            return
        alloc = self._alloc.setdefault(r.node_name, nm.NodeAllocation())
        opts = self._topo.get(r.node_name)
        if present and r.is_available() and r.cpus and opts is not None and opts.topology is not None:
            alloc.update(uid, list(r.cpus), r.cpu_exclusive, [])
        else:
            alloc.release(uid)
        self._dirty.add(r.node_name)

    def _nodeinfo_reserve_pod(self, r: rv.Reservation, present: bool):
        """An Available Reservation's reserve pod is a pod of its node's NodeInfo
        (addReservationToSchedulerCache, frameworkext/eventhandlers/
        reservation_handler.go:250-281; NewReservePod carries its labels and
        annotations) and of the nodeDevice cache (ReservationToPodEventHandler,
        deviceshare/pod_handler.go:43-45).  An operating-mode pod is its own."""
        old = self._resv_pods.pop(r.name, None)
        if old is not None:
            self.cluster.node_pods[old.node_name] = [p for p in self.cluster.node_pods.get(old.node_name, [])
                                                     if p is not old]
            self._dirty.add(old.node_name)
        if present and r.pod is None and r.is_available():
            p = r.reserve_pod()
            self._resv_pods[r.name] = p
            self.cluster.node_pods.setdefault(r.node_name, []).append(p)
            self._dirty.add(r.node_name)

    def on_reservation(self, r: rv.Reservation):
        """Add or update."""
        old = self.reservations.get(r.name)
        if old is not None:
            self._numa_reservation(old, False)
        self.reservations[r.name] = r
        self._numa_reservation(r, True)
        self._nodeinfo_reserve_pod(r, True)
        for nn in ({old.node_name} if old is not None else set()) | {r.node_name}:
            if nn:
                self._dirty.add(nn)
        order = rv.parse_order(r.labels)
        if r.is_available() and order != 0 and order not in self._resv_rank:
            self._reload = True

    def on_reservation_delete(self, name: str):
        old = self.reservations.pop(name, None)
        if old is not None:
            self._numa_reservation(old, False)
            self._nodeinfo_reserve_pod(old, False)
        if old is not None and old.node_name:
            self._dirty.add(old.node_name)

    def register_pods(self, pods) -> bool:
        """Register the pods about to be scheduled: their required reservation
        affinities (ReservationIndex.register_affinities) and upstream static
        filter classes.  True when the loaded snapshot does not cover them:
        rebuild it (table()) before pod_records."""
        from .marshal import pod_static, static_keyed
        pods = list(pods)
        if self.resv_index.register_affinities(pods):
            self._reload = True
        if static_keyed(self.profile):
            for p in pods:
                if self.static_classes.classify(pod_static(p, self.profile)) >= self.static_classes.frozen:
                    self._reload = True
        if self._spread_on():
            for p in pods:
                if not self.cluster.spread.covers(p):
                    self._reload = True
        if self._ipa_on():
            for p in pods:
                if not self.cluster.ipa.covers(p):
                    self._reload = True
        return self._reload

    def _spread_on(self) -> bool:
        from .config import PLUGIN_PTS
        return PLUGIN_PTS in self.profile.filters or PLUGIN_PTS in self.profile.scores

    def _ipa_on(self) -> bool:
        from .config import PLUGIN_IPA
        return PLUGIN_IPA in self.profile.filters or PLUGIN_IPA in self.profile.scores

    def on_namespace(self, name: str, labels: Dict[str, str]):
        """Namespace add / update: the labels affinity terms' namespaceSelectors read."""
        if self.cluster.ipa.ns_labels.get(name) != dict(labels or {}):
            self.cluster.ipa.ns_labels[name] = dict(labels or {})
            if self._ipa_on():
                self._reload = True

    def pod_ext_records(self, pods):
        """koordhip_pod_ext records (DeviceShare, extended scalars, topology
        spread constraints in the loaded snapshot's tables)."""
        from .marshal import pod_ext_records
        return pod_ext_records(pods, self.profile, self.cluster.spread, self.cluster.ipa, self.reservations, self._index)

    def pod_records(self, pods):
        """Pod records with the current owner groups' match masks and static classes."""
        from .marshal import pod_records
        return pod_records(pods, self.profile, self.resv_index, self.static_classes, self.reservations)

    # ---- deltas ----------------------------------------------------------------------------
    def _sync_assigned(self):
        self.cluster.assigned = {nn: list(m.values()) for nn, m in self.assign_cache.items.items()}

    def _expiry_states(self, now: float) -> Dict[str, bool]:
        exp = self.profile.resolved().loadaware.node_metric_expiration_seconds
        return {nn: is_node_metric_expired(nm, exp, now) for nn, nm in self.cluster.node_metrics.items()}

    def pending(self) -> Set[str]:
        return set(self._dirty)

    def delta(self, now: float, apply: bool = True):
        """(row indices, NodeTable of those rows, FlushResult); with `apply` the
        rows also go into the informer's own table image (flush applies them
        only after the engine took them)."""
        res = FlushResult(needs_reload=self._reload)
        if self._reload or self._table is None:
            res.needs_reload = True
            return np.zeros(0, np.int32), None, res
        states = self._expiry_states(now)
        dirty = set(n for n in self._dirty if n in self._index)
        for nn, st in states.items():
            if self._expired.get(nn) != st and nn in self._index and nn not in dirty:
                dirty.add(nn)
                res.expired_flips += 1
        self._expired = states
        self._now = now
        if not dirty:
            self._dirty.clear()
            return np.zeros(0, np.int32), None, res
        self._sync_assigned()
        idx = np.array(sorted(self._index[n] for n in dirty), np.int32)
        rows = self._table.rows(idx)
        over: list = []
        placed = rv.available_by_node(self._index, self._live_reservations(), over)
        self._note_overflow(over)
        if self.nrts or self._classes is not None:
            try:
                for j, i in enumerate(idx):
                    self._numa_row(rows, j, self.cluster.nodes[int(i)], frozen=True)
            except nm.TopologyError:
                res.needs_reload = True              # a CPU topology shape the loaded snapshot has no class for
                return np.zeros(0, np.int32), None, res
        if any(len(placed.get(int(i), [])) > rows.resv_slots for i in idx):
            res.needs_reload = True                  # more reservations on a node than the snapshot's slots
            return np.zeros(0, np.int32), None, res
        labels = self._node_labels()
        for j, i in enumerate(idx):
            node = self.cluster.nodes[int(i)]
            try:
                node_row(rows, j, node, self.cluster, self.profile, now, self.static_classes, node_index=int(i))
            except NewTopologyValue:
                res.needs_reload = True              # a topology value the snapshot has no domain for
                return np.zeros(0, np.int32), None, res
            r = placed.get(int(i))
            if r is None:
                rv.clear_reservation_row(rows, j)
                continue
            try:
                rv.reservation_row(rows, j, r, self.resv_index, self._resv_rank, labels.get(node.name))
            except rv.ReservationError:
                if len(self.resv_index.groups) < abi.RESV_MAX_GROUPS:
                    raise
                res.needs_reload = True              # owner groups full: a reload regroups the live reservations
                return np.zeros(0, np.int32), None, res
        if not self._resv_cpus_loaded and _has_resv_cpus(rows):
            res.needs_reload = True                  # reserved CPUs need the resv_cpus columns at load_snapshot
            return np.zeros(0, np.int32), None, res
        res.rows = len(idx)
        if apply:
            self._adopt(idx, rows)
        return idx, rows, res

    def _adopt(self, idx, rows):
        for c in rows.cols:
            self._table.cols[c][idx] = rows.cols[c]
        self._dirty.clear()

    def flush(self, engine, now: float) -> FlushResult:
        """Push the pending row deltas into `engine` (one koordhip_update_nodes
        call); the informer's image takes them only once the engine has."""
        idx, rows, res = self.delta(now, apply=False)
        if res.needs_reload or rows is None:
            return res
        engine.update_nodes(idx, rows)
        self._adopt(idx, rows)
        return res


def _has_resv_cpus(t: NodeTable) -> bool:
    from .snapshot import RESV_CPU_COLS, slot_col
    return any(t.cols[slot_col(c, q)].any() for q in range(t.resv_slots) for c in RESV_CPU_COLS
               if slot_col(c, q) in t.cols)


def _keep_numa(dst: NodeTable, src: NodeTable):
    """NUMA columns are not derived from objects: carry them over, row by node
    name (rows of nodes new to `dst` keep build_table's no-topology values)."""
    from .snapshot import NUMA_MUTABLE, U64_COLS, ZONE_COLS
    pos = {nm: i for i, nm in enumerate(src.names)}
    pairs = [(j, pos[nm]) for j, nm in enumerate(dst.names) if nm in pos]
    if not pairs:
        return
    dj = np.array([a for a, _ in pairs], np.int64)
    sj = np.array([b for _, b in pairs], np.int64)
    for c in set(U64_COLS) | set(NUMA_MUTABLE) | set(ZONE_COLS) | {"numa_class", "numa_flags", "numa_amp_cpu"}:
        if c in src.cols and c in dst.cols:
            dst.cols[c][dj] = src.cols[c][sj]
    dst.numa_classes = src.numa_classes
