"""Columnar node snapshot (SoA) and pod records, in the exact byte layout of
include/koordhip.h.  Both the HIP engine and the test oracle consume these
arrays, so a snapshot is marshalled once and evaluated by both.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import Dict, List

import numpy as np

from . import abi

I64_COLS = (
    [f"alloc{r}" for r in range(abi.NRES)]
    + [f"requested{r}" for r in range(abi.NRES)]
    + ["nz_cpu_m", "nz_mem", "la_alloc_cpu_m", "la_alloc_mem", "la_used_cpu_m", "la_used_mem",
       "la_used_prod_cpu_m", "la_used_prod_mem",
       "laf_used_m0", "laf_used_m1", "laf_total_m0", "laf_total_m1", "laf_prod_used_m0", "laf_prod_used_m1",
       "laf_thr0", "laf_thr1", "laf_prod_thr0", "laf_prod_thr1",
       "resv_alloc0", "resv_alloc1", "resv_nz0", "resv_nz1", "resv_allocated0", "resv_allocated1"]
)
I32_COLS = ["alloc_pods", "npods", "numa_class", "numa_alloc_cnt", "resv_order_rank", "resv_assigned"]
U8_COLS = ["la_flags", "numa_flags"]
U32_COLS = ["resv_flags",   # KOORDHIP_RESV_* (0 = no reservation on the node)
            "static_allow"]  # static node filters: allowed pod static classes (all ones = every class)
U64_COLS = ([f"numa_free{w}" for w in range(abi.NUMA_WORDS)] + [f"numa_excl_pcpu{w}" for w in range(abi.NUMA_WORDS)]
            + [f"numa_excl_numa{w}" for w in range(abi.NUMA_WORDS)])
# per reservation slot: the reserved CPUs not held by its assigned pods
# (NodeNUMAResource RestoreReservation, nodenumaresource/reservation.go:76-113)
RESV_CPU_COLS = [f"resv_cpus{w}" for w in range(abi.NUMA_WORDS)]
# NUMA zone resources, [n][2][NUMA_MAX_NODES] int64 per column (cpu milli, memory bytes)
ZONE_COLS = ["numa_zone_alloc", "numa_zone_used"]
F64_COLS = ["numa_amp_cpu"]   # CPU amplification ratio (1.0 = none)
ALL_COLS = I64_COLS + I32_COLS + U8_COLS + U64_COLS + ZONE_COLS + F64_COLS + U32_COLS + RESV_CPU_COLS
# NodeNUMAResource mutable columns (advanced by cpuset / NUMA-zone Reserves)
NUMA_MUTABLE = [c for c in U64_COLS] + ["numa_alloc_cnt", "numa_zone_used"]
# Reservation columns (the node's Available reservation) and the mutable ones
RESV_COLS = ["resv_flags", "resv_order_rank", "resv_alloc0", "resv_alloc1", "resv_nz0", "resv_nz1",
             "resv_allocated0", "resv_allocated1", "resv_assigned"] + RESV_CPU_COLS
RESV_MUTABLE = ["resv_allocated0", "resv_allocated1", "resv_assigned"] + RESV_CPU_COLS
# ABI 9 (the sequential cycle): DeviceShare devices, NodeResourcesFit extended
# scalars, upstream static Scores.  Present only after NodeTable.enable_ext();
# every one is row-major per node here (as_soa transposes to the ABI's layouts).
EXT_COLS = ["dev_present", "dev_minor", "dev_total", "dev_used", "xalloc", "xrequested", "static_score"]
EXT_MUTABLE = ["dev_used", "xrequested"]
# PodTopologySpread (sequential cycle): per node its domain per topology key
# [n][PTS_KEYS] i32 (-1: no label), matching pods per constraint [n][PTS_CONS]
# i32 (mutable), spread-class eligibility bits u16.  Present after enable_pts().
PTS_COLS = ["pts_dom", "pts_cnt", "pts_elig"]
PTS_MUTABLE = ["pts_cnt"]
# InterPodAffinity: per node the pods each count entry counts [n][IPA_ENTRIES]
# i32 (mutable; the topology keys are the pts_* ones).  Present after enable_ipa().
IPA_COLS = ["ipa_cnt"]
IPA_MUTABLE = ["ipa_cnt"]
# DeviceShare with a reservation holding devices (ABI 13): per node the slot of
# its one such reservation [n] i32 (-1: none) and that reservation's device
# allocatable / allocated [n][2][TYPES][dev_slots][RES] i64 (the allocated half
# mutable).  Present after enable_resv_dev().
RESV_DEV_COLS = ["resv_dev_slot", "resv_dev", "resv_xalloc", "resv_xallocated"]
RESV_DEV_MUTABLE = ["resv_dev", "resv_xallocated"]
# (ABI 14: that reservation's NodeResourcesFit extended scalars [n][NXRES] i64,
# its Allocatable -- the reserve pod's scalar requests -- and Allocated, the
# latter mutable)


@dataclass
class PtsMeta:
    """koordhip_node_soa's PodTopologySpread scalars: the keys (bit k of hostname:
    kubernetes.io/hostname), domains per key, the constraint table's keys, the
    spread classes."""
    keys: int = 0
    hostname: int = 0
    ndom: List[int] = field(default_factory=lambda: [0] * abi.PTS_KEYS)
    cons_key: List[int] = field(default_factory=list)
    classes: int = 0


@dataclass
class IpaMeta:
    """koordhip_node_soa's InterPodAffinity scalars: the count entries' topology keys."""
    ent_key: List[int] = field(default_factory=list)


def slot_col(col: str, s: int) -> str:
    """Column name of reservation slot s (slot 0 is the plain column)."""
    return col if s == 0 else f"{col}@{s}"


def _shape(col: str, n: int):
    return (n, 2, abi.NUMA_MAX_NODES) if col in ZONE_COLS else (n,)


def _dtype(col: str):
    if col in I32_COLS:
        return np.int32
    if col in U8_COLS:
        return np.uint8
    if col in U64_COLS or col in RESV_CPU_COLS:
        return np.uint64
    if col in U32_COLS:
        return np.uint32
    if col in F64_COLS:
        return np.float64
    return np.int64


@dataclass
class NodeTable:
    """n rows of the koordhip_node_soa columns (numpy, C-contiguous)."""
    n: int
    cols: Dict[str, np.ndarray] = field(default_factory=dict)
    names: List[str] = field(default_factory=list)
    # NodeNUMAResource topology classes (abi.NUMA_CLASS_DTYPE), indexed by numa_class
    numa_classes: np.ndarray = field(default_factory=lambda: np.zeros(0, abi.NUMA_CLASS_DTYPE))
    # reservation slots per node: slot 0 in the RESV_COLS columns, slot s >= 1
    # in the columns slot_col(c, s) (koordhip_node_soa.resv_slots)
    resv_slots: int = 1
    # DeviceShare minors per type per node held by the dev_* columns (0: none)
    dev_slots: int = 0
    # PodTopologySpread tables (None: no pts_* columns)
    pts: "PtsMeta" = None
    # InterPodAffinity count entries (None: no ipa_* columns; needs the pts_* keys)
    ipa: "IpaMeta" = None

    @property
    def has_ipa(self) -> bool:
        return self.ipa is not None

    def enable_ipa(self, meta: "IpaMeta"):
        """Add the InterPodAffinity count column (every node: no pods counted)."""
        if not self.has_pts:
            raise ValueError("InterPodAffinity entries need the topology keys (enable_pts first)")
        if not (0 < len(meta.ent_key) <= abi.IPA_ENTRIES and all(0 <= k < self.pts.keys for k in meta.ent_key)):
            raise ValueError("InterPodAffinity entries outside the engine's envelope")
        self.ipa = meta
        self.cols["ipa_cnt"] = np.zeros((self.n, abi.IPA_ENTRIES), np.int32)
        return self

    @property
    def has_pts(self) -> bool:
        return self.pts is not None

    def enable_pts(self, meta: "PtsMeta"):
        """Add the PodTopologySpread columns (every node: no label, no pods, no class)."""
        if not (0 < meta.keys <= abi.PTS_KEYS and len(meta.cons_key) <= abi.PTS_CONS
                and meta.classes <= abi.PTS_CLASSES):
            raise ValueError("PodTopologySpread tables outside the engine's envelope")
        for k in range(meta.keys):
            if not (meta.hostname >> k) & 1 and not 0 < meta.ndom[k] <= abi.PTS_DOMAINS:
                raise ValueError(f"topology key {k}: 1..{abi.PTS_DOMAINS} domains")
        self.pts = meta
        self.cols["pts_dom"] = np.full((self.n, abi.PTS_KEYS), -1, np.int32)
        self.cols["pts_cnt"] = np.zeros((self.n, abi.PTS_CONS), np.int32)
        self.cols["pts_elig"] = np.zeros(self.n, np.uint16)
        return self

    @property
    def has_ext(self) -> bool:
        return "xalloc" in self.cols

    def enable_ext(self, dev_slots: int = 0):
        """Add the ABI 9 columns (empty): dev_present [n] u8, dev_minor
        [n][TYPES][dev_slots] i32 (-1 empty), dev_total / dev_used
        [n][TYPES][dev_slots][RES] i64, xalloc / xrequested [n][NXRES] i64,
        static_score [n][2][MAX_STATIC_CLASSES] u16."""
        if not 0 <= dev_slots <= abi.DEV_SLOTS:
            raise ValueError(f"dev_slots must be in [0, {abi.DEV_SLOTS}]")
        n = self.n
        S = max(dev_slots, 1)
        self.dev_slots = dev_slots
        self.cols["dev_present"] = np.zeros(n, np.uint8)
        self.cols["dev_minor"] = np.full((n, abi.DEV_TYPES, S), -1, np.int32)
        self.cols["dev_total"] = np.zeros((n, abi.DEV_TYPES, S, abi.DEV_RES), np.int64)
        self.cols["dev_used"] = np.zeros((n, abi.DEV_TYPES, S, abi.DEV_RES), np.int64)
        self.cols["xalloc"] = np.zeros((n, abi.NXRES), np.int64)
        self.cols["xrequested"] = np.zeros((n, abi.NXRES), np.int64)
        self.cols["static_score"] = np.zeros((n, 2, abi.MAX_STATIC_CLASSES), np.uint16)
        return self

    @property
    def has_resv_dev(self) -> bool:
        return "resv_dev_slot" in self.cols

    def enable_resv_dev(self):
        """Add the device-holding reservation columns (no node has one);
        needs the device columns (enable_ext with dev_slots > 0)."""
        if not self.has_ext or self.dev_slots <= 0:
            raise ValueError("device-holding reservations need the device columns (enable_ext(dev_slots > 0))")
        self.cols["resv_dev_slot"] = np.full(self.n, -1, np.int32)
        self.cols["resv_dev"] = np.zeros((self.n, 2, abi.DEV_TYPES, self.dev_slots, abi.DEV_RES), np.int64)
        self.cols["resv_xalloc"] = np.zeros((self.n, abi.NXRES), np.int64)
        self.cols["resv_xallocated"] = np.zeros((self.n, abi.NXRES), np.int64)
        return self

    def set_resv_slots(self, slots: int):
        """Hold up to `slots` reservations per node (new slots empty)."""
        if not 1 <= slots <= abi.RESV_SLOTS_MAX:
            raise ValueError(f"resv_slots must be in [1, {abi.RESV_SLOTS_MAX}]")
        for s in range(1, abi.RESV_SLOTS_MAX):
            for c in RESV_COLS:
                name = slot_col(c, s)
                if s < slots and name not in self.cols:
                    self.cols[name] = np.zeros(self.n, dtype=_dtype(c))
                elif s >= slots:
                    self.cols.pop(name, None)
        self.resv_slots = slots

    def col_names(self) -> List[str]:
        return (ALL_COLS + [slot_col(c, s) for s in range(1, self.resv_slots) for c in RESV_COLS]
                + (EXT_COLS if self.has_ext else []) + (PTS_COLS if self.has_pts else [])
                + (IPA_COLS if self.has_ipa else []) + (RESV_DEV_COLS if self.has_resv_dev else []))

    @classmethod
    def empty(cls, n: int) -> "NodeTable":
        t = cls(n=n)
        for c in ALL_COLS:
            t.cols[c] = np.zeros(_shape(c, n), dtype=_dtype(c))
        t.cols["numa_class"][:] = -1
        t.cols["numa_amp_cpu"][:] = 1.0
        t.cols["static_allow"][:] = 0xFFFFFFFF
        t.names = [f"node-{i}" for i in range(n)]
        return t

    def __getitem__(self, c: str) -> np.ndarray:
        return self.cols[c]

    def rows(self, idx) -> "NodeTable":
        idx = np.asarray(idx, dtype=np.int64)
        t = NodeTable(n=len(idx))
        for c in self.col_names():
            t.cols[c] = np.ascontiguousarray(self.cols[c][idx])
        t.names = [self.names[i] for i in idx] if self.names else []
        t.numa_classes = self.numa_classes
        t.resv_slots = self.resv_slots
        t.dev_slots = self.dev_slots
        t.pts = self.pts
        t.ipa = self.ipa
        return t

    def copy(self) -> "NodeTable":
        t = NodeTable(n=self.n)
        t.cols = {k: v.copy() for k, v in self.cols.items()}
        t.names = list(self.names)
        t.numa_classes = self.numa_classes.copy()
        t.resv_slots = self.resv_slots
        t.dev_slots = self.dev_slots
        t.pts = self.pts
        t.ipa = self.ipa
        return t

    def as_soa(self) -> abi.KoordhipNodeSoa:
        """Build a koordhip_node_soa pointing at this table's arrays (keep `self` alive)."""
        for c in ALL_COLS:
            a = self.cols[c]
            if not a.flags.c_contiguous or a.dtype != _dtype(c) or a.shape != _shape(c, self.n):
                self.cols[c] = np.ascontiguousarray(a, dtype=_dtype(c)).reshape(_shape(c, self.n))
        s = abi.KoordhipNodeSoa()
        p64 = lambda c: self.cols[c].ctypes.data_as(C.POINTER(C.c_int64))
        p32 = lambda c: self.cols[c].ctypes.data_as(C.POINTER(C.c_int32))
        for r in range(abi.NRES):
            s.alloc[r] = p64(f"alloc{r}")
            s.requested[r] = p64(f"requested{r}")
        s.alloc_pods = p32("alloc_pods")
        s.npods = p32("npods")
        for c in ["nz_cpu_m", "nz_mem", "la_alloc_cpu_m", "la_alloc_mem", "la_used_cpu_m", "la_used_mem",
                  "la_used_prod_cpu_m", "la_used_prod_mem"]:
            setattr(s, c, p64(c))
        for k in range(2):
            s.laf_used_m[k] = p64(f"laf_used_m{k}")
            s.laf_total_m[k] = p64(f"laf_total_m{k}")
            s.laf_prod_used_m[k] = p64(f"laf_prod_used_m{k}")
            s.laf_thr[k] = p64(f"laf_thr{k}")
            s.laf_prod_thr[k] = p64(f"laf_prod_thr{k}")
        s.la_flags = self.cols["la_flags"].ctypes.data_as(C.POINTER(C.c_uint8))
        self.numa_classes = np.ascontiguousarray(self.numa_classes, dtype=abi.NUMA_CLASS_DTYPE)
        s.numa_classes = self.numa_classes.ctypes.data if len(self.numa_classes) else None
        s.n_numa_classes = len(self.numa_classes)
        s.numa_class = p32("numa_class")
        p64u = lambda c: self.cols[c].ctypes.data_as(C.POINTER(C.c_uint64))
        for w in range(abi.NUMA_WORDS):
            s.numa_free[w] = p64u(f"numa_free{w}")
            s.numa_excl_pcpu[w] = p64u(f"numa_excl_pcpu{w}")
            s.numa_excl_numa[w] = p64u(f"numa_excl_numa{w}")
        s.numa_alloc_cnt = p32("numa_alloc_cnt")
        s.numa_flags = self.cols["numa_flags"].ctypes.data_as(C.POINTER(C.c_uint8))
        s.numa_zone_alloc = p64("numa_zone_alloc")
        s.numa_zone_used = p64("numa_zone_used")
        s.numa_amp_cpu = self.cols["numa_amp_cpu"].ctypes.data_as(C.POINTER(C.c_double))
        if self.resv_slots > 1:
            # slot-major [S][n] copies of the reservation columns, kept alive by
            # the returned struct (each call makes its own: a caller holding an
            # earlier struct keeps valid pointers)
            rc = {c: np.ascontiguousarray(np.concatenate(
                [self.cols[slot_col(c, q)] for q in range(self.resv_slots)]), dtype=_dtype(c)) for c in RESV_COLS}
        else:
            rc = self.cols
        s.resv_flags = rc["resv_flags"].ctypes.data_as(C.POINTER(C.c_uint32))
        s.resv_order_rank = rc["resv_order_rank"].ctypes.data_as(C.POINTER(C.c_int32))
        for k in range(2):
            s.resv_alloc[k] = rc[f"resv_alloc{k}"].ctypes.data_as(C.POINTER(C.c_int64))
            s.resv_nz[k] = rc[f"resv_nz{k}"].ctypes.data_as(C.POINTER(C.c_int64))
            s.resv_allocated[k] = rc[f"resv_allocated{k}"].ctypes.data_as(C.POINTER(C.c_int64))
        s.resv_assigned = rc["resv_assigned"].ctypes.data_as(C.POINTER(C.c_int32))
        s.resv_slots = self.resv_slots if self.resv_slots > 1 else 0
        if any(rc[c].any() for c in RESV_CPU_COLS):   # NULL: no reservation holds CPUs
            for w in range(abi.NUMA_WORDS):
                s.resv_cpus[w] = rc[f"resv_cpus{w}"].ctypes.data_as(C.POINTER(C.c_uint64))
        s._keep = rc
        s.static_allow = self.cols["static_allow"].ctypes.data_as(C.POINTER(C.c_uint32))
        if self.has_ext:
            keep = {}
            if self.dev_slots > 0:
                for c in ("dev_present", "dev_minor", "dev_total", "dev_used"):
                    keep[c] = np.ascontiguousarray(self.cols[c])
                s.dev_slots = self.dev_slots
                s.dev_present = keep["dev_present"].ctypes.data_as(C.POINTER(C.c_uint8))
                s.dev_minor = keep["dev_minor"].ctypes.data_as(C.POINTER(C.c_int32))
                s.dev_total = keep["dev_total"].ctypes.data_as(C.POINTER(C.c_int64))
                s.dev_used = keep["dev_used"].ctypes.data_as(C.POINTER(C.c_int64))
            keep["xalloc"] = np.ascontiguousarray(self.cols["xalloc"].T)        # [NXRES][n]
            keep["xrequested"] = np.ascontiguousarray(self.cols["xrequested"].T)
            s.xalloc = keep["xalloc"].ctypes.data_as(C.POINTER(C.c_int64))
            s.xrequested = keep["xrequested"].ctypes.data_as(C.POINTER(C.c_int64))
            ss = self.cols["static_score"]
            for w in range(2):
                if ss[:, w].any():
                    keep[f"ss{w}"] = np.ascontiguousarray(ss[:, w].T)      # [MAX_STATIC_CLASSES][n]
                    s.static_score[w] = keep[f"ss{w}"].ctypes.data_as(C.POINTER(C.c_uint16))
            if self.has_resv_dev and (self.cols["resv_dev_slot"] >= 0).any():
                keep["resv_dev_slot"] = np.ascontiguousarray(self.cols["resv_dev_slot"], dtype=np.int32)
                keep["resv_dev"] = np.ascontiguousarray(self.cols["resv_dev"], dtype=np.int64)
                s.resv_dev_slot = keep["resv_dev_slot"].ctypes.data_as(C.POINTER(C.c_int32))
                s.resv_dev = keep["resv_dev"].ctypes.data_as(C.POINTER(C.c_int64))
                if self.cols["resv_xalloc"].any():      # NULL: no reservation holds extended scalars
                    keep["resv_xalloc"] = np.ascontiguousarray(self.cols["resv_xalloc"].T)          # [NXRES][n]
                    keep["resv_xallocated"] = np.ascontiguousarray(self.cols["resv_xallocated"].T)
                    s.resv_xalloc = keep["resv_xalloc"].ctypes.data_as(C.POINTER(C.c_int64))
                    s.resv_xallocated = keep["resv_xallocated"].ctypes.data_as(C.POINTER(C.c_int64))
            s._keep_ext = keep
        if self.has_pts:
            m = self.pts
            kp = {"dom": np.ascontiguousarray(self.cols["pts_dom"][:, :m.keys].T),          # [keys][n]
                  "cnt": np.ascontiguousarray(self.cols["pts_cnt"][:, :max(1, len(m.cons_key))].T),  # [cons][n]
                  "elig": np.ascontiguousarray(self.cols["pts_elig"])}
            s.pts_keys = m.keys
            s.pts_hostname = m.hostname
            for k in range(abi.PTS_KEYS):
                s.pts_ndom[k] = m.ndom[k] if k < m.keys else 0
            s.pts_cons = len(m.cons_key)
            s.pts_classes = m.classes
            for c in range(abi.PTS_CONS):
                s.pts_cons_key[c] = m.cons_key[c] if c < len(m.cons_key) else 0
            s.pts_dom = kp["dom"].ctypes.data_as(C.POINTER(C.c_int32))
            s.pts_cnt = kp["cnt"].ctypes.data_as(C.POINTER(C.c_int32))
            s.pts_elig = kp["elig"].ctypes.data_as(C.POINTER(C.c_uint16))
            s._keep_pts = kp
        if self.has_ipa:
            ne = len(self.ipa.ent_key)
            ki = np.ascontiguousarray(self.cols["ipa_cnt"][:, :ne].T)             # [ents][n]
            s.ipa_ents = ne
            for e in range(abi.IPA_ENTRIES):
                s.ipa_ent_key[e] = self.ipa.ent_key[e] if e < ne else 0
            s.ipa_cnt = ki.ctypes.data_as(C.POINTER(C.c_int32))
            s._keep_ipa = ki
        return s

    def nbytes(self) -> int:
        return sum(v.nbytes for v in self.cols.values())


def concat(tables: List[NodeTable]) -> NodeTable:
    t = NodeTable(n=sum(x.n for x in tables))
    slots = max(x.resv_slots for x in tables)
    for x in tables:
        if x.resv_slots < slots:
            x.set_resv_slots(slots)
    t.resv_slots = slots
    for c in tables[0].col_names():
        t.cols[c] = np.concatenate([x.cols[c] for x in tables])
    t.names = [nm for x in tables for nm in x.names]
    t.dev_slots = max(x.dev_slots for x in tables)
    # merge topology class tables, re-indexing each part's numa_class
    classes, off = [], 0
    pos = 0
    for x in tables:
        cls = t.cols["numa_class"][pos:pos + x.n]
        cls[cls >= 0] += off
        classes.append(x.numa_classes)
        off += len(x.numa_classes)
        pos += x.n
    t.numa_classes = (np.concatenate(classes) if classes else np.zeros(0, abi.NUMA_CLASS_DTYPE)).astype(
        abi.NUMA_CLASS_DTYPE)
    return t


def pod_array(n: int) -> np.ndarray:
    return np.zeros(n, dtype=abi.POD_DTYPE)
