"""PlacementEngine: the Python face of libkoordhip.so (what the Go shim binds
through cgo).  Thin: every call goes straight to the C-ABI,
there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import numpy as np

from . import abi
from .config import Profile, to_c_config
from .snapshot import NodeTable


class PlacementEngine:
    def __init__(self, profile: Profile, device: int = -1, profile_kernels: bool = False):
        self.lib = abi.load_library()
        self.cfg = to_c_config(profile, device)
        self.cfg.profile_kernels = 1 if profile_kernels else 0
        self._ctx = C.c_void_p()
        abi.check(self.lib, self.lib.koordhip_create(C.byref(self.cfg), C.byref(self._ctx)))
        self.n = 0
        self._table: Optional[NodeTable] = None

    def close(self):
        if self._ctx:
            self.lib.koordhip_destroy(self._ctx)
            self._ctx = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # ---- snapshot -----------------------------------------------------------
    def load_snapshot(self, table: NodeTable):
        soa = table.as_soa()
        abi.check(self.lib, self.lib.koordhip_load_snapshot(self._ctx, C.byref(soa), table.n))
        self.n = table.n
        self._table = table

    def update_nodes(self, idx, rows: NodeTable):
        idx = np.ascontiguousarray(idx, dtype=np.int32)
        soa = rows.as_soa()
        abi.check(self.lib, self.lib.koordhip_update_nodes(self._ctx, abi.ptr(idx, C.c_int32), C.byref(soa), len(idx)))

    def read_nodes(self) -> dict:
        n = self.n
        req = np.zeros((abi.NRES, n), np.int64)
        nz = np.zeros((2, n), np.int64)
        npods = np.zeros(n, np.int32)
        la = np.zeros((2, n), np.int64)
        lap = np.zeros((2, n), np.int64)
        abi.check(self.lib, self.lib.koordhip_read_nodes(self._ctx, abi.ptr(req, C.c_int64), abi.ptr(nz, C.c_int64),
                                                         abi.ptr(npods, C.c_int32), abi.ptr(la, C.c_int64),
                                                         abi.ptr(lap, C.c_int64)))
        return {"requested": req, "nz": nz, "npods": npods, "la_used": la, "la_used_prod": lap}

    # ---- evaluation ---------------------------------------------------------
    def eval(self, pods: np.ndarray, status: bool = True, scores: bool = True, k: int = 0) -> dict:
        pods = np.ascontiguousarray(pods, dtype=abi.POD_DTYPE)
        p, n = len(pods), self.n
        st = np.zeros((p, n), np.uint8) if status else None
        sc = np.zeros((p, abi.NPLUGINS, n), np.int32) if scores else None
        tk = np.zeros((p, k), abi.TOPK_DTYPE) if k else None
        abi.check(self.lib, self.lib.koordhip_eval(
            self._ctx, pods.ctypes.data, p, abi.ptr(st, C.c_uint8), abi.ptr(sc, C.c_int32),
            tk.ctypes.data if tk is not None else None, k))
        return {"status": st, "scores": sc, "topk": tk}

    def place_stream(self, pods: np.ndarray) -> np.ndarray:
        pods = np.ascontiguousarray(pods, dtype=abi.POD_DTYPE)
        out = np.zeros(len(pods), np.int32)
        abi.check(self.lib, self.lib.koordhip_place_stream(self._ctx, pods.ctypes.data, len(pods),
                                                           abi.ptr(out, C.c_int32)))
        return out

    def place_stream_ext(self, pods: np.ndarray, ext: Optional[np.ndarray] = None) -> np.ndarray:
        """The greedy stream with koordhip_pod_ext records (DeviceShare requests,
        extended scalars); profiles with a normalized Score run the exact
        sequential cycle."""
        pods = np.ascontiguousarray(pods, dtype=abi.POD_DTYPE)
        x = None if ext is None else np.ascontiguousarray(ext, dtype=abi.POD_EXT_DTYPE)
        out = np.zeros(len(pods), np.int32)
        abi.check(self.lib, self.lib.koordhip_place_stream_ext(self._ctx, pods.ctypes.data,
                                                               x.ctypes.data if x is not None else None, len(pods),
                                                               abi.ptr(out, C.c_int32)))
        return out

    def eval_ext(self, pods: np.ndarray, ext: Optional[np.ndarray] = None, status: bool = True, scores: bool = True,
                 k: int = 0) -> dict:
        pods = np.ascontiguousarray(pods, dtype=abi.POD_DTYPE)
        x = None if ext is None else np.ascontiguousarray(ext, dtype=abi.POD_EXT_DTYPE)
        p, n = len(pods), self.n
        st = np.zeros((p, n), np.uint16) if status else None
        sc = np.zeros((p, abi.NPLUGINS + abi.NEXT_PLUGINS, n), np.int32) if scores else None
        tk = np.zeros((p, k), abi.TOPK_DTYPE) if k else None
        abi.check(self.lib, self.lib.koordhip_eval_ext(
            self._ctx, pods.ctypes.data, x.ctypes.data if x is not None else None, p, abi.ptr(st, C.c_uint16),
            abi.ptr(sc, C.c_int32), tk.ctypes.data if tk is not None else None, k))
        return {"status": st, "scores": sc, "topk": tk}

    def fetch_devices(self, n: int) -> np.ndarray:
        """[n][DEV_TYPES] device-slot masks the last place call allocated."""
        out = np.zeros((n, abi.DEV_TYPES), np.uint32)
        abi.check(self.lib, self.lib.koordhip_fetch_devices(self._ctx, abi.ptr(out, C.c_uint32), n))
        return out

    def read_devices(self) -> dict:
        S = max(1, self._table.dev_slots if self._table is not None else 0)
        used = np.zeros((self.n, abi.DEV_TYPES, S, abi.DEV_RES), np.int64)
        xr = np.zeros((abi.NXRES, self.n), np.int64)
        abi.check(self.lib, self.lib.koordhip_read_devices(self._ctx, abi.ptr(used, C.c_int64), abi.ptr(xr, C.c_int64)))
        return {"dev_used": used, "xrequested": xr.T.copy()}

    def read_resv_devices(self) -> np.ndarray:
        """The device-holding reservations' column [n][2][TYPES][dev_slots][RES]
        (allocatable, allocated; the allocated half advanced by Reserve)."""
        S = max(1, self._table.dev_slots if self._table is not None else 0)
        out = np.zeros((self.n, 2, abi.DEV_TYPES, S, abi.DEV_RES), np.int64)
        abi.check(self.lib, self.lib.koordhip_read_resv_devices(self._ctx, abi.ptr(out, C.c_int64)))
        return out

    def read_resv_scalars(self) -> np.ndarray:
        """The device-holding reservations' extended-scalar Allocated [n][NXRES]
        (advanced by Reserve; zeros without the resv_xalloc column)."""
        out = np.zeros((abi.NXRES, self.n), np.int64)
        abi.check(self.lib, self.lib.koordhip_read_resv_scalars(self._ctx, abi.ptr(out, C.c_int64)))
        return out.T.copy()

    def read_pts(self) -> np.ndarray:
        """PodTopologySpread matching pods per node and table constraint [n][cons]."""
        m = self._table.pts if self._table is not None else None
        C_ = len(m.cons_key) if m is not None else 0
        out = np.zeros((C_, self.n), np.int32)
        if C_:
            abi.check(self.lib, self.lib.koordhip_read_pts(self._ctx, abi.ptr(out, C.c_int32)))
        return out.T.copy()

    def read_ipa(self) -> np.ndarray:
        """InterPodAffinity count entries' pods per node [n][ents]."""
        m = self._table.ipa if self._table is not None else None
        E = len(m.ent_key) if m is not None else 0
        out = np.zeros((E, self.n), np.int32)
        if E:
            abi.check(self.lib, self.lib.koordhip_read_ipa(self._ctx, abi.ptr(out, C.c_int32)))
        return out.T.copy()

    def stage_pods(self, pods: np.ndarray):
        pods = np.ascontiguousarray(pods, dtype=abi.POD_DTYPE)
        self._staged = pods
        abi.check(self.lib, self.lib.koordhip_stage_pods(self._ctx, pods.ctypes.data, len(pods)))

    def stage_pods_ext(self, pods: np.ndarray, ext: Optional[np.ndarray] = None):
        """Stage pods with their koordhip_pod_ext records (the sequential cycle's place_staged)."""
        pods = np.ascontiguousarray(pods, dtype=abi.POD_DTYPE)
        x = None if ext is None else np.ascontiguousarray(ext, dtype=abi.POD_EXT_DTYPE)
        self._staged = pods
        abi.check(self.lib, self.lib.koordhip_stage_pods_ext(self._ctx, pods.ctypes.data,
                                                             x.ctypes.data if x is not None else None, len(pods)))

    def place_staged(self):
        abi.check(self.lib, self.lib.koordhip_place_staged(self._ctx))

    def synchronize(self):
        abi.check(self.lib, self.lib.koordhip_synchronize(self._ctx))

    def fetch_placements(self, n: int) -> np.ndarray:
        out = np.zeros(n, np.int32)
        abi.check(self.lib, self.lib.koordhip_fetch_placements(self._ctx, abi.ptr(out, C.c_int32), n))
        return out

    def checkpoint(self):
        abi.check(self.lib, self.lib.koordhip_checkpoint(self._ctx))

    def restore(self):
        abi.check(self.lib, self.lib.koordhip_restore(self._ctx))

    def commit(self, pod, node: int) -> np.ndarray:
        """Reserve; returns the allocated cpuset mask (zeros for a non-cpuset pod).
        Raises KoordhipError(code=abi.E_RESERVE) when the NUMA Allocate fails."""
        pod = np.ascontiguousarray(np.atleast_1d(pod), dtype=abi.POD_DTYPE)
        cpus = np.zeros(abi.NUMA_WORDS, np.uint64)
        abi.check(self.lib, self.lib.koordhip_commit(self._ctx, pod.ctypes.data, int(node),
                                                     abi.ptr(cpus, C.c_uint64)))
        return cpus

    def uncommit(self, pod, node: int, cpus=None):
        pod = np.ascontiguousarray(np.atleast_1d(pod), dtype=abi.POD_DTYPE)
        c = None if cpus is None else np.ascontiguousarray(cpus, dtype=np.uint64)
        abi.check(self.lib, self.lib.koordhip_uncommit(self._ctx, pod.ctypes.data, int(node),
                                                       abi.ptr(c, C.c_uint64)))

    def commit_ext(self, pod, ext, node: int):
        """Reserve of one pod with its koordhip_pod_ext record (DeviceShare, the
        extended scalars, PodTopologySpread / InterPodAffinity counts besides
        koordhip_commit's plugins): returns (cpus [NUMA_WORDS], device slots [DEV_TYPES])."""
        pod = np.ascontiguousarray(np.atleast_1d(pod), dtype=abi.POD_DTYPE)
        x = np.ascontiguousarray(np.atleast_1d(ext), dtype=abi.POD_EXT_DTYPE)
        cpus = np.zeros(abi.NUMA_WORDS, np.uint64)
        dev = np.zeros(abi.DEV_TYPES, np.uint32)
        abi.check(self.lib, self.lib.koordhip_commit_ext(self._ctx, pod.ctypes.data, x.ctypes.data, int(node),
                                                         abi.ptr(cpus, C.c_uint64), abi.ptr(dev, C.c_uint32)))
        return cpus, dev

    def uncommit_ext(self, pod, ext, node: int, cpus=None, dev=None):
        pod = np.ascontiguousarray(np.atleast_1d(pod), dtype=abi.POD_DTYPE)
        x = np.ascontiguousarray(np.atleast_1d(ext), dtype=abi.POD_EXT_DTYPE)
        c = None if cpus is None else np.ascontiguousarray(cpus, dtype=np.uint64)
        d = None if dev is None else np.ascontiguousarray(dev, dtype=np.uint32)
        abi.check(self.lib, self.lib.koordhip_uncommit_ext(self._ctx, pod.ctypes.data, x.ctypes.data, int(node),
                                                           abi.ptr(c, C.c_uint64), abi.ptr(d, C.c_uint32)))

    def read_numa(self) -> dict:
        n = self.n
        fr = np.zeros((abi.NUMA_WORDS, n), np.uint64)
        ep = np.zeros((abi.NUMA_WORDS, n), np.uint64)
        en = np.zeros((abi.NUMA_WORDS, n), np.uint64)
        cnt = np.zeros(n, np.int32)
        abi.check(self.lib, self.lib.koordhip_read_numa(self._ctx, abi.ptr(fr, C.c_uint64), abi.ptr(ep, C.c_uint64),
                                                        abi.ptr(en, C.c_uint64), abi.ptr(cnt, C.c_int32)))
        zu = np.zeros((n, 2, abi.NUMA_MAX_NODES), np.int64)
        abi.check(self.lib, self.lib.koordhip_read_numa_zones(self._ctx, abi.ptr(zu, C.c_int64)))
        return {"free": fr, "excl_pcpu": ep, "excl_numa": en, "alloc_cnt": cnt, "zone_used": zu}

    def read_reservations(self) -> dict:
        """Reservation mutable state: Allocated [2][S n] (cpu milli, memory), len(AssignedPods) [S n],
        S = the loaded table's reservation slots, slot-major."""
        n = self.n * max(1, self._table.resv_slots)
        al = np.zeros((2, n), np.int64)
        asg = np.zeros(n, np.int32)
        abi.check(self.lib, self.lib.koordhip_read_reservations(self._ctx, abi.ptr(al, C.c_int64), abi.ptr(asg, C.c_int32)))
        rc = np.zeros((abi.NUMA_WORDS, n), np.uint64)
        abi.check(self.lib, self.lib.koordhip_read_resv_cpus(self._ctx, abi.ptr(rc, C.c_uint64)))
        return {"allocated": al, "assigned": asg, "cpus": rc}

    def fetch_cpusets(self, n: int) -> np.ndarray:
        out = np.zeros((n, abi.NUMA_WORDS), np.uint64)
        abi.check(self.lib, self.lib.koordhip_fetch_cpusets(self._ctx, abi.ptr(out, C.c_uint64), n))
        return out

    def last_stats(self) -> dict:
        em, tm = C.c_double(), C.c_double()
        nl, ne = C.c_int64(), C.c_int64()
        abi.check(self.lib, self.lib.koordhip_last_stats(self._ctx, C.byref(em), C.byref(nl), C.byref(ne), C.byref(tm)))
        return {"eval_ms": em.value, "eval_launches": nl.value, "evals": ne.value, "total_ms": tm.value}

    def set_profile_kernels(self, on: bool):
        abi.check(self.lib, self.lib.koordhip_set_profile_kernels(self._ctx, 1 if on else 0))

    def kernel_stats(self) -> dict:
        """Per-kernel device time of the last place call (profile_kernels=True)."""
        st = abi.KoordhipKernelStats()
        abi.check(self.lib, self.lib.koordhip_last_kernel_stats(self._ctx, C.byref(st)))
        return {f: getattr(st, f) for f, _ in abi.KoordhipKernelStats._fields_ if f != "reserved"}

    def kernel_names(self) -> dict:
        """Template instantiations of the last place call's evaluation and
        resolve launches, spelled as rocprofv3 names them."""
        ev, rs = C.create_string_buffer(64), C.create_string_buffer(64)
        abi.check(self.lib, self.lib.koordhip_last_kernel_names(self._ctx, ev, rs, 64))
        return {"eval": ev.value.decode(), "resolve": rs.value.decode()}

    # ---- multi-GPU ----------------------------------------------------------
    @staticmethod
    def comm_unique_id() -> bytes:
        lib = abi.load_library()
        buf = C.create_string_buffer(abi.UNIQUE_ID_BYTES)
        abi.check(lib, lib.koordhip_comm_unique_id(buf))
        return buf.raw

    def comm_init(self, uid: bytes, world: int, rank: int):
        abi.check(self.lib, self.lib.koordhip_comm_init(self._ctx, uid, world, rank))

    @staticmethod
    def comm_init_local(engines):
        """One process, several contexts (GPUs, or contexts sharing one GPU):
        engines[r] becomes rank r of a node-sharded group (koordhip_comm_init_local)."""
        lib = abi.load_library()
        arr = (C.c_void_p * len(engines))(*[e._ctx.value for e in engines])
        abi.check(lib, lib.koordhip_comm_init_local(arr, len(engines)))


def place_stream_group(engines, pods: np.ndarray) -> list:
    """Collective place_stream over a local group: one host thread per context
    (ctypes releases the GIL for the duration of each call)."""
    import threading
    out = [None] * len(engines)
    err = [None] * len(engines)

    def run(r):
        try:
            out[r] = engines[r].place_stream(pods)
        except Exception as e:  # noqa: BLE001 - re-raised below
            err[r] = e

    ts = [threading.Thread(target=run, args=(r,)) for r in range(len(engines))]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for e in err:
        if e is not None:
            raise e
    return out
