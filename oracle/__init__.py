"""TEST INFRASTRUCTURE: ctypes binding of the CPU oracle (oracle/koord_oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module.  It is the checker, never the thing measured or shipped.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

from koordinator_amd import abi
from koordinator_amd.snapshot import NodeTable

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(_HERE, "build", "libkoord_oracle.so")

_NRES = abi.NRES


class OrcState(C.Structure):
    _fields_ = [
        ("n", C.c_int32),
        ("soa", C.POINTER(abi.KoordhipNodeSoa)),
        ("flags", C.POINTER(C.c_uint8)),
        ("requested", C.POINTER(C.c_int64) * _NRES),
        ("nz_cpu_m", C.POINTER(C.c_int64)),
        ("nz_mem", C.POINTER(C.c_int64)),
        ("npods", C.POINTER(C.c_int32)),
        ("la_used_cpu_m", C.POINTER(C.c_int64)),
        ("la_used_mem", C.POINTER(C.c_int64)),
        ("la_used_prod_cpu_m", C.POINTER(C.c_int64)),
        ("la_used_prod_mem", C.POINTER(C.c_int64)),
        ("numa_free", C.POINTER(C.c_uint64) * abi.NUMA_WORDS),
        ("numa_excl_pcpu", C.POINTER(C.c_uint64) * abi.NUMA_WORDS),
        ("numa_excl_numa", C.POINTER(C.c_uint64) * abi.NUMA_WORDS),
        ("numa_alloc_cnt", C.POINTER(C.c_int32)),
        ("numa_zone_used", C.POINTER(C.c_int64)),
        ("cpuset_out", C.c_void_p),
        ("resv_allocated", C.POINTER(C.c_int64) * 2),
        ("resv_assigned", C.POINTER(C.c_int32)),
        ("resv_cpus", C.POINTER(C.c_uint64) * abi.NUMA_WORDS),
        ("no_prescore", C.c_int32),
        ("dev_used", C.POINTER(C.c_int64)),
        ("xrequested", C.POINTER(C.c_int64)),
        ("dev_out", C.c_void_p),
        ("pts_cnt", C.POINTER(C.c_int32)),
        ("ipa_cnt", C.POINTER(C.c_int32)),
        ("resv_dev", C.POINTER(C.c_int64)),
        ("resv_xallocated", C.POINTER(C.c_int64)),
        ("cur_ext", C.c_void_p),
        ("resv_restore", C.c_int32),
    ]


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        vp = C.c_void_p
        L.orc_usage_percent.restype = C.c_int64
        L.orc_usage_percent.argtypes = [C.c_int64, C.c_int64]
        L.orc_least_requested.restype = C.c_int64
        L.orc_least_requested.argtypes = [C.c_int64, C.c_int64]
        L.orc_state_init.argtypes = [C.POINTER(OrcState), C.POINTER(abi.KoordhipNodeSoa), C.c_int32]
        L.orc_state_free.argtypes = [C.POINTER(OrcState)]
        L.orc_eval.argtypes = [C.POINTER(abi.KoordhipConfig), C.POINTER(OrcState), vp, C.c_int32,
                               vp, vp, vp, C.c_int32]
        L.orc_commit.argtypes = [C.POINTER(abi.KoordhipConfig), C.POINTER(OrcState), vp, C.c_int32, C.c_int, vp]
        L.orc_commit.restype = C.c_int
        L.orc_take_cpus.argtypes = [vp, vp, vp, vp, C.c_int, C.c_int, C.c_int, C.c_int, vp]
        L.orc_take_cpus.restype = C.c_int
        L.orc_spread_order.argtypes = [vp, vp, C.c_int, vp]
        L.orc_spread_order.restype = C.c_int
        L.orc_set_cpuset_out.argtypes = [C.POINTER(OrcState), vp]
        L.orc_numa_allocate_hint.argtypes = [C.POINTER(OrcState), vp, C.c_int32, C.c_uint64, vp, vp]
        L.orc_numa_allocate_hint.restype = C.c_int
        L.orc_place_stream.argtypes = [C.POINTER(abi.KoordhipConfig), C.POINTER(OrcState), vp, C.c_int32,
                                       vp, C.c_int32]
        L.orc_la_flags.argtypes = [C.POINTER(abi.KoordhipNodeSoa), C.c_int32, vp]
        L.orc_tm_merge.argtypes = [C.c_int, C.c_uint64, vp, C.c_int32, vp]
        L.orc_tm_merge.restype = C.c_int
        L.orc_numa_hint_alloc.argtypes = [C.POINTER(OrcState), vp, C.c_int32, vp, vp, vp, vp]
        L.orc_numa_hint_alloc.restype = C.c_int
        L.orc_resv_restore.argtypes = [C.POINTER(OrcState), vp, C.c_int]
        L.orc_resv_filter.argtypes = [C.POINTER(OrcState), vp, C.c_int32]
        L.orc_resv_filter.restype = C.c_int
        L.orc_resv_nominate.argtypes = [C.POINTER(OrcState), vp, C.c_int32]
        L.orc_resv_nominate.restype = C.c_int
        L.orc_resv_nominated.argtypes = [C.POINTER(OrcState), vp, C.c_int32]
        L.orc_resv_nominated.restype = C.c_int
        L.orc_resv_score.argtypes = [C.POINTER(OrcState), vp, C.c_int32]
        L.orc_resv_score.restype = C.c_int64
        L.orc_resv_normalized.argtypes = [C.POINTER(OrcState), vp, vp, C.c_int32, vp]
        L.orc_resv_restore_delta.argtypes = [C.POINTER(OrcState), vp, C.c_int32, vp, vp, vp]
        L.orc_place_stream_ext.argtypes = [C.POINTER(abi.KoordhipConfig), C.POINTER(OrcState), vp, vp, C.c_int32,
                                           vp, C.c_int32]
        L.orc_eval_ext.argtypes = [C.POINTER(abi.KoordhipConfig), C.POINTER(OrcState), vp, vp, C.c_int32,
                                   vp, vp, vp, C.c_int32]
        L.orc_set_dev_out.argtypes = [C.POINTER(OrcState), vp]
        L.orc_dev_filter.argtypes = [C.POINTER(OrcState), vp, vp, C.c_int32]
        L.orc_dev_filter.restype = C.c_int
        L.orc_dev_score.argtypes = [C.POINTER(abi.KoordhipConfig), C.POINTER(OrcState), vp, vp, C.c_int32, C.c_int]
        L.orc_dev_score.restype = C.c_int64
        L.orc_dev_reserve.argtypes = [C.POINTER(abi.KoordhipConfig), C.POINTER(OrcState), vp, vp, C.c_int32, C.c_int, vp,
                                      C.c_int]
        L.orc_dev_reserve.restype = C.c_int
        L.orc_default_normalize.argtypes = [vp, C.c_int32, C.c_int]
        L.orc_dev_try_from_reservation.argtypes = [C.POINTER(OrcState), vp, vp, C.c_int32, C.c_int, vp]
        L.orc_dev_try_from_reservation.restype = C.c_int
        _lib = L
    return _lib


class Oracle:
    """CPU oracle over one snapshot (the same NodeTable the engine loads)."""

    def __init__(self, cfg: abi.KoordhipConfig, table: NodeTable):
        self.cfg = cfg
        self.table = table
        self._soa = table.as_soa()
        self.st = OrcState()
        if lib().orc_state_init(C.byref(self.st), C.byref(self._soa), table.n) != 0:
            raise RuntimeError("orc_state_init failed")

    def __del__(self):
        try:
            lib().orc_state_free(C.byref(self.st))
        except Exception:
            pass

    @property
    def n(self):
        return self.table.n

    def eval(self, pods: np.ndarray, status=True, scores=True, k=0):
        n, p = self.n, len(pods)
        st = np.zeros((p, n), np.uint8) if status else None
        sc = np.zeros((p, abi.NPLUGINS, n), np.int32) if scores else None
        tk = np.zeros((p, k), abi.TOPK_DTYPE) if k else None
        pods = np.ascontiguousarray(pods)
        lib().orc_eval(C.byref(self.cfg), C.byref(self.st), pods.ctypes.data, p,
                       st.ctypes.data if st is not None else None, sc.ctypes.data if sc is not None else None,
                       tk.ctypes.data if tk is not None else None, k)
        return {"status": st, "scores": sc, "topk": tk}

    def eval_ext(self, pods: np.ndarray, ext=None, status=True, scores=True, k=0):
        """koordhip_eval_ext: raw planes of the normalized plugins too, topk by the normalized totals."""
        n, p = self.n, len(pods)
        st = np.zeros((p, n), np.uint16) if status else None
        sc = np.zeros((p, abi.NPLUGINS + abi.NEXT_PLUGINS, n), np.int32) if scores else None
        tk = np.zeros((p, k), abi.TOPK_DTYPE) if k else None
        pods = np.ascontiguousarray(pods)
        x = None if ext is None else np.ascontiguousarray(ext, dtype=abi.POD_EXT_DTYPE)
        lib().orc_eval_ext(C.byref(self.cfg), C.byref(self.st), pods.ctypes.data, x.ctypes.data if x is not None else None,
                           p, st.ctypes.data if st is not None else None, sc.ctypes.data if sc is not None else None,
                           tk.ctypes.data if tk is not None else None, k)
        self.st.cur_ext = None              # (the records die with this call)
        return {"status": st, "scores": sc, "topk": tk}

    def place_stream_ext(self, pods: np.ndarray, ext=None, threads: int = 1, cpusets: bool = False,
                         devices: bool = False):
        """The reference cycle with koordhip_pod_ext records: (placements[, cpusets][, device slots [n][TYPES]])."""
        pods = np.ascontiguousarray(pods)
        x = None if ext is None else np.ascontiguousarray(ext, dtype=abi.POD_EXT_DTYPE)
        out = np.zeros(len(pods), np.int32)
        cs = np.zeros((len(pods), abi.NUMA_WORDS), np.uint64) if cpusets else None
        dv = np.zeros((len(pods), abi.DEV_TYPES), np.uint32) if devices else None
        lib().orc_set_cpuset_out(C.byref(self.st), cs.ctypes.data if cs is not None else None)
        lib().orc_set_dev_out(C.byref(self.st), dv.ctypes.data if dv is not None else None)
        rc = lib().orc_place_stream_ext(C.byref(self.cfg), C.byref(self.st), pods.ctypes.data,
                                        x.ctypes.data if x is not None else None, len(pods), out.ctypes.data, threads)
        lib().orc_set_cpuset_out(C.byref(self.st), None)
        lib().orc_set_dev_out(C.byref(self.st), None)
        self.st.cur_ext = None
        if rc != 0:
            raise RuntimeError("orc_place_stream_ext failed")
        res = (out,) + ((cs,) if cpusets else ()) + ((dv,) if devices else ())
        return res if len(res) > 1 else out

    def resv_dev_state(self) -> np.ndarray:
        """The device-holding reservations' column [n][2][TYPES][dev_slots][RES] (zeros without one)."""
        S = max(1, self.table.dev_slots)
        shape = (self.n, 2, abi.DEV_TYPES, S, abi.DEV_RES)
        if not self.st.resv_dev:
            return np.zeros(shape, np.int64)
        return np.ctypeslib.as_array(self.st.resv_dev, shape=shape).copy()

    def resv_scalar_state(self) -> np.ndarray:
        """The device-holding reservations' extended-scalar Allocated, [n][NXRES]
        (zeros without the resv_xalloc column)."""
        if not self.st.resv_xallocated:
            return np.zeros((self.n, abi.NXRES), np.int64)
        return np.ctypeslib.as_array(self.st.resv_xallocated, shape=(abi.NXRES, self.n)).T.copy()

    def dev_try_from_reservation(self, pod, ext_rec, node: int, from_resv: bool = False):
        """tryAllocateFromReservation over node's matched reservation holding
        devices: (1 allocated / 0 none / -1 Unschedulable, slots [TYPES])."""
        pod = np.ascontiguousarray(np.atleast_1d(pod))
        x = np.ascontiguousarray(np.atleast_1d(ext_rec), dtype=abi.POD_EXT_DTYPE)
        sl = np.zeros(abi.DEV_TYPES, np.uint32)
        self.st.resv_restore = 1
        r = lib().orc_dev_try_from_reservation(C.byref(self.st), pod.ctypes.data, x.ctypes.data, node,
                                               int(from_resv), sl.ctypes.data)
        return int(r), sl

    def dev_state(self) -> dict:
        """DeviceShare deviceUsed [n][TYPES][S][RES] and the extended scalars' Requested [n][NXRES]."""
        n, S = self.n, max(1, self.table.dev_slots)
        du = (np.ctypeslib.as_array(self.st.dev_used, shape=(n, abi.DEV_TYPES, S, abi.DEV_RES)).copy()
              if self.table.dev_slots else np.zeros((n, abi.DEV_TYPES, S, abi.DEV_RES), np.int64))
        xr = np.ctypeslib.as_array(self.st.xrequested, shape=(abi.NXRES, n)).T.copy()
        return {"dev_used": du, "xrequested": xr}

    def pts_counts(self) -> np.ndarray:
        """PodTopologySpread matching pods per node and table constraint [n][cons]."""
        m = self.table.pts
        if m is None or not m.cons_key:
            return np.zeros((self.n, 0), np.int32)
        return np.ctypeslib.as_array(self.st.pts_cnt, shape=(len(m.cons_key), self.n)).T.copy()

    def ipa_counts(self) -> np.ndarray:
        """InterPodAffinity count entries' pods per node [n][ents]."""
        m = self.table.ipa
        if m is None or not m.ent_key:
            return np.zeros((self.n, 0), np.int32)
        return np.ctypeslib.as_array(self.st.ipa_cnt, shape=(len(m.ent_key), self.n)).T.copy()

    def dev_filter(self, ext_rec, node: int) -> bool:
        x = np.ascontiguousarray(np.atleast_1d(ext_rec), dtype=abi.POD_EXT_DTYPE)
        return bool(lib().orc_dev_filter(C.byref(self.st), None, x.ctypes.data, node))

    def dev_score(self, ext_rec, node: int, nominated: bool = False) -> int:
        x = np.ascontiguousarray(np.atleast_1d(ext_rec), dtype=abi.POD_EXT_DTYPE)
        return int(lib().orc_dev_score(C.byref(self.cfg), C.byref(self.st), None, x.ctypes.data, node, int(nominated)))

    def dev_reserve(self, ext_rec, node: int, nominated: bool = False, apply: bool = True):
        """(ok, slots [TYPES])"""
        x = np.ascontiguousarray(np.atleast_1d(ext_rec), dtype=abi.POD_EXT_DTYPE)
        sl = np.zeros(abi.DEV_TYPES, np.uint32)
        rc = lib().orc_dev_reserve(C.byref(self.cfg), C.byref(self.st), None, x.ctypes.data, node, int(nominated),
                                   sl.ctypes.data, int(apply))
        return rc == 0, sl

    def commit(self, pod: np.ndarray, node: int, sign: int = 1, cpus=None):
        """Reserve (sign 1) / Unreserve (sign -1).  Returns (rc, cpus): rc is
        abi.E_RESERVE when the NUMA Allocate fails; for Unreserve of a cpuset
        pod pass the cpus it was given."""
        pod = np.ascontiguousarray(np.atleast_1d(pod))
        buf = np.zeros(abi.NUMA_WORDS, np.uint64) if cpus is None else np.ascontiguousarray(cpus, np.uint64).copy()
        rc = lib().orc_commit(C.byref(self.cfg), C.byref(self.st), pod.ctypes.data, node, sign, buf.ctypes.data)
        return rc, buf

    def place_stream(self, pods: np.ndarray, threads: int = 1, cpusets: bool = False):
        pods = np.ascontiguousarray(pods)
        out = np.zeros(len(pods), np.int32)
        cs = np.zeros((len(pods), abi.NUMA_WORDS), np.uint64) if cpusets else None
        lib().orc_set_cpuset_out(C.byref(self.st), cs.ctypes.data if cs is not None else None)
        rc = lib().orc_place_stream(C.byref(self.cfg), C.byref(self.st), pods.ctypes.data, len(pods),
                                    out.ctypes.data, threads)
        lib().orc_set_cpuset_out(C.byref(self.st), None)
        if rc != 0:
            raise RuntimeError("orc_place_stream failed")
        return (out, cs) if cpusets else out

    def flags(self) -> np.ndarray:
        return np.ctypeslib.as_array(self.st.flags, shape=(self.n,)).copy()

    def state(self) -> dict:
        n = self.n
        a64 = lambda p: np.ctypeslib.as_array(p, shape=(n,)).copy()
        return {
            "requested": np.stack([a64(self.st.requested[r]) for r in range(_NRES)]),
            "nz": np.stack([a64(self.st.nz_cpu_m), a64(self.st.nz_mem)]),
            "npods": np.ctypeslib.as_array(self.st.npods, shape=(n,)).copy(),
            "la_used": np.stack([a64(self.st.la_used_cpu_m), a64(self.st.la_used_mem)]),
            "la_used_prod": np.stack([a64(self.st.la_used_prod_cpu_m), a64(self.st.la_used_prod_mem)]),
        }

    def numa_state(self) -> dict:
        n = self.n
        a = lambda p, shape=(n,): np.ctypeslib.as_array(p, shape=shape).copy()
        return {
            "free": np.stack([a(self.st.numa_free[w]) for w in range(abi.NUMA_WORDS)]),
            "excl_pcpu": np.stack([a(self.st.numa_excl_pcpu[w]) for w in range(abi.NUMA_WORDS)]),
            "excl_numa": np.stack([a(self.st.numa_excl_numa[w]) for w in range(abi.NUMA_WORDS)]),
            "alloc_cnt": a(self.st.numa_alloc_cnt),
            "zone_used": a(self.st.numa_zone_used, (n, 2, abi.NUMA_MAX_NODES)),
        }

    def resv_state(self) -> dict:
        """Allocated [2][S n], assigned [S n] (S = the table's reservation slots, slot-major)."""
        n = self.n * max(1, self.table.resv_slots)
        a = lambda p: np.ctypeslib.as_array(p, shape=(n,)).copy()
        rc = (np.stack([a(self.st.resv_cpus[w]) for w in range(abi.NUMA_WORDS)]) if self.st.resv_cpus[0]
              else np.zeros((abi.NUMA_WORDS, n), np.uint64))
        return {"allocated": np.stack([a(self.st.resv_allocated[0]), a(self.st.resv_allocated[1])]),
                "assigned": a(self.st.resv_assigned), "cpus": rc}

    def numa_allocate_hint(self, pod: np.ndarray, node: int, mask: int):
        """resourceManager.Allocate with hint `mask` (0 = none): (ok, zone
        amounts [2][NUMA_MAX_NODES] (cpu milli, memory), cpus [WORDS])."""
        pod = np.ascontiguousarray(np.atleast_1d(pod))
        z = np.zeros((2, abi.NUMA_MAX_NODES), np.int64)
        c = np.zeros(abi.NUMA_WORDS, np.uint64)
        ok = lib().orc_numa_allocate_hint(C.byref(self.st), pod.ctypes.data, node, mask, z.ctypes.data, c.ctypes.data)
        return bool(ok), z, c

    def resv_restore_delta(self, pod: np.ndarray, node: int):
        """(requested delta [cpu, mem], non-zero delta [cpu, mem], pod-count delta) of the restore."""
        self.st.cur_ext = None    # a plain record: no scalar requests (no stale ext pointer)
        pod = np.ascontiguousarray(np.atleast_1d(pod))
        dr, dn, dp = np.zeros(2, np.int64), np.zeros(2, np.int64), np.zeros(1, np.int32)
        lib().orc_resv_restore_delta(C.byref(self.st), pod.ctypes.data, node, dr.ctypes.data, dn.ctypes.data,
                                     dp.ctypes.data)
        return dr, dn, int(dp[0])

    def resv_filter(self, pod: np.ndarray, node: int) -> bool:
        """filterWithReservations of (pod, node) inside the pod's cycle (restore applied)."""
        self.st.cur_ext = None    # a plain record: no scalar requests (no stale ext pointer)
        pod = np.ascontiguousarray(np.atleast_1d(pod))
        lib().orc_resv_restore(C.byref(self.st), pod.ctypes.data, 1)
        ok = lib().orc_resv_filter(C.byref(self.st), pod.ctypes.data, node)
        lib().orc_resv_restore(C.byref(self.st), pod.ctypes.data, -1)
        return bool(ok)

    def resv_nominated(self, pod: np.ndarray, node: int) -> bool:
        self.st.cur_ext = None    # a plain record: no scalar requests (no stale ext pointer)
        pod = np.ascontiguousarray(np.atleast_1d(pod))
        return bool(lib().orc_resv_nominated(C.byref(self.st), pod.ctypes.data, node))

    def resv_nominate(self, pod: np.ndarray, node: int) -> int:
        """NominateReservation on `node`: the nominated reservation's slot, -1 for none."""
        self.st.cur_ext = None    # a plain record: no scalar requests (no stale ext pointer)
        pod = np.ascontiguousarray(np.atleast_1d(pod))
        return int(lib().orc_resv_nominate(C.byref(self.st), pod.ctypes.data, node))

    def resv_score(self, pod: np.ndarray, node: int) -> int:
        self.st.cur_ext = None    # a plain record: no scalar requests (no stale ext pointer)
        pod = np.ascontiguousarray(np.atleast_1d(pod))
        return int(lib().orc_resv_score(C.byref(self.st), pod.ctypes.data, node))

    def resv_normalized(self, pod: np.ndarray, feasible) -> np.ndarray:
        """PreScore + Score + DefaultNormalizeScore of the Reservation plugin over `feasible`."""
        self.st.cur_ext = None    # a plain record: no scalar requests (no stale ext pointer)
        pod = np.ascontiguousarray(np.atleast_1d(pod))
        f = np.ascontiguousarray(feasible, np.int32)
        out = np.zeros(len(f), np.int64)
        lib().orc_resv_normalized(C.byref(self.st), pod.ctypes.data, f.ctypes.data, len(f), out.ctypes.data)
        return out

    def hint_alloc(self, pod: np.ndarray, node: int):
        """The topology-manager admit + allocateResourcesByHint for (pod, node):
        (ok, mask or None for a nil hint, admit, zones [2][NUMA_MAX_NODES])."""
        pod = np.ascontiguousarray(np.atleast_1d(pod))
        mask, nil, admit = C.c_uint64(), C.c_int32(), C.c_int32()
        zones = np.zeros((2, abi.NUMA_MAX_NODES), np.int64)
        ok = lib().orc_numa_hint_alloc(C.byref(self.st), pod.ctypes.data, node, C.byref(mask), C.byref(nil),
                                       C.byref(admit), zones.ctypes.data)
        return bool(ok), (None if nil.value else mask.value), bool(admit.value), zones


def take_cpus(cls: np.ndarray, avail, need: int, bind_policy: int, excl_policy: int = 0, most_allocated: bool = True,
              excl_pcpu=None, excl_numa=None):
    """takeCPUs on one topology class (a NUMA_CLASS_DTYPE record); masks are
    [NUMA_WORDS] uint64 over core-major positions.  Returns the mask or None."""
    cls = np.ascontiguousarray(cls, dtype=abi.NUMA_CLASS_DTYPE)
    m = lambda x: np.ascontiguousarray(np.zeros(abi.NUMA_WORDS, np.uint64) if x is None else x, np.uint64)
    av, ep, en = m(avail), m(excl_pcpu), m(excl_numa)
    out = np.zeros(abi.NUMA_WORDS, np.uint64)
    ok = lib().orc_take_cpus(cls.ctypes.data, av.ctypes.data, ep.ctypes.data, en.ctypes.data, need, bind_policy,
                             excl_policy, int(most_allocated), out.ctypes.data)
    return out if ok else None


def spread_order(cls: np.ndarray, avail, most_allocated: bool = True):
    cls = np.ascontiguousarray(cls, dtype=abi.NUMA_CLASS_DTYPE)
    av = np.ascontiguousarray(avail, np.uint64)
    ids = np.zeros(abi.NUMA_MAX_CPUS, np.int32)
    n = lib().orc_spread_order(cls.ctypes.data, av.ctypes.data, int(most_allocated), ids.ctypes.data)
    return ids[:n].tolist()


TM_PROVIDER_EMPTY, TM_RES_NIL, TM_RES_EMPTY, TM_RES_HINTS = 0, 1, 2, 3
TM_HINT_DTYPE = np.dtype([("mask", "<u8"), ("preferred", "<i4"), ("nil", "<i4")])
TM_ENTRY_DTYPE = np.dtype([("kind", "<i4"), ("n", "<i4"), ("h", TM_HINT_DTYPE, (255,))])


def tm_merge(policy: int, numa_nodes: int, entries):
    """Topology-manager Merge.  entries: one item per filterProvidersHints
    list -- "provider-empty", "nil", "empty", or a list of (mask|None,
    preferred).  Returns (admit, mask|None, preferred)."""
    e = np.zeros(max(1, len(entries)), TM_ENTRY_DTYPE)
    for q, ent in enumerate(entries):
        if isinstance(ent, str):
            e[q]["kind"] = {"provider-empty": TM_PROVIDER_EMPTY, "nil": TM_RES_NIL, "empty": TM_RES_EMPTY}[ent]
            continue
        e[q]["kind"] = TM_RES_HINTS
        e[q]["n"] = len(ent)
        for j, (m, pref) in enumerate(ent):
            e[q]["h"][j] = (0 if m is None else m, int(pref), int(m is None))
    out = np.zeros(1, TM_HINT_DTYPE)
    admit = lib().orc_tm_merge(policy, numa_nodes, e.ctypes.data, len(entries), out.ctypes.data)
    h = out[0]
    return bool(admit), (None if h["nil"] else int(h["mask"])), bool(h["preferred"])


def usage_percent(used_milli: int, total_milli: int) -> int:
    return lib().orc_usage_percent(used_milli, total_milli)


def least_requested(req: int, cap: int) -> int:
    return lib().orc_least_requested(req, cap)


def default_normalize(scores, reverse: bool = False) -> np.ndarray:
    """(upstream) DefaultNormalizeScore(MaxNodeScore, reverse) over a list."""
    a = np.ascontiguousarray(scores, dtype=np.int64).copy()
    lib().orc_default_normalize(a.ctypes.data, len(a), int(reverse))
    return a
