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
        L.orc_commit.argtypes = [C.POINTER(abi.KoordhipConfig), C.POINTER(OrcState), vp, C.c_int32, C.c_int]
        L.orc_place_stream.argtypes = [C.POINTER(abi.KoordhipConfig), C.POINTER(OrcState), vp, C.c_int32,
                                       vp, C.c_int32]
        L.orc_la_flags.argtypes = [C.POINTER(abi.KoordhipNodeSoa), C.c_int32, vp]
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

    def commit(self, pod: np.ndarray, node: int, sign: int = 1):
        pod = np.ascontiguousarray(np.atleast_1d(pod))
        lib().orc_commit(C.byref(self.cfg), C.byref(self.st), pod.ctypes.data, node, sign)

    def place_stream(self, pods: np.ndarray, threads: int = 1) -> np.ndarray:
        pods = np.ascontiguousarray(pods)
        out = np.zeros(len(pods), np.int32)
        rc = lib().orc_place_stream(C.byref(self.cfg), C.byref(self.st), pods.ctypes.data, len(pods),
                                    out.ctypes.data, threads)
        if rc != 0:
            raise RuntimeError("orc_place_stream failed")
        return out

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


def usage_percent(used_milli: int, total_milli: int) -> int:
    return lib().orc_usage_percent(used_milli, total_milli)


def least_requested(req: int, cap: int) -> int:
    return lib().orc_least_requested(req, cap)
