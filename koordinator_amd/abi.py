"""ctypes mirror of include/koordhip.h and the loader for libkoordhip.so.

The library is built in-tree by __graft_entry__.build() into
koordinator_amd/lib/libkoordhip.so.  There is no fallback: if the library is
missing, importing the engine raises.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

KOORDHIP_ABI_VERSION = 14
NRES = 5
NPLUGINS = 4

PLUGIN_FIT, PLUGIN_LOADAWARE, PLUGIN_NUMA, PLUGIN_RESERVATION = 1, 2, 4, 8
PLUGIN_NODE_STATIC, PLUGIN_BALANCED = 16, 32
# normalized-score plugins (the exact sequential cycle, koordhip_place_stream_ext)
PLUGIN_DEVICESHARE, PLUGIN_AFFINITY_SCORE, PLUGIN_TAINT_SCORE, PLUGIN_PTS, PLUGIN_IPA = 64, 128, 256, 512, 1024
NEXT_PLUGINS = 5
EXT_PLUGIN_BITS = (PLUGIN_DEVICESHARE, PLUGIN_AFFINITY_SCORE, PLUGIN_TAINT_SCORE, PLUGIN_PTS, PLUGIN_IPA)
NORMALIZED_PLUGINS = PLUGIN_DEVICESHARE | PLUGIN_AFFINITY_SCORE | PLUGIN_TAINT_SCORE | PLUGIN_PTS | PLUGIN_IPA
PTS_KEYS, PTS_DOMAINS, PTS_CONS, PTS_CLASSES, PTS_POD = 4, 64, 8, 8, 4
PTS_HARD, PTS_SELF = 1, 2
IPA_ENTRIES = 32
IPA_SELF = 1
NXRES = 8
DEV_TYPES, DEV_SLOTS, DEV_RES = 3, 8, 3
DEV_GPU, DEV_RDMA, DEV_FPGA = 0, 1, 2
PODX_DEVICE = 1
# upstream NodeUnschedulable / NodeName / NodeAffinity / TaintToleration all map
# to the host-resolved static filter bit
PLUGIN_BITS = {"NodeResourcesFit": PLUGIN_FIT, "LoadAwareScheduling": PLUGIN_LOADAWARE,
               "NodeNUMAResource": PLUGIN_NUMA, "Reservation": PLUGIN_RESERVATION,
               "NodeUnschedulable": PLUGIN_NODE_STATIC, "NodeAffinity": PLUGIN_NODE_STATIC,
               "NodeName": PLUGIN_NODE_STATIC,
               "TaintToleration": PLUGIN_NODE_STATIC, "NodeResourcesBalancedAllocation": PLUGIN_BALANCED}
# plugin_weight[p] / score plane p
SCORE_PLUGIN_BITS = (PLUGIN_FIT, PLUGIN_LOADAWARE, PLUGIN_NUMA, PLUGIN_BALANCED)
MAX_STATIC_CLASSES = 32
RES_CPU, RES_MEM, RES_EPH, RES_BCPU, RES_BMEM = range(5)

LA_HAS_METRIC, LA_FILTER_SKIP, LA_SCORE_EXPIRED, LA_FILTER_USAGE = 1, 2, 4, 8
LA_PROD_MODE, LA_HAS_PODS_METRIC, LA_AGGREGATED = 16, 32, 64

POD_PROD, POD_DAEMONSET, POD_HAS_REQ, POD_REQ_BCPU, POD_REQ_BMEM = 1, 2, 4, 8, 16
POD_CPUSET, POD_NUMA_SKIP, POD_NUMA_ERROR = 32, 64, 128
POD_KEY_CPU, POD_KEY_MEM = 256, 512
POD_RESV_AFFINITY = 1024
POD_RESERVE = 2048                  # a reserve pod (IsReservePod): its reservation's nodeName / AllocatePolicy checks
POD_RESERVE_POLICY_SHIFT = 12       # bits 12-13: the reserve pod's AllocatePolicy (RESV_POLICY_* codes)
POD_RESV_OPERATING = 16384          # a reservation-operating-mode pod (AllocatePolicy Aligned in bits 12-13)
POD_CPUSET_QOS = 32768              # AllowUseCPUSet: koord-prod and QoS LSE / LSR (nodenumaresource/util.go:42-49)

RESV_PRESENT, RESV_ALLOCATE_ONCE, RESV_UNSCHEDULABLE, RESV_ORDERED = 1, 2, 4, 8
RESV_KEY_CPU, RESV_KEY_MEM = 16, 32
RESV_POLICY_SHIFT, RESV_GROUP_SHIFT = 6, 8
RESV_POLICY_DEFAULT, RESV_POLICY_ALIGNED, RESV_POLICY_RESTRICTED = 0, 1, 2
RESV_MAX_GROUPS, RESV_MAX_ORDERS = 64, 1024
RESV_SLOTS = 4   # Available reservations per node on the pipelined greedy
RESV_SLOTS_MAX = 8   # ... in a snapshot (koordhip_node_soa.resv_slots <= this; more than RESV_SLOTS: the sequential cycle)

CPUBIND_NONE, CPUBIND_FULL_PCPUS, CPUBIND_SPREAD_BY_PCPUS = 0, 1, 2
CPUEXCL_NONE, CPUEXCL_PCPU, CPUEXCL_NUMA = 0, 1, 2
NODE_CPUBIND_NONE, NODE_CPUBIND_FULL_PCPUS_ONLY, NODE_CPUBIND_SPREAD_BY_PCPUS = 0, 1, 2
NODE_NUMA_MOST_ALLOCATED = 4
NODE_NUMA_POLICY_SHIFT = 3
NUMA_TOPO_NONE, NUMA_TOPO_BEST_EFFORT, NUMA_TOPO_RESTRICTED, NUMA_TOPO_SINGLE_NUMA_NODE = 0, 1, 2, 3
NUMA_MAX_CPUS, NUMA_MAX_NODES, NUMA_WORDS = 256, 8, 4
NUMA_MAX_ZONES = 8


def numa_policy(required: int = 0, preferred: int = 0, exclusive: int = 0) -> int:
    return (required & 3) | ((preferred & 3) << 2) | ((exclusive & 3) << 4)

ST_FIT_FAIL, ST_LA_FAIL, ST_NUMA_FAIL, ST_RESV_FAIL, ST_STATIC_FAIL = 1, 2, 4, 8, 16
ST_DEVICE_FAIL, ST_XFIT_FAIL, ST_PTS_FAIL, ST_IPA_FAIL = 32, 64, 128, 256
UNSCHEDULABLE, RESERVE_FAILED = -1, -2
E_INVAL, E_RESERVE = -1, -6
UNIQUE_ID_BYTES = 128

_i64p = C.POINTER(C.c_int64)
_i32p = C.POINTER(C.c_int32)
_u8p = C.POINTER(C.c_uint8)
_u64p = C.POINTER(C.c_uint64)


class KoordhipKernelStats(C.Structure):
    """include/koordhip.h koordhip_kernel_stats"""
    _fields_ = [("scan_ms", C.c_double), ("scan_launches", C.c_int64),
                ("select_ms", C.c_double), ("select_launches", C.c_int64),
                ("resolve_ms", C.c_double), ("resolve_launches", C.c_int64),
                ("total_ms", C.c_double), ("evals", C.c_int64), ("pods", C.c_int64), ("rounds", C.c_int64),
                ("round_pods", C.c_int64), ("lag", C.c_int64), ("executed_evals", C.c_int64),
                ("plan_us", C.c_int32), ("flags", C.c_int32)]


KSTAT_LOCAL = 1


class KoordhipConfig(C.Structure):
    _fields_ = [
        ("abi_version", C.c_int32),
        ("filter_plugins", C.c_uint32),
        ("score_plugins", C.c_uint32),
        ("device", C.c_int32),
        ("plugin_weight", C.c_int64 * NPLUGINS),
        ("fit_weight", C.c_int64 * NRES),
        ("la_weight_cpu", C.c_int64),
        ("la_weight_mem", C.c_int64),
        ("la_score_according_prod_usage", C.c_int32),
        ("batch_pods", C.c_int32),
        ("numa_weight_cpu", C.c_int32),
        ("numa_weight_mem", C.c_int32),
        ("profile_kernels", C.c_int32),
        ("numa_most_allocated", C.c_int32),
        ("reservation_weight", C.c_int32),
        ("reserved", C.c_int32 * 5),
        ("ext_weight", C.c_int32 * NEXT_PLUGINS),
        ("dev_most_allocated", C.c_int32),
        ("dev_res_weight", C.c_int32 * 5),
        ("reserved2", C.c_int32 * 1),
    ]


class KoordhipNodeSoa(C.Structure):
    _fields_ = [
        ("alloc", _i64p * NRES),
        ("alloc_pods", _i32p),
        ("requested", _i64p * NRES),
        ("nz_cpu_m", _i64p),
        ("nz_mem", _i64p),
        ("npods", _i32p),
        ("la_alloc_cpu_m", _i64p),
        ("la_alloc_mem", _i64p),
        ("la_used_cpu_m", _i64p),
        ("la_used_mem", _i64p),
        ("la_used_prod_cpu_m", _i64p),
        ("la_used_prod_mem", _i64p),
        ("laf_used_m", _i64p * 2),
        ("laf_total_m", _i64p * 2),
        ("laf_prod_used_m", _i64p * 2),
        ("laf_thr", _i64p * 2),
        ("laf_prod_thr", _i64p * 2),
        ("la_flags", _u8p),
        ("numa_classes", C.c_void_p),
        ("n_numa_classes", C.c_int32),
        ("reserved0", C.c_int32),
        ("numa_class", _i32p),
        ("numa_free", _u64p * NUMA_WORDS),
        ("numa_excl_pcpu", _u64p * NUMA_WORDS),
        ("numa_excl_numa", _u64p * NUMA_WORDS),
        ("numa_alloc_cnt", _i32p),
        ("numa_flags", _u8p),
        ("numa_zone_alloc", _i64p),
        ("numa_zone_used", _i64p),
        ("numa_amp_cpu", C.POINTER(C.c_double)),
        ("resv_flags", C.POINTER(C.c_uint32)),
        ("resv_order_rank", _i32p),
        ("resv_alloc", _i64p * 2),
        ("resv_nz", _i64p * 2),
        ("resv_allocated", _i64p * 2),
        ("resv_assigned", _i32p),
        ("static_allow", C.POINTER(C.c_uint32)),
        ("resv_slots", C.c_int32),
        ("reserved1", C.c_int32),
        ("resv_cpus", _u64p * NUMA_WORDS),
        ("dev_slots", C.c_int32),
        ("reserved2", C.c_int32),
        ("dev_present", _u8p),
        ("dev_minor", _i32p),
        ("dev_total", _i64p),
        ("dev_used", _i64p),
        ("xalloc", _i64p),
        ("xrequested", _i64p),
        ("static_score", C.POINTER(C.c_uint16) * 2),
        ("pts_keys", C.c_int32),
        ("pts_hostname", C.c_uint32),
        ("pts_ndom", C.c_int32 * PTS_KEYS),
        ("pts_cons", C.c_int32),
        ("pts_classes", C.c_int32),
        ("pts_cons_key", C.c_int32 * PTS_CONS),
        ("pts_dom", _i32p),
        ("pts_cnt", _i32p),
        ("pts_elig", C.POINTER(C.c_uint16)),
        ("ipa_ents", C.c_int32),
        ("ipa_reserved", C.c_int32),
        ("ipa_ent_key", C.c_int32 * IPA_ENTRIES),
        ("ipa_cnt", _i32p),
        ("resv_dev_slot", _i32p),
        ("resv_dev", _i64p),
        ("resv_xalloc", _i64p),
        ("resv_xallocated", _i64p),
    ]


# numpy twin of koordhip_numa_class
NUMA_CLASS_DTYPE = np.dtype([
    ("num_cpus", "<i4"), ("num_cores", "<i4"), ("num_nodes", "<i4"), ("num_sockets", "<i4"),
    ("cpus_per_core", "<i4"), ("reserved0", "<i4"),
    ("cpu_id", "<i4", (NUMA_MAX_CPUS,)),
    ("node_of", "u1", (NUMA_MAX_CPUS,)),
    ("socket_of", "u1", (NUMA_MAX_CPUS,)),
], align=True)
assert NUMA_CLASS_DTYPE.itemsize == 24 + 4 * 256 + 512


class KoordhipTopk(C.Structure):
    _fields_ = [("node", C.c_int32), ("score", C.c_int32)]


# numpy twin of koordhip_pod (96 bytes)
POD_DTYPE = np.dtype([
    ("req", "<i8", (NRES,)),
    ("nz_cpu_m", "<i8"),
    ("nz_mem", "<i8"),
    ("est_cpu", "<i8"),
    ("est_mem", "<i8"),
    ("flags", "<u4"),
    ("numa_cpus", "<i4"),
    ("numa_policy", "<u4"),
    ("static_class", "<i4"),
    ("resv_match", "<u8"),
], align=True)
assert POD_DTYPE.itemsize == 96
TOPK_DTYPE = np.dtype([("node", "<i4"), ("score", "<i4")])
# numpy twin of koordhip_pod_ext (176 bytes)
POD_EXT_DTYPE = np.dtype([
    ("dev_req", "<i8", (DEV_TYPES, DEV_RES)),
    ("xreq", "<i8", (NXRES,)),
    ("flags", "<u4"),
    ("xmask", "<u4"),
    ("pts_n", "u1"),
    ("pts_class", "u1"),
    ("pts_match", "u1"),
    ("pts_pad", "u1"),
    ("pts_c", "u1", (PTS_POD,)),
    ("pts_fl", "u1", (PTS_POD,)),
    ("pts_skew", "<i4", (PTS_POD,)),
    ("reserve_node", "<i4"),
    ("ipa_inc", "<u4"),
    ("ipa_aff", "<u4"),
    ("ipa_anti", "<u4"),
    ("ipa_score", "<u4"),
    ("ipa_flags", "<u4"),
    ("ipa_reserved", "<i4"),
    ("ipa_w", "<i4", (IPA_ENTRIES,)),
], align=True)
assert POD_EXT_DTYPE.itemsize == 328


def pod_ext_array(n: int) -> np.ndarray:
    """n koordhip_pod_ext records with no device request (dev_req -1 / 0)."""
    a = np.zeros(n, POD_EXT_DTYPE)
    a["dev_req"][:, DEV_GPU, :] = -1
    return a

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libkoordhip.so")


class KoordhipError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"koordhip error {code}: {msg}")
        self.code = code


_lib = None


def load_library(path: str = LIB_PATH):
    """Load libkoordhip.so.  Fails loudly when it has not been built.

    KOORDHIP_LIB names another build of the same library (A/B of compile-time
    variants, e.g. `make VARIANT=...`); it must still be a libkoordhip build."""
    global _lib
    if _lib is not None:
        return _lib
    path = os.environ.get("KOORDHIP_LIB", path)
    if not os.path.exists(path):
        raise RuntimeError(f"{path} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
                           " (there is no CPU fallback)")
    lib = C.CDLL(path)
    vp = C.c_void_p
    sig = {
        "koordhip_last_error": (C.c_char_p, []),
        "koordhip_abi_version": (C.c_int, []),
        "koordhip_create": (C.c_int, [C.POINTER(KoordhipConfig), C.POINTER(vp)]),
        "koordhip_destroy": (C.c_int, [vp]),
        "koordhip_load_snapshot": (C.c_int, [vp, C.POINTER(KoordhipNodeSoa), C.c_int32]),
        "koordhip_update_nodes": (C.c_int, [vp, _i32p, C.POINTER(KoordhipNodeSoa), C.c_int32]),
        "koordhip_read_nodes": (C.c_int, [vp, _i64p, _i64p, _i32p, _i64p, _i64p]),
        "koordhip_eval": (C.c_int, [vp, vp, C.c_int32, _u8p, _i32p, vp, C.c_int32]),
        "koordhip_place_stream": (C.c_int, [vp, vp, C.c_int32, _i32p]),
        "koordhip_place_stream_ext": (C.c_int, [vp, vp, vp, C.c_int32, _i32p]),
        "koordhip_eval_ext": (C.c_int, [vp, vp, vp, C.c_int32, C.POINTER(C.c_uint16), _i32p, vp, C.c_int32]),
        "koordhip_fetch_devices": (C.c_int, [vp, C.POINTER(C.c_uint32), C.c_int32]),
        "koordhip_read_devices": (C.c_int, [vp, _i64p, _i64p]),
        "koordhip_read_pts": (C.c_int, [vp, _i32p]),
        "koordhip_read_ipa": (C.c_int, [vp, _i32p]),
        "koordhip_stage_pods": (C.c_int, [vp, vp, C.c_int32]),
        "koordhip_stage_pods_ext": (C.c_int, [vp, vp, vp, C.c_int32]),
        "koordhip_place_staged": (C.c_int, [vp]),
        "koordhip_fetch_placements": (C.c_int, [vp, _i32p, C.c_int32]),
        "koordhip_synchronize": (C.c_int, [vp]),
        "koordhip_checkpoint": (C.c_int, [vp]),
        "koordhip_restore": (C.c_int, [vp]),
        "koordhip_commit": (C.c_int, [vp, vp, C.c_int32, _u64p]),
        "koordhip_uncommit": (C.c_int, [vp, vp, C.c_int32, _u64p]),
        "koordhip_commit_ext": (C.c_int, [vp, vp, vp, C.c_int32, _u64p, C.POINTER(C.c_uint32)]),
        "koordhip_uncommit_ext": (C.c_int, [vp, vp, vp, C.c_int32, _u64p, C.POINTER(C.c_uint32)]),
        "koordhip_fetch_cpusets": (C.c_int, [vp, _u64p, C.c_int32]),
        "koordhip_read_numa": (C.c_int, [vp, _u64p, _u64p, _u64p, _i32p]),
        "koordhip_read_numa_zones": (C.c_int, [vp, _i64p]),
        "koordhip_read_reservations": (C.c_int, [vp, _i64p, _i32p]),
        "koordhip_read_resv_cpus": (C.c_int, [vp, _u64p]),
        "koordhip_read_resv_devices": (C.c_int, [vp, _i64p]),
        "koordhip_read_resv_scalars": (C.c_int, [vp, _i64p]),
        "koordhip_last_stats": (C.c_int, [vp, C.POINTER(C.c_double), C.POINTER(C.c_int64),
                                          C.POINTER(C.c_int64), C.POINTER(C.c_double)]),
        "koordhip_last_kernel_stats": (C.c_int, [vp, C.POINTER(KoordhipKernelStats)]),
        "koordhip_set_profile_kernels": (C.c_int, [vp, C.c_int32]),
        "koordhip_last_kernel_names": (C.c_int, [vp, C.c_char_p, C.c_char_p, C.c_int32]),
        "koordhip_comm_unique_id": (C.c_int, [C.c_char_p]),
        "koordhip_comm_init": (C.c_int, [vp, C.c_char_p, C.c_int32, C.c_int32]),
        "koordhip_comm_init_local": (C.c_int, [C.POINTER(vp), C.c_int32]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    if lib.koordhip_abi_version() != KOORDHIP_ABI_VERSION:
        raise RuntimeError("libkoordhip.so ABI version mismatch; rebuild")
    _lib = lib
    return lib


EXPORTED_SYMBOLS = [
    "koordhip_last_error", "koordhip_abi_version", "koordhip_create", "koordhip_destroy",
    "koordhip_load_snapshot", "koordhip_update_nodes", "koordhip_read_nodes", "koordhip_eval",
    "koordhip_place_stream", "koordhip_place_stream_ext", "koordhip_eval_ext", "koordhip_fetch_devices",
    "koordhip_read_devices", "koordhip_read_pts", "koordhip_read_ipa", "koordhip_stage_pods", "koordhip_stage_pods_ext", "koordhip_place_staged", "koordhip_fetch_placements",
    "koordhip_synchronize", "koordhip_checkpoint", "koordhip_restore", "koordhip_commit", "koordhip_uncommit",
    "koordhip_commit_ext", "koordhip_uncommit_ext",
    "koordhip_fetch_cpusets", "koordhip_read_numa", "koordhip_read_numa_zones", "koordhip_read_reservations",
    "koordhip_read_resv_cpus", "koordhip_read_resv_devices", "koordhip_read_resv_scalars", "koordhip_last_stats", "koordhip_last_kernel_stats",
    "koordhip_set_profile_kernels", "koordhip_last_kernel_names",
    "koordhip_comm_unique_id", "koordhip_comm_init", "koordhip_comm_init_local",
]


def check(lib, rc: int):
    if rc != 0:
        raise KoordhipError(rc, (lib.koordhip_last_error() or b"").decode())
    return rc


def ptr(a: np.ndarray, ctype):
    return a.ctypes.data_as(C.POINTER(ctype)) if a is not None else None
