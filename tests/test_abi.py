"""The C-ABI library loads, exports every symbol include/koordhip.h declares,
and its structs have the byte layout the ctypes / numpy mirrors assume
(checked against gcc's own view of the header).  No GPU calls."""
import ctypes as C
import os
import re
import subprocess
import tempfile

import pytest

from koordinator_amd import abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "koordhip.h")


def declared_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"\b(koordhip_[a-z_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    lib = abi.load_library()
    names = declared_functions()
    assert len(names) >= 15
    for name in names:
        assert hasattr(lib, name), name
    assert sorted(abi.EXPORTED_SYMBOLS) == names
    assert lib.koordhip_abi_version() == abi.KOORDHIP_ABI_VERSION


def test_nm_exports():
    out = subprocess.run(["nm", "-D", "--defined-only", abi.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (koordhip_\w+)", out))
    assert set(declared_functions()) <= exported


PROBE = r"""
#include <stdio.h>
#include <stddef.h>
#include "koordhip.h"
int main(void) {
  printf("%zu %zu %zu %zu\n", sizeof(koordhip_config), sizeof(koordhip_node_soa), sizeof(koordhip_pod), sizeof(koordhip_topk));
  printf("%zu %zu %zu %zu\n", offsetof(koordhip_pod, est_mem), offsetof(koordhip_pod, flags), offsetof(koordhip_config, batch_pods), offsetof(koordhip_node_soa, la_flags));
  printf("%zu %zu\n", sizeof(koordhip_kernel_stats), offsetof(koordhip_kernel_stats, rounds));
  return 0;
}
"""


def test_struct_layout_matches_header():
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "p.c")
        exe = os.path.join(d, "p")
        open(src, "w").write(PROBE)
        subprocess.run(["gcc", "-std=c11", "-I", os.path.dirname(HEADER), src, "-o", exe], check=True)
        lines = subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split("\n")
    sizes = [int(x) for x in lines[0].split()]
    offs = [int(x) for x in lines[1].split()]
    assert sizes == [C.sizeof(abi.KoordhipConfig), C.sizeof(abi.KoordhipNodeSoa), abi.POD_DTYPE.itemsize,
                     C.sizeof(abi.KoordhipTopk)]
    assert offs[0] == abi.POD_DTYPE.fields["est_mem"][1]
    assert offs[1] == abi.POD_DTYPE.fields["flags"][1]
    assert offs[2] == abi.KoordhipConfig.batch_pods.offset
    assert offs[3] == abi.KoordhipNodeSoa.la_flags.offset
    ks = [int(x) for x in lines[2].split()]
    assert ks == [C.sizeof(abi.KoordhipKernelStats), abi.KoordhipKernelStats.rounds.offset]


def test_create_rejects_bad_config_without_gpu():
    """Argument validation happens before any device call (validation_pluginargs.go analogue)."""
    lib = abi.load_library()
    cfg = abi.KoordhipConfig()
    cfg.abi_version = 999
    ctx = C.c_void_p()
    assert lib.koordhip_create(C.byref(cfg), C.byref(ctx)) == -1
    assert b"abi_version" in lib.koordhip_last_error()
    cfg.abi_version = abi.KOORDHIP_ABI_VERSION
    cfg.score_plugins = abi.PLUGIN_LOADAWARE
    cfg.plugin_weight[1] = 0
    assert lib.koordhip_create(C.byref(cfg), C.byref(ctx)) == -1
    cfg.plugin_weight[1] = 1
    cfg.batch_pods = 65
    assert lib.koordhip_create(C.byref(cfg), C.byref(ctx)) == -1


def test_engine_requires_library(monkeypatch, tmp_path):
    monkeypatch.setattr(abi, "_lib", None)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        abi.load_library(str(tmp_path / "missing.so"))
