"""The kernarg layout karg.hpp assumes (CPU check of the built code object).

k_eval_topk re-reads DevCfg at kernarg offset 0 and DevNodes right after it
(koordinator_amd/csrc/karg.hpp).  The offsets follow the explicit argument
order; this reads the gfx950 code object's metadata out of libkoordhip.so and
checks every k_eval_topk instantiation against that assumption, so a change
to either struct or to the kernel's parameter list fails here, not on the GPU.
"""
import os
import re
import shutil
import subprocess
import tempfile

import pytest

from koordinator_amd import abi

LLVM = "/opt/rocm/lib/llvm/bin"


def _tool(name):
    p = os.path.join(LLVM, name)
    return p if os.path.exists(p) else shutil.which(name)


@pytest.mark.skipif(not (os.path.exists(abi.LIB_PATH) and _tool("llvm-objcopy") and _tool("clang-offload-bundler")
                         and _tool("llvm-readelf")), reason="needs the built library and the ROCm LLVM tools")
def test_eval_topk_kernarg_offsets():
    with tempfile.TemporaryDirectory() as d:
        fb, co, tmp = os.path.join(d, "fb.bin"), os.path.join(d, "co.o"), os.path.join(d, "tmp.so")
        subprocess.run([_tool("llvm-objcopy"), "--dump-section", f".hip_fatbin={fb}", abi.LIB_PATH, tmp], check=True)
        subprocess.run([_tool("clang-offload-bundler"), "--type=o", f"--input={fb}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}", "--unbundle"], check=True)
        notes = subprocess.run([_tool("llvm-readelf"), "--notes", co], check=True, capture_output=True,
                               text=True).stdout
    seen = 0
    for m in re.finditer(r"\.name:\s+(_ZN2kh11k_eval_topk\w+)", notes):
        blk = notes[notes.rfind("- .agpr_count", 0, m.start()):m.start()]
        args = [(int(o), int(z)) for o, z in re.findall(r"\.offset:\s+(\d+)\s+\.size:\s+(\d+)", blk)]
        cfg, nodes = args[0], args[1]
        assert cfg[0] == 0, m.group(1)
        assert nodes[0] == cfg[1], (m.group(1), args[:3])  # KARG_NODES = sizeof(DevCfg)
        seen += 1
    assert seen >= 18  # every (NM, VT, R, G) instantiation launch_eval_topk dispatches
