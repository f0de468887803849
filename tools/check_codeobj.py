"""Resource and call report of the gfx950 kernels inside a hipcc-built shared
library or object (test infrastructure: tests/test_codeobj.py).

The fused append + stream kernel (k_inc_stream) relies on producers and cell
workgroups being resident together and on code with no out-of-line calls: an
outlined producer once stalled the hand-off for seconds.
This module extracts the code object (.hip_fatbin -> clang-offload-bundler),
reads the AMDGPU metadata note (VGPRs, spills, LDS) and counts call
instructions (s_swappc_b64) in each kernel's disassembly.

usage: python tools/check_codeobj.py mfgp_coverage_amd/libmfgp_hip.so
"""
from __future__ import annotations

import os
import re
import subprocess
import sys
import tempfile

import yaml

LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"


def code_object(path, workdir):
    fat = os.path.join(workdir, "fatbin.bin")
    co = os.path.join(workdir, "gfx950.co")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", path, os.path.join(workdir, "x")],
                   check=True, capture_output=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--targets={TARGET}",
                    f"--input={fat}", f"--output={co}"], check=True, capture_output=True)
    return co


def metadata(co):
    out = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True, text=True).stdout
    y = out[out.index("---"):]
    y = y[: y.index("\n...")] if "\n..." in y else y
    return yaml.safe_load(y)["amdhsa.kernels"]


def calls(co):
    """{kernel symbol: number of s_swappc_b64 in its body}."""
    dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", co], check=True, capture_output=True, text=True).stdout
    out, cur = {}, None
    for line in dis.splitlines():
        m = re.match(r"^[0-9a-f]+ <([^>]+)>:", line)
        if m:
            cur = m.group(1)
            out[cur] = 0
        elif cur and "s_swappc_b64" in line:
            out[cur] += 1
    return out


def kernel_report(path):
    with tempfile.TemporaryDirectory() as td:
        co = code_object(path, td)
        md = metadata(co)
        cl = calls(co)
    rep = {}
    for k in md:
        name = k[".name"]
        rep[name] = {"vgpr": k[".vgpr_count"], "agpr": k.get(".agpr_count", 0),
                     "vgpr_spill": k.get(".vgpr_spill_count", 0), "sgpr_spill": k.get(".sgpr_spill_count", 0),
                     "lds": k[".group_segment_fixed_size"], "scratch": k.get(".private_segment_fixed_size", 0),
                     "calls": cl.get(name, 0)}
    return rep


if __name__ == "__main__":
    for n, r in sorted(kernel_report(sys.argv[1]).items()):
        print(n, r)
