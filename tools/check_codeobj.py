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


def disassembly(co):
    """{kernel symbol: [(address, mnemonic, operands, branch target address or None)]}."""
    dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co], check=True, capture_output=True,
                         text=True).stdout
    out, cur, base = {}, None, 0
    for line in dis.splitlines():
        m = re.match(r"^([0-9a-f]+) <([^>]+)>:", line)
        if m:
            cur, base = out.setdefault(m.group(2), []), int(m.group(1), 16)
            continue
        m = re.match(r"^\s+([a-z_0-9]+)\s*(.*?)\s*//\s*([0-9A-Fa-f]+):", line)
        if cur is not None and m:
            t = re.search(r"<[^+>]+\+0x([0-9a-f]+)>", line)
            cur.append((int(m.group(3), 16), m.group(1), m.group(2), base + int(t.group(1), 16) if t else None))
    return out


VMEM_LOAD = ("global_load", "buffer_load", "flat_load")


def poll_iterations(ins):
    """The hand-off waits' poll iterations of one kernel. Every bounded spin sleeps
    (s_sleep) between polls, so each s_sleep marks one spin loop: the instructions
    from the target of the first branch after the s_sleep that jumps back to it or
    above (the loop's back edge; the compiler may put the bound's test on it) up to
    that branch. Returns one record per s_sleep: the loop's vector loads (its polls
    of the hand-off words); whether all carry sc1 (device scope, L2-coherent across
    the XCDs: a flag is never served from a stale line); and whether every one of
    them is followed by an s_waitcnt vmcnt(0) before the next conditional branch
    (the branch reads the flag's value, so nothing after the exit is issued before
    the flag was seen)."""
    at = {a: i for i, (a, _, _, _) in enumerate(ins)}
    out = []
    for i, (addr, op, _, _) in enumerate(ins):
        if op != "s_sleep":
            continue
        head = br = None
        for j in range(i + 1, min(len(ins), i + 400)):
            _, op2, _, tgt = ins[j]
            if op2.startswith(("s_branch", "s_cbranch")) and tgt is not None and tgt <= addr and tgt in at:
                head, br = at[tgt], j
                break
        body = ins[head:br + 1] if head is not None else []
        loads, waited, pending = [], True, False
        for _, op2, args, _ in body:
            if op2.startswith(VMEM_LOAD):
                loads.append((op2, args))
                pending = True
            elif op2 == "s_waitcnt" and "vmcnt(0)" in args:
                pending = False
            elif op2.startswith("s_cbranch") and pending:
                waited = False
        out.append({"loads": loads, "sc1": bool(loads) and all(re.search(r"\bsc1\b", a) for _, a in loads),
                    "waited": waited and bool(loads)})
    return out


def hand_off_report(path, names):
    """{kernel: poll iterations} for the kernels whose symbol contains one of `names`."""
    with tempfile.TemporaryDirectory() as td:
        dis = disassembly(code_object(path, td))
    return {k: poll_iterations(v) for k, v in dis.items() if any(n in k for n in names)}


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
