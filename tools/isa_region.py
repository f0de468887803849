"""Diagnostic: the disassembly of one kernel of a hipcc-built object or library
between its first and last non-temporal 16-byte load (the lattice step's F
stream), with the scratch accesses and vmcnt waits in it.

usage: python tools/isa_region.py build/k.o '<kernel symbol regex>' [out.s]
"""
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import check_codeobj as C  # noqa: E402


def kernel_asm(path, pat):
    with tempfile.TemporaryDirectory() as td:
        co = C.code_object(path, td)
        dis = subprocess.run([f"{C.LLVM}/llvm-objdump", "-d", "--symbolize-operands", co], check=True,
                             capture_output=True, text=True).stdout.split("\n")
    out, on = [], False
    for l in dis:
        m = re.match(r"^[0-9a-f]+ <([^>]+)>:", l)
        if m and not re.fullmatch(r"L\d+", m.group(1)):
            on = re.search(pat, m.group(1)) is not None
        if on:
            out.append(l)
    return out


if __name__ == "__main__":
    f = kernel_asm(sys.argv[1], sys.argv[2])
    nt = [i for i, l in enumerate(f) if "global_load_dwordx4" in l and " nt" in l]
    print(len(f), "lines;", len(nt), "nt dwordx4 loads at", nt[:4], "...", nt[-4:])
    if nt:
        seg = f[nt[0]:nt[-1] + 1]
        print("scratch ops in the region:", sum("scratch_" in l for l in seg))
        print("vmcnt waits:", [l.split("s_waitcnt")[1].strip() for l in seg if "s_waitcnt" in l and "vmcnt" in l])
        if len(sys.argv) > 3:
            open(sys.argv[3], "w").write("\n".join(f[max(0, nt[0] - 200):nt[-1] + 200]))
