"""Every read of a hand-off buffer in the kernel sources is an sc1 read or an
audited first access. CPU only.

Inside one launch the producers, w units, Z units, scan units and the finish hand
data to other workgroups through write-through (sc1) stores, a drain and a flag,
with no acquire. A consumer may then read the data either with a device-scope
(sc1) load, which no stale L2 / L1 line can serve, or with a plain load of a line
that no workgroup of its XCD read earlier in the launch (L2 and L1 are invalidated
at the kernel boundary and never filled since), i.e. the first access to it.
tests/test_codeobj.py checks the polls in the code object; this test checks the
loads after them in the source: it lists every line of mfgp_lattice.inl and
mfgp_kernels.hip that names a hand-off buffer -- a GPDesc field below or a local
pointer derived from one -- and classifies it as a store, a pointer derivation,
an sc1 read (or a poll), or a plain read. Each plain read must be one of the
audited sites in PLAIN, with the reason it is a first access (or is not a hand-off
within the launch at all: k_lat_gemm2 reads what the previous launch wrote). A new
plain read of a hand-off buffer fails here until it is audited and listed."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "mfgp_coverage_amd", "csrc")
# buffers written in a launch and read by other workgroups of the same launch
FIELDS = ("l21c", "l22r", "iscr", "wpart", "wv", "zb", "csr", "zvl",
          "pflag", "wflag", "zflag", "sync", "ldone", "wcnt")
SC1 = ("ldx<true>", "ldx<FUSED>", "ldx<XW>", "__hip_atomic_load", "l21c_ld<", "ldu(", "wait_flag(",
       "wait_flags_all(", "spin_wave(", "wait_l21(", "wait_l21_from(", "wait_phase(", "__hip_atomic_fetch_add",
       "atomicMin(")
STORE = ("stx<", "st16_wt(", "__hip_atomic_store(", "publish(", "store_l21c<", "arrive_phase(", "st_u(", "st_i(")
# (file, code snippet) -> why the plain read is a first access (or no hand-off)
PLAIN = {
    ("mfgp_lattice.inl", ": reinterpret_cast<const VT*>(l21c) + (a < k ? a : 0);"):
        "w unit: a pointer into the compact rows; load_a reads through it with __hip_atomic_load (sc1)",
    ("mfgp_lattice.inl", "const __amdgpu_buffer_rsrc_t rZ = make_rsrc(d.zb, (int64_t)8 * P * zrows * tabw * KA);"):
        "GEMM tiles: the Z rows' DMA, each stage issued only after the Z unit that stores it raised its flag; "
        "no workgroup of the XCD reads those rows earlier in the launch (k_lat_gemm2: written by the previous launch)",
    ("mfgp_lattice.inl", "lat_scan(d, (int)role, sm, d.zflag + d.nzu + role);"):
        "the scan unit's own flag: lat_scan stores it (write-through, after its lists are drained)",
    ("mfgp_lattice.inl", "L22[e] = use ? d.l22r[e] : 0.0;"):
        "k_lat_gemm2: the L22 record of the previous launch (kernel boundary)",
    ("mfgp_lattice.inl", "for (int pt = 0; pt < P; ++pt) nvs[pt] = (d.zvl[pt * (zrows + 1)] + ZKS - 1) / ZKS;"):
        "k_lat_gemm2: the virtual-row lists of the previous launch (kernel boundary)",
    ("mfgp_lattice.inl", "const int64_t j = (lane >> 5) ? vl[1] : vl[0];"):
        "k_lat_gemm2: the virtual-row lists of the previous launch (kernel boundary)",
    ("mfgp_kernels.hip", "if (ra < k && cb <= ra) v = d.l21c_ok ? d.l22r[e] : d.A[(n0 + cb) * ld + n0 + ra];"):
        "V-stream cells: the L22 record after sync[2]; no line of it is read in the launch before that flag",
    ("mfgp_kernels.hip", "v = d.l21c_ok ? d.l22r[e] : d.zv[n0 + e - KINC * KINC];"):
        "V-stream cells: the L22 record after sync[2] (as above)",
    ("mfgp_kernels.hip", "WsPrefetch pf{(FUSED && mma) ? d.sync + 2 : nullptr, d.epoch, d.l22r, 0u, 0.0, 0.0, false};"):
        "ws_prefetch polls sync[2] with __hip_atomic_load and reads the L22 record only once it holds the epoch",
    ("mfgp_kernels.hip", "const WsSrc<2> src{vb, gp(d.l21c) + r, KINC, nullptr, j_hi, j_lo};"):
        "V stream (fp64): the compact rows, streamed after wait_l21 saw every producer chunk's flag; "
        "nothing reads them in the launch before",
    ("mfgp_kernels.hip", "const WfSrc src{vb, reinterpret_cast<const GLOBAL float*>(gp(d.l21c)) + r, nullptr, 0, nullptr, n0};"):
        "V stream (fp32): the compact rows after wait_l21 (as above)",
    ("mfgp_kernels.hip", "const double v = d.l22r[e];"):
        "V-stream epilogue: the L22 record after its sync[2] wait; no line of it is read earlier in the launch",
}


def _strip(line):
    return line.split("//")[0].rstrip()


def classify(path):
    """Yield (line number, kind, code) for every line naming a hand-off buffer;
    kind: decl / store / sc1 / plain. Local pointers derived from a buffer
    (p = d.field + ..., q = p + ...) are tracked within their function."""
    depth, alias = 0, set()
    field_re = re.compile(r"(?<![\w.])d\.(%s)\b" % "|".join(FIELDS))
    decl_re = re.compile(r"(?:const\s+)?[\w:]+(?:<[^>]*>)?\s*\*\s*(?:const\s+)?(?:__restrict__\s+)?(\w+)\s*=\s*(.+);")
    for no, raw in enumerate(open(path), 1):
        line = _strip(raw)
        if depth == 0:
            alias = set()
        names = [m.group(0) for m in field_re.finditer(line)]
        names += [a for a in alias if re.search(r"(?<![\w.])%s\b" % re.escape(a), line)]
        dm = decl_re.search(line)
        if dm:
            names = [n for n in names if n != dm.group(1)]   # (the declared name itself)
            if not names:
                alias.discard(dm.group(1))   # a new local of that name (shadowing)
        if names:
            deref = any(re.search(r"(?<![\w.])%s\s*\[" % re.escape(n), line) for n in names)
            if any(s in line for s in SC1):
                kind = "sc1"
            elif any(s in line for s in STORE):
                kind = "store"
            elif dm and not deref and "?" not in dm.group(2):
                kind = "decl"
                alias.add(dm.group(1))
            else:
                kind = "plain"
            yield no, kind, line.strip()
        depth += line.count("{") - line.count("}")


def _sites():
    out = []
    for f in ("mfgp_lattice.inl", "mfgp_kernels.hip"):
        for no, kind, code in classify(os.path.join(CSRC, f)):
            out.append((f, no, kind, code))
    return out


def test_every_plain_read_of_a_hand_off_buffer_is_audited():
    plain = [(f, no, code) for f, no, kind, code in _sites() if kind == "plain"]
    unaudited = [(f, no, code) for f, no, code in plain if (f, code) not in PLAIN]
    assert not unaudited, "plain reads of hand-off buffers that are not audited first accesses:\n" + \
        "\n".join(f"{f}:{no}: {c}" for f, no, c in unaudited)


def test_audit_list_is_current():
    """Every audited site still exists (a stale entry would hide nothing, but it
    means the audit no longer describes the code)."""
    present = {(f, code) for f, _, kind, code in _sites() if kind == "plain"}
    stale = [k for k in PLAIN if k not in present]
    assert not stale, stale


def test_consumers_read_hand_offs_through_sc1():
    """The bulk of the hand-off reads are sc1: the w units' partials and blocks,
    the Z units' w rows and member lists, the finish's chunk partials, the
    producers' flags -- and the scan sees them (a guard on the scanner itself)."""
    sites = _sites()
    sc1 = [(f, code) for f, _, kind, code in sites if kind == "sc1"]
    assert len(sc1) >= 20, len(sc1)
    for needle in ("ldx<true>(p0p", "ldx<true>(&wv[", "ldx<FUSED>(d.iscr", "ldx<true>(d.l22r"):
        assert any(needle in code for _, code in sc1), needle


def test_scanner_flags_a_plain_read(tmp_path):
    """The scanner itself: a plain read through a derived pointer is caught, an sc1
    read and a store through it are not."""
    src = tmp_path / "k.hip"
    src.write_text("__device__ void f(const GPDesc& d, int j) {\n"
                   "  const double* const wv = d.wv + 64;\n"
                   "  double a = ldx<true>(&wv[j]);\n"
                   "  stx<true>(d.wpart + j, a);\n"
                   "  double b = wv[j];\n"
                   "}\n")
    kinds = [(no, kind) for no, kind, _ in classify(str(src))]
    assert kinds == [(2, "decl"), (3, "sc1"), (4, "store"), (5, "plain")], kinds
