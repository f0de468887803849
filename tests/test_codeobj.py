"""Guards on the built gfx950 code object (CPU; no GPU needed).

k_inc_stream hands L21 / L22 from producer workgroups to cell workgroups of
the same launch: it needs every producer resident
before the cells that wait for it, and code with no out-of-line calls -- the
compiler once outlined the producer (inc_produce) and the launch stalled for
seconds, surfacing only as MFGP_ERR_DEVICE after the bounded spin. These tests
read the library's code object (tools/check_codeobj.py) and fail if either
precondition is lost to a toolchain or inlining change: no call instruction in
the stream kernels, <= 128 VGPRs and <= 40 KB of LDS (four 256-thread
workgroups per CU), and no scratch beyond the few spill slots measured.

The lattice step (k_inc_lat / k_inc_lat_arg, mfgp_lattice.inl) rests on the same
residency: its roles wait only on roles dispatched before them, and with split-K
the splits of a tile wait for each other, which the host allows only while every
GEMM workgroup of the launch fits beside the rest (tiles x S <= 2 per CU of the
four). Its guard: call-free, <= 128 VGPR + AGPR, <= 40 KB LDS, scratch <= 256
bytes per lane (the measured spill slots: 80-180), and a forced-spill build
(MFGP_LAT_WAVES=8: a 64-VGPR budget) must fail that bound."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
STREAM = ("k_inc_stream", "k_vstream")
LATTICE = ("k_inc_lat",)
LAT_SCRATCH_MAX = 256


@pytest.fixture(scope="module")
def report():
    import __graft_entry__ as ge
    ge.build()
    import check_codeobj
    return check_codeobj.kernel_report(os.path.join(ROOT, "mfgp_coverage_amd", "libmfgp_hip.so"))


def _stream(rep):
    ks = {n: r for n, r in rep.items() if any(s in n for s in STREAM)}
    assert len(ks) == 8, sorted(rep)   # <double> and <float> of k_inc_stream, k_inc_stream1, k_inc_stream_arg, k_vstream
    return ks


def test_stream_kernels_have_no_calls(report):
    for n, r in _stream(report).items():
        assert r["calls"] == 0, (n, r)


def test_stream_kernels_fit_four_workgroups_per_cu(report):
    for n, r in _stream(report).items():
        assert r["vgpr"] + r["agpr"] <= 128, (n, r)
        assert r["lds"] <= 40 * 1024, (n, r)
        assert r["scratch"] <= 128, (n, r)


def test_every_kernel_is_call_free(report):
    for n, r in report.items():
        assert r["calls"] == 0, (n, r)


@pytest.fixture(scope="module")
def diag_report(tmp_path_factory):
    """One diagnostic build for both negative checks: the producer outlined
    (MFGP_NOINLINE_PRODUCE) and the lattice kernels squeezed to 64 VGPRs
    (MFGP_LAT_WAVES=8)."""
    import check_codeobj
    obj = tmp_path_factory.mktemp("diag") / "k.o"
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                    "-DMFGP_NOINLINE_PRODUCE", "-DMFGP_LAT_WAVES=8", "-c",
                    os.path.join(ROOT, "mfgp_coverage_amd", "csrc", "mfgp_kernels.hip"), "-o", str(obj)],
                   check=True, capture_output=True)
    return check_codeobj.kernel_report(str(obj))


def test_forced_outline_is_caught(diag_report):
    """The check fires on the failure it guards against: a build with the
    producer outlined (MFGP_NOINLINE_PRODUCE) has a call inside k_inc_stream."""
    inc = [r for n, r in diag_report.items() if "k_inc_stream" in n]
    assert inc and all(r["calls"] > 0 for r in inc), inc


def _lattice(rep):
    ks = {n: r for n, r in rep.items() if any(s in n for s in LATTICE)}
    # KA 8 / 16 x <double> / <float> x GEMM roles in the launch or not (k_lat_gemm2), of
    # k_inc_lat and k_inc_lat_arg
    assert len(ks) == 16, sorted(rep)
    return ks


def _lattice_ok(r):
    return (r["calls"] == 0 and r["vgpr"] + r["agpr"] <= 128 and r["lds"] <= 40 * 1024
            and r["scratch"] <= LAT_SCRATCH_MAX)


def test_lattice_kernels_fit_four_workgroups_per_cu(report):
    for n, r in _lattice(report).items():
        assert _lattice_ok(r), (n, r)


def test_forced_spill_lattice_build_is_caught(diag_report):
    """A lattice build squeezed to 64 VGPRs spills far past the scratch bound."""
    lat = _lattice(diag_report)
    assert all(not _lattice_ok(r) for r in lat.values()), lat


def test_lattice_gemm2_kernels_fit_one_workgroup_per_cu(report):
    """The lattice step's second launch (k_lat_gemm2, 1024-thread workgroups): no
    calls, <= 128 VGPRs (16 waves on a CU), its LDS within the CU's 160 KB, no spills."""
    ks = {n: r for n, r in report.items() if "k_lat_gemm2" in n}
    assert len(ks) == 8, sorted(report)
    for n, r in ks.items():
        assert r["calls"] == 0 and r["vgpr"] + r["agpr"] <= 128 and r["lds"] <= 160 * 1024, (n, r)
        assert r["scratch"] == 0 and r["vgpr_spill"] == 0, (n, r)


@pytest.fixture(scope="module")
def hand_offs(report):
    import check_codeobj
    return check_codeobj.hand_off_report(os.path.join(ROOT, "mfgp_coverage_amd", "libmfgp_hip.so"),
                                         ("k_inc_stream", "k_inc_lat"))


def test_hand_off_polls_read_device_scope_and_wait(hand_offs):
    """the hand-offs inside one launch carry no acquire (its L2
    invalidate costs 8 % at the headline); their order rests on the code
    the compiler emits, which this checks in every consumer kernel: each poll of a
    hand-off word (every spin iteration, found by its s_sleep) reads the word with a
    device-scope (sc1) load, and an s_waitcnt vmcnt(0) completes that load before
    the branch that leaves the spin -- so the flag's value is seen before anything
    after the wait is issued (no speculation), and a stale L2 line never serves it.
    The loads of the handed-off data are sc1 loads, or plain loads of lines no
    workgroup of that XCD read earlier in the launch."""
    assert len(hand_offs) == 22, sorted(hand_offs)   # 6 k_inc_stream*, 16 k_inc_lat*
    for name, its in hand_offs.items():
        # every consumer kernel waits (k_inc_stream*: L21 and L22; k_inc_lat*: more)
        assert len(its) >= 10 if "k_inc_stream" in name else len(its) >= 14, (name, len(its))
        for it in its:
            assert it["loads"] and it["sc1"], (name, it)
            assert it["waited"], (name, it)


def test_poll_check_catches_plain_and_unwaited_polls(report):
    """The poll check itself: in a real spin loop of k_inc_lat, a flag load without
    sc1 or a missing s_waitcnt vmcnt(0) before the loop's exit branch is reported."""
    import tempfile
    import check_codeobj
    with tempfile.TemporaryDirectory() as td:
        dis = check_codeobj.disassembly(check_codeobj.code_object(
            os.path.join(ROOT, "mfgp_coverage_amd", "libmfgp_hip.so"), td))
    name = next(n for n in dis if "k_inc_lat_arg" in n)
    ins = dis[name]
    its = check_codeobj.poll_iterations(ins)
    assert its and all(it["loads"] and it["sc1"] and it["waited"] for it in its)
    # the first spin's first load: drop its sc1; separately, drop the waits after it
    i = next(k for k, x in enumerate(ins) if x[1] == "s_sleep")
    first = check_codeobj.poll_iterations(ins[:i + 400])[0]
    assert first["loads"], first
    plain = [(a, op, args.replace(" sc1", ""), t) if op.startswith(check_codeobj.VMEM_LOAD) else (a, op, args, t)
             for a, op, args, t in ins]
    assert not check_codeobj.poll_iterations(plain)[0]["sc1"]
    unwaited = [(a, "s_nop", "0", t) if op == "s_waitcnt" and "vmcnt(0)" in args else (a, op, args, t)
                for a, op, args, t in ins]
    assert not check_codeobj.poll_iterations(unwaited)[0]["waited"]
