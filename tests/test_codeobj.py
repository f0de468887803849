"""Guards on the built gfx950 code object (CPU; no GPU needed).

k_inc_stream hands L21 / L22 from producer workgroups to cell workgroups of
the same launch: it needs every producer resident
before the cells that wait for it, and code with no out-of-line calls -- the
compiler once outlined the producer (inc_produce) and the launch stalled for
seconds, surfacing only as MFGP_ERR_DEVICE after the bounded spin. These tests
read the library's code object (tools/check_codeobj.py) and fail if either
precondition is lost to a toolchain or inlining change: no call instruction in
the stream kernels, <= 128 VGPRs and <= 40 KB of LDS (four 256-thread
workgroups per CU), and no scratch beyond the few spill slots measured."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
STREAM = ("k_inc_stream", "k_vstream")


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


def test_forced_outline_is_caught(tmp_path):
    """The check fires on the failure it guards against: a build with the
    producer outlined (MFGP_NOINLINE_PRODUCE) has a call inside k_inc_stream."""
    import check_codeobj
    obj = tmp_path / "k.o"
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                    "-DMFGP_NOINLINE_PRODUCE", "-c", os.path.join(ROOT, "mfgp_coverage_amd", "csrc", "mfgp_kernels.hip"),
                    "-o", str(obj)], check=True, capture_output=True)
    rep = check_codeobj.kernel_report(str(obj))
    inc = [r for n, r in rep.items() if "k_inc_stream" in n]
    assert inc and all(r["calls"] > 0 for r in inc), inc
