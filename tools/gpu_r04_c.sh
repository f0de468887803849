#!/bin/bash
# round-4: coverage tests + driver-style and long bench runs
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_coverage.py > gpurun_out/r04c_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r04c_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r04c_bench20.json 2> gpurun_out/r04c_bench20.err || exit $?
timeout -k 10 600 python -u bench.py --no-cpu-baseline --sim-iterations 0 > gpurun_out/r04c_bench200.json 2> gpurun_out/r04c_bench200.err || exit $?
python - <<'PY'
import json
for f in ("r04c_bench20", "r04c_bench200"):
    d = json.load(open(f"gpurun_out/{f}.json"))
    print(f, d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"], d.get("extra_warmup_steps"))
    if "simulation" in d:
        print(json.dumps(d["simulation"]))
PY
# A/B: the w units gather L21 from V themselves at B = 8 (default: only one GP)
MFGP_LAT_SELFG=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-full --sim-iterations 0 --diagnostic > gpurun_out/r04c_selfg1.json 2> gpurun_out/r04c_selfg1.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/r04c_selfg1.json'));print('selfg1', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
timeout -k 10 120 python -u tools/dropin_r04.py > gpurun_out/r04c_dropin.json 2>/dev/null || exit $?
timeout -k 10 120 python -u tools/dropin_r04.py --timing > gpurun_out/r04c_dropin_t.json 2>/dev/null || exit $?
cat gpurun_out/r04c_dropin.json gpurun_out/r04c_dropin_t.json
