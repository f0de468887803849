#!/bin/bash
# One parameterised GPU-box runner (replaces the round-4 one-off gpu_r04_*.sh scripts).
# usage (inside gpurun): bash tools/gpu_run.sh TAG step [step ...]
# steps:
#   tests[=PATTERN]   pytest -m gpu (optionally -k PATTERN) -> gpurun_out/TAG_tests.log
#   smoke             __graft_entry__.smoke()
#   bench             bench.py (defaults: 200 steps)             -> gpurun_out/TAG_bench.json
#   bench20           bench.py --steps 20 --warmup 5 (the driver's) -> gpurun_out/TAG_bench20.json
#   quick             bench.py 200 steps, GP leg only             -> gpurun_out/TAG_quick.json
#   configs4          bench.py --workload configs4                -> gpurun_out/TAG_configs4.json
#   dropin            tools/bench_dropin.py, 4 env settings        -> gpurun_out/TAG_dropin.jsonl
#   choi              tools/bench_planner.py --batch 8            -> gpurun_out/TAG_choi.json
#   profile           tools/profile_round.sh TAG                  -> gpurun_out/prof_TAG
#   trace=LIB         tools/trace_dump.py LIB                     -> gpurun_out/TAG_trace.npz
#   py=SCRIPT         python -u SCRIPT                            -> gpurun_out/TAG_py.log
# Every GPU step runs under its own time limit; the first failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out
TAG=$1
shift
O=gpurun_out/$TAG
run() {   # run LIMIT LOG CMD...: fail loudly
  local lim=$1 log=$2
  shift 2
  echo "== $(date +%T) $*"
  timeout -k 10 "$lim" "$@" > "$log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then
    echo "FAILED rc=$rc: $*"
    tail -25 "$log"
    exit $rc
  fi
}
for step in "$@"; do
  case "$step" in
    tests) run 1500 ${O}_tests.log python -u -m pytest -v --timeout 600 --timeout-method thread -m gpu tests/
           tail -3 ${O}_tests.log ;;
    tests=*) K="${step#tests=}"; K="${K//_or_/ or }"   # tests=a_or_b -> -k "a or b"
           run 1200 ${O}_tests.log python -u -m pytest -v --timeout 600 --timeout-method thread -m gpu tests/ -k "$K"
           tail -3 ${O}_tests.log ;;
    smoke) run 300 ${O}_smoke.log python -c "import __graft_entry__ as g; g.smoke()"; tail -1 ${O}_smoke.log ;;
    bench) run 400 ${O}_bench.log python -u bench.py
           grep '^{' ${O}_bench.log > ${O}_bench.json ;;
    bench20) run 300 ${O}_bench20.log python -u bench.py --steps 20 --warmup 5
           grep '^{' ${O}_bench20.log > ${O}_bench20.json ;;
    quick) run 300 ${O}_quick.log python -u bench.py --steps 200 --warmup 20 --no-full --no-cpu-baseline --sim-iterations 0
           grep '^{' ${O}_quick.log > ${O}_quick.json ;;
    configs4) run 600 ${O}_configs4.log python -u bench.py --workload configs4
           grep '^{' ${O}_configs4.log > ${O}_configs4.json ;;
    dropin) : > ${O}_dropin.jsonl   # default, then without the early return, then the V stream
           for v in "MFGP_EARLY_PD=1" "MFGP_EARLY_PD=0" "MFGP_LATTICE=0" "MFGP_EARLY_PD=1"; do
             run 200 ${O}_dropin.log env $v python -u tools/bench_dropin.py
             grep '^{' ${O}_dropin.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); d['env']='$v'; print(json.dumps(d))" >> ${O}_dropin.jsonl
           done
           cat ${O}_dropin.jsonl ;;
    choi) run 300 ${O}_choi.log python -u tools/bench_planner.py --batch 8
           grep '^{' ${O}_choi.log > ${O}_choi.json; cat ${O}_choi.json ;;
    profile) run 1100 ${O}_prof.log bash tools/profile_round.sh "$TAG" ;;
    trace=*) run 200 ${O}_trace.log python -u tools/trace_dump.py "${step#trace=}" ${O}_trace.npz ;;
    py=*) run 300 ${O}_py.log python -u "${step#py=}" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  echo "== $(date +%T) done $step"
done
python3 - "$O" <<'EOF'
import glob, json, sys
for f in sorted(glob.glob(sys.argv[1] + "_*.json")):
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            print(f, round(d["value"]), round(1e3 * d["ms_per_step"], 2), d.get("roofline", {}).get("frac"))
EOF
exit 0
