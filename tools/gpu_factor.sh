#!/bin/bash
# GPU pass for the fused factor step (k_fstep): parity tests, the A/B timing of
# tools/bench_factor.py (default library, then the variants given as arguments),
# and a rocprofv3 kernel-trace summary of the default run. Each step bounded;
# stop at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/factor
timeout -k 10 400 python -u -m pytest tests/test_gpu_factor.py -x -v --timeout 240 --timeout-method thread \
  > gpurun_out/factor/tests.log 2>&1 || { echo "factor tests failed"; tail -30 gpurun_out/factor/tests.log; exit 1; }
tail -3 gpurun_out/factor/tests.log
timeout -k 10 240 python -u tools/bench_factor.py > gpurun_out/factor/default.json 2> gpurun_out/factor/default.err \
  || { echo "bench_factor failed"; tail -20 gpurun_out/factor/default.err; exit 1; }
cat gpurun_out/factor/default.json
for v in "$@"; do
  MFGP_LIB=$R/$v timeout -k 10 240 python -u tools/bench_factor.py > gpurun_out/factor/$(basename $v).json \
    2> gpurun_out/factor/$(basename $v).err || { echo "variant $v failed"; tail -20 gpurun_out/factor/$(basename $v).err; exit 1; }
  echo "$v: $(cat gpurun_out/factor/$(basename $v).json)"
done
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/bench_nlml.py > gpurun_out/factor/nlml.json 2>&1 && cat gpurun_out/factor/nlml.json || { echo nlml failed; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/factor/prof -o factor -- \
  python3 $R/tools/bench_factor.py --steps 5 > gpurun_out/factor/prof.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/factor/prof.log; exit 1; }
find gpurun_out/factor/prof -name "*kernel_stats.csv" -exec head -12 {} \;
