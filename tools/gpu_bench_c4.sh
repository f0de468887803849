#!/bin/bash
# GPU box: the N>1 launch rehearsal (gloo, two ranks on the one GPU) and the
# BASELINE configs[4] fp32 bench line. Each step bounded; stop at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
MFGP_DIST_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --steps 16 --warmup 2 --no-full --no-cpu-baseline \
  > gpurun_out/bench_gpus2_gloo.json 2> gpurun_out/bench_gpus2_gloo.err || { echo "gpus2 failed"; tail -20 gpurun_out/bench_gpus2_gloo.err; exit 1; }
cat gpurun_out/bench_gpus2_gloo.json
timeout -k 10 600 python -u bench.py --workload configs4 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || { echo "configs4 failed"; tail -30 gpurun_out/bench_c4.err; exit 1; }
cat gpurun_out/bench_c4.json
timeout -k 10 300 python -u bench.py --no-full --no-cpu-baseline > gpurun_out/bench_headline_quick.json 2> gpurun_out/bench_headline_quick.err || { echo "headline failed"; tail -30 gpurun_out/bench_headline_quick.err; exit 1; }
cat gpurun_out/bench_headline_quick.json
