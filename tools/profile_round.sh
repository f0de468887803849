#!/bin/bash
# rocprofv3 evidence for one round: kernel trace + stats of the default bench,
# then counters in passes of their own (FETCH_SIZE; WRITE_SIZE; MFMA busy cycles).
# usage (on the GPU box): bash tools/profile_round.sh r01
set -e
TAG=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench -- \
  python3 $R/bench.py --steps 200 --warmup 20 --no-cpu-baseline > $OUT/trace.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/fetch -o bench -- \
  python3 $R/bench.py --steps 8 --warmup 2 --no-cpu-baseline > $OUT/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/write -o bench -- \
  python3 $R/bench.py --steps 8 --warmup 2 --no-cpu-baseline > $OUT/write.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace \
  --output-format csv -d $OUT/mfma -o bench -- \
  python3 $R/bench.py --steps 8 --warmup 2 --no-cpu-baseline > $OUT/mfma.log 2>&1 || echo "mfma pass failed"
echo done
