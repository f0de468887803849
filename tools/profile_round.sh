#!/bin/bash
# rocprofv3 evidence for one round: kernel trace + stats of a bench run, then
# counters in passes of their own (FETCH_SIZE; WRITE_SIZE; MFMA busy cycles).
# usage (on the GPU box): bash tools/profile_round.sh r02 [extra bench.py args]
#   e.g. bash tools/profile_round.sh r02_configs4 --workload configs4
set -e
TAG=${1:-r01}
shift || true
EXTRA="$*"
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
case "$EXTRA" in *configs4*) TS="--steps 20 --warmup 3"; PS="--steps 8 --warmup 1";; *) TS="--steps 200 --warmup 20"; PS="--steps 8 --warmup 2";; esac
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench -- \
  python3 $R/bench.py $TS --no-cpu-baseline $EXTRA > $OUT/trace.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/fetch -o bench -- \
  python3 $R/bench.py $PS --no-cpu-baseline --no-full $EXTRA > $OUT/fetch.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/write -o bench -- \
  python3 $R/bench.py $PS --no-cpu-baseline --no-full $EXTRA > $OUT/write.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace \
  --output-format csv -d $OUT/mfma -o bench -- \
  python3 $R/bench.py $PS --no-cpu-baseline $EXTRA > $OUT/mfma.log 2>&1 || echo "mfma pass failed"
echo done
