#!/bin/bash
# Round profile (tools/profile_round.sh), then a 2-rank rehearsal of the N>1 bench
# path on one GPU (gloo; both ranks share the card), each step bounded.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/profile_round.sh ${1:-r01} || exit 1
MFGP_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 50 --warmup 10 --no-cpu-baseline --no-full \
  > gpurun_out/rehearse2.json 2> gpurun_out/rehearse2.err || { echo "rehearsal failed"; tail -20 gpurun_out/rehearse2.err; exit 1; }
tail -1 gpurun_out/rehearse2.json
