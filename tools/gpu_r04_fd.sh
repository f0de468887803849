#!/bin/bash
# round 4: factor group depth sweep (bit-equal across depths: test_two_level_factor_bit_equal)
set -e
mkdir -p gpurun_out
: > gpurun_out/fd_sweep.txt
for fd in 2 3 4 5 6 8 4 6; do
  echo "depth=$fd $(MFGP_FACTOR_DEPTH=$fd timeout -k 10 180 python tools/bench_factor.py --steps 10)" >> gpurun_out/fd_sweep.txt
done
cat gpurun_out/fd_sweep.txt
