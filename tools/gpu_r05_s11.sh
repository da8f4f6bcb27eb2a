#!/bin/bash
# Round-5 session 11: the asynchronous exchange order bitwise at the engine
# level; then temporal segments (the default N>1 split), rank-simulated on one
# GPU at C3 and C4 for N = 2, 4, 8 (every rank), against N = 1.
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -k async_exchange -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/r05_pytest_s11.log 2>&1 || exit 1
L=gpurun_out/r05_segments_sim.log
: > $L
for C in 3 4; do
  timeout -k 10 300 python3 -u tools/strip_rank.py --config $C --n 1 --split segments --reps 3 >> $L 2>&1 || exit 2
  for N in 2 4 8; do
    timeout -k 10 600 python3 -u tools/strip_rank.py --config $C --n $N --split segments --reps 2 >> $L 2>&1 || exit 3
  done
done
exit 0
