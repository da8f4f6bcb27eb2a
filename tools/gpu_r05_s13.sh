#!/bin/bash
# Round-5 session 13: farms_last_stamps bucketed by pixel tile (no scattered
# atomics): the segment tests, then the C4 segment rank host times and the
# N = 8 simulation.
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_segments.py tests/test_multirank.py -m gpu -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/r05_pytest_s13.log 2>&1 || exit 1
L=gpurun_out/r05_segments_times2.log
: > $L
timeout -k 10 300 python3 -u tools/strip_rank.py --config 4 --n 2 --split segments --reps 3 --host-times >> $L 2>&1 || exit 2
L=gpurun_out/r05_segments_sim2.log
: > $L
for C in 3 4; do
  timeout -k 10 300 python3 -u tools/strip_rank.py --config $C --n 1 --split segments --reps 3 >> $L 2>&1 || exit 3
  timeout -k 10 600 python3 -u tools/strip_rank.py --config $C --n 8 --split segments --reps 2 >> $L 2>&1 || exit 4
done
exit 0
