#!/bin/bash
# Round-5 session 12: host call times of a temporal-segment rank step (C4,
# N = 2, ranks 0 and 1) against N = 1.
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
L=gpurun_out/r05_segments_times.log
: > $L
timeout -k 10 300 python3 -u tools/strip_rank.py --config 4 --n 1 --split segments --reps 3 --host-times >> $L 2>&1 || exit 1
timeout -k 10 300 python3 -u tools/strip_rank.py --config 4 --n 2 --split segments --reps 3 --host-times >> $L 2>&1 || exit 2
exit 0
