#!/bin/bash
# Round-5 session 14: kernel durations of a segment rank's step (C4, N = 2,
# rank 1) under rocprofv3 --kernel-trace --stats.
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_seg -o kt --output-format csv -- \
  python3 -u tools/strip_rank.py --config 4 --n 2 --ranks 1 --split segments --reps 2 > gpurun_out/r05_seg_prof.log 2>&1 || exit 1
cp gpurun_out/kt_seg/kt_kernel_stats.csv gpurun_out/r05_seg_kernel_stats.csv
rm -rf gpurun_out/kt_seg
exit 0
