#!/bin/bash
# Sub-batches of the pipelined strip step (multirank.Stepper nsub): rank 3 of 8 at C3.
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
for S in ${NSUBS:-2 4 16}; do
  timeout -k 10 300 python3 -u tools/strip_rank.py --split strips --n 8 --ranks 3 --nsub $S \
    > gpurun_out/strip_nsub_$S.log 2>&1 || exit $?
  tail -1 gpurun_out/strip_nsub_$S.log
done
exit 0
