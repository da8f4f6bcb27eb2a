#!/bin/bash
# Chunk-size tuning on the current build: each "fit:pool:batch" of TUNE on one
# resident stream (sweep.py, pipelined timings).
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
for CFG in ${TUNE:-65536:8192:64}; do
  IFS=: read F P B <<< "$CFG"
  timeout -k 10 300 python3 tools/sweep.py --events ${EVENTS:-50000000} --pool $P --batch $B --fit $F --reps 2 \
     > gpurun_out/tune.log 2>&1
  rc=$?; echo "[$CFG] rc=$rc"; grep fit_chunk gpurun_out/tune.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
