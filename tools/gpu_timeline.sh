#!/bin/bash
# GPU session: pipelined kernel trace of one sweep configuration + timeline summary.
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS="--events ${EVENTS:-50000000} --pool ${POOL:-16384} --batch ${BATCH:-16} --fit ${FIT:-65536} --reps 1"
timeout -k 10 500 rocprofv3 --kernel-trace -d gpurun_out/tl -o tl --output-format csv -- \
   python3 tools/sweep.py $ARGS > gpurun_out/tl.log 2>&1
rc=$?; echo "kernel-trace rc=$rc"; grep fit_chunk gpurun_out/tl.log
[ $rc -ne 0 ] && exit $rc
python3 tools/timeline.py gpurun_out/tl/tl_kernel_trace.csv
