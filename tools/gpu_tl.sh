#!/bin/bash
# Serialized kernel-trace timelines (FARMS_SERIALIZE=1: one stream, kernel
# durations without overlap) for each "pool:batch:fit" entry of TL_CFG.
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
for CFG in ${TL_CFG:-16384:16:65536}; do
  IFS=: read P B F <<< "$CFG"
  FARMS_SERIALIZE=1 timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/tl_$P_$B -o kt --output-format csv -- \
     python3 tools/sweep.py --events ${EVENTS:-50000000} --pool $P --batch $B --fit $F --reps 1 > gpurun_out/tl.log 2>&1
  rc=$?; echo "[$CFG] kernel-trace rc=$rc"; grep fit_chunk gpurun_out/tl.log
  [ $rc -ne 0 ] && exit $rc
  python3 tools/timeline.py gpurun_out/tl_$P_$B/kt_kernel_trace.csv | grep -E "span|k_"
done
