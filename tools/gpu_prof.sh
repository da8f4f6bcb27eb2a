#!/bin/bash
# GPU session: serialized kernel-trace statistics (kernel durations without
# stream overlap) and one PMC group, on the sweep driver.
#   POOL / BATCH / FIT: chunking;  EVENTS: stream length;  PMC_SET: see gpu_pmc.sh
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
EV=${EVENTS:-50000000}
ARGS="--events $EV --pool ${POOL:-16384} --batch ${BATCH:-16} --fit ${FIT:-262144} --reps 1"
FARMS_SERIALIZE=1 timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/kt -o kt --output-format csv -- \
   python3 tools/sweep.py $ARGS > gpurun_out/kt.log 2>&1
rc=$?; echo "kernel-trace rc=$rc"; grep fit_chunk gpurun_out/kt.log
[ $rc -ne 0 ] && exit $rc
if [ -n "${PMC_SET:-}" ]; then
  FARMS_SERIALIZE=1 POOL=${POOL:-16384} BATCH=${BATCH:-16} EVENTS=${PMC_EVENTS:-10000000} bash tools/gpu_pmc.sh
  rc=$?
fi
exit $rc
