#!/bin/bash
# Iteration loop: gpu parity tests, then sweep.py timings for each setting of
# AB_ENV (space-separated VAR=value entries; "-" = defaults) on one stream.
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
for V in ${AB_ENV:--}; do
  if [ "$V" = "-" ]; then E=""; else E="$V"; fi
  env $E timeout -k 10 300 python3 tools/sweep.py --events ${EVENTS:-50000000} --pool ${POOL:-16384} --batch ${BATCH:-16} \
      --fit ${FIT:-65536} --reps 2 > gpurun_out/ab.log 2>&1
  rc=$?; echo "[$V] rc=$rc"; grep fit_chunk gpurun_out/ab.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
