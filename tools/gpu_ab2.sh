#!/bin/bash
# A/B of library builds: gpu parity tests on the default build, then sweep.py
# timings for each library in AB_LIBS (paths relative to the package; "-" =
# the default build) and each fit chunk in FIT, on one resident stream.
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 300 > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
  [ $rc -ne 0 ] && exit $rc
fi
for L in ${AB_LIBS:--}; do
  if [ "$L" = "-" ]; then unset FARMS_HIP_LIB; else export FARMS_HIP_LIB=$L; fi
  timeout -k 10 300 python3 tools/sweep.py --events ${EVENTS:-50000000} --pool ${POOL:-8192} --batch ${BATCH:-64} \
      --fit ${FIT:-65536} --reps 2 > gpurun_out/ab.log 2>&1
  rc=$?; echo "[$L] rc=$rc"; grep fit_chunk gpurun_out/ab.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
