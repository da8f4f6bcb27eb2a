#!/bin/bash
# Iteration: gpu parity tests (default build), then for each library in AB_LIBS
# ("-" = default build): a serialized kernel-trace timeline (one stream, kernel
# durations without overlap) and a pipelined sweep.py timing.
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 300 > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
  [ $rc -ne 0 ] && exit $rc
fi
i=0
for L in ${AB_LIBS:--}; do
  if [ "$L" = "-" ]; then unset FARMS_HIP_LIB; else export FARMS_HIP_LIB=$L; fi
  if [ "${TIMELINE:-1}" = "1" ]; then
    FARMS_SERIALIZE=1 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tl_$i -o kt --output-format csv -- \
       python3 tools/sweep.py --events ${EVENTS:-50000000} --pool ${POOL:-8192} --batch ${BATCH:-64} --fit ${FIT:-65536} --reps 1 \
       > gpurun_out/tl_$i.log 2>&1
    rc=$?; echo "[$L] timeline rc=$rc"
    [ $rc -ne 0 ] && exit $rc
    python3 tools/timeline.py gpurun_out/tl_$i/kt_kernel_trace.csv | grep -E "span|k_pool|k_fit|k_chain"
  fi
  timeout -k 10 300 python3 tools/sweep.py --events ${EVENTS:-50000000} --pool ${POOL:-8192} --batch ${BATCH:-64} \
      --fit ${FIT:-65536} --reps 2 > gpurun_out/ab_$i.log 2>&1
  rc=$?; echo "[$L] sweep rc=$rc"; grep fit_chunk gpurun_out/ab_$i.log
  [ $rc -ne 0 ] && exit $rc
  i=$((i+1))
done
exit 0
