#!/bin/bash
# Iteration loop: gpu parity tests, one bench line (no CPU baseline), and a
# serialized kernel-trace timeline of the same stream.
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log
[ $rc -ne 0 ] && exit $rc
if [ "${TIMELINE:-1}" = "1" ]; then
  FARMS_SERIALIZE=1 timeout -k 10 500 rocprofv3 --kernel-trace -d gpurun_out/kt -o kt --output-format csv -- \
     python3 tools/sweep.py --events ${EVENTS:-50000000} --pool ${POOL:-16384} --batch ${BATCH:-16} --fit ${FIT:-65536} --reps 1 \
     > gpurun_out/kt.log 2>&1
  rc=$?; echo "kernel-trace rc=$rc"; grep fit_chunk gpurun_out/kt.log
  [ $rc -ne 0 ] && exit $rc
  python3 tools/timeline.py gpurun_out/kt/kt_kernel_trace.csv
fi
