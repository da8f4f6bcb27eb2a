#!/bin/bash
# GPU session: parity tests, then a bench line, then a rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; a crash/abort/timeout stops the script.
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
EVENTS=${EVENTS:-50000000}
timeout -k 10 900 python -m pytest tests -q -m gpu -rA > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --events $EVENTS --steps 3 --warmup 1 > gpurun_out/bench.log 2>&1
rc=$?
echo "bench rc=$rc"; tail -1 gpurun_out/bench.log
if [ $rc -ne 0 ]; then exit $rc; fi
if [ "${PROFILE:-1}" = "1" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
      python3 bench.py --events $EVENTS --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1
  rc=$?
  echo "rocprof rc=$rc"; tail -1 gpurun_out/prof.log
fi
exit $rc
