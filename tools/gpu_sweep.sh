#!/bin/bash
# GPU session: parity tests, then a chunk-size sweep on config 3 (tuning aid).
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -q -m gpu -rA > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 800 python tools/sweep.py ${SWEEP_ARGS:---pool 8192,16384,32768,65536} > gpurun_out/sweep.log 2>&1
rc=$?
echo "sweep rc=$rc"; grep fit_chunk gpurun_out/sweep.log
exit $rc
