#!/bin/bash
# GPU session: the -m gpu tests only (each test under pytest-timeout), log to gpurun_out/.
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 ${TLIM:-900} python -u -m pytest ${TESTS:-tests} -x -v -m gpu --timeout 300 --timeout-method thread -rA \
    > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -40
exit $rc
