#!/bin/bash
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu -rA > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --events 5000000 --steps 2 --warmup 1 --cpu-sample 100000 > gpurun_out/bench_small.log 2>&1
rc=$?
echo "bench rc=$rc"
tail -3 gpurun_out/bench_small.log
exit $rc
