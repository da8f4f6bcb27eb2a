#!/bin/bash
# x-strip checks on one box: the strip gpu tests, then gloo rehearsals of
# bench.py --gpus 2 (every rank on device 0) for the split modes.
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_strips.py tests/test_gpu_parity.py -v -m gpu -x -k "strips or host_path" --timeout 300 --timeout-method thread > gpurun_out/pytest_strips.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_strips.log
[ $rc -ne 0 ] && exit $rc
N=2 SPLITS="strips segments strips-recompute" REH_EVENTS=${REH_EVENTS:-5000000} bash tools/gpu_rehearse.sh
