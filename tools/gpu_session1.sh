#!/bin/bash
# Round session: gpu parity tests, PMC traffic passes of the bench workload
# (installed as profiles/rNN_traffic_c3.json on the box so the bench line
# carries roofline.traffic), the bench line, and the kernel-trace statistics.
# Stops at the first failure.
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
ROUND=${ROUND:-r01}
timeout -k 10 900 python -m pytest tests -q -m gpu -rA > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_traffic.sh || exit $?
cp gpurun_out/traffic_c3.json profiles/${ROUND}_traffic_c3.json
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -1 gpurun_out/prof.log
exit $rc
