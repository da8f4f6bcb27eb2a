#!/bin/bash
# Round evidence on one box: gpu parity suite, HBM traffic of the hot kernels
# (two --pmc passes, copied into profiles/ so that the bench line reports it),
# the bench line (with CPU baseline and parity), and a rocprofv3 kernel-trace
# --stats summary of the same bench command.
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${ROUND:-r01}
timeout -k 10 600 python -u -m pytest tests -v -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
TRAFFIC_OUT=gpurun_out/traffic_c3.json bash tools/gpu_traffic.sh > gpurun_out/traffic.log 2>&1
rc=$?; echo "traffic rc=$rc"
[ $rc -ne 0 ] && exit $rc
cp gpurun_out/traffic_c3.json profiles/${R}_traffic_c3.json
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -1 gpurun_out/prof.log
[ $rc -ne 0 ] && exit $rc
if [ "${RANKSIM:-0}" = "1" ]; then  # ranks 0, 4, 7 of an N=8 temporal-segment run, one after the other
  timeout -k 10 900 python3 tools/strip_rank.py --split segments --n 8 --ranks 0,4,7 > gpurun_out/seg8_rank_sim.log 2>&1
  rc=$?; echo "rank sim rc=$rc"; tail -1 gpurun_out/seg8_rank_sim.log
fi
exit $rc
