#!/bin/bash
# Round evidence on one box, every GPU step under its own time limit, stopping at
# the first failure: the gpu parity suite, PMC traffic (2 passes) and SQ counters
# (1 pass) of the bench workload, then the bench line (it reads the fresh PMC
# summaries) and a rocprofv3 kernel-trace --stats summary of the same command.
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${ROUND:-r02}
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -v -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log
  [ $rc -ne 0 ] && exit $rc
fi
TRAFFIC_OUT=gpurun_out/${R}_traffic_c3.json bash tools/gpu_traffic.sh > gpurun_out/traffic.log 2>&1
rc=$?; echo "traffic rc=$rc"
[ $rc -ne 0 ] && exit $rc
SQ_OUT=gpurun_out/${R}_sq_c3.json bash tools/gpu_sq.sh > gpurun_out/sq.log 2>&1
rc=$?; echo "sq rc=$rc"
[ $rc -ne 0 ] && exit $rc
# the bench reads profiles/: stage the fresh summaries there (the copy is merged back only via gpurun_out)
cp gpurun_out/${R}_traffic_c3.json gpurun_out/${R}_sq_c3.json profiles/
timeout -k 10 600 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/${R}_bench_c3.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/${R}_bench_c3.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --host-steps 0 ${BENCH_ARGS:-} > gpurun_out/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -1 gpurun_out/prof.log
exit $rc
