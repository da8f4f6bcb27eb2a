#!/bin/bash
# A/B of library builds on the bench workload: optional gpu parity tests (TESTS=...),
# then one bench line per library in LIBS (paths relative to the package dir).
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -v -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
  [ $rc -ne 0 ] && exit $rc
fi
for L in ${LIBS:-build/libfarms_hip.so}; do
  FARMS_HIP_LIB=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps ${STEPS:-5} ${BENCH_ARGS:-} > gpurun_out/ab_$(basename $L .so).log 2>&1
  rc=$?; echo "[$L] rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['detail'])" gpurun_out/ab_$(basename $L .so).log
done
exit 0
