#!/bin/bash
# A/B of engine environment settings on the bench workload: optional gpu tests
# (TESTS=...), then one bench line per entry of AB_ENV (entries separated by
# spaces, VAR=value pairs within an entry joined by commas; "-" = defaults).
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -v -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
  [ $rc -ne 0 ] && exit $rc
fi
i=0
for V in ${AB_ENV:--}; do
  i=$((i+1))
  if [ "$V" = "-" ]; then E=""; else E="${V//,/ }"; fi
  env $E timeout -k 10 300 python -u bench.py --no-cpu-baseline --host-steps 0 --steps ${STEPS:-5} ${BENCH_ARGS:-} > gpurun_out/abenv_$i.log 2>&1
  rc=$?; echo "[$V] rc=$rc"
  [ $rc -ne 0 ] && { tail -5 gpurun_out/abenv_$i.log; exit $rc; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['detail'])" gpurun_out/abenv_$i.log
done
exit 0
