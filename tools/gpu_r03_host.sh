#!/bin/bash
# Round-3 GPU step: host-path tests, the bench with its host legs, and an A/B
# of a k_pool variant build (FARMS_HIP_LIB).
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_cli.py -v -m gpu -rA --timeout 400 --timeout-method thread -k "host_path or cli or chunking or streaming or serial or reset or empty or out_of_sensor or fit_variants" > gpurun_out/pytest_host.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_host.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --host-steps 3 > gpurun_out/bench_host.log 2>&1
rc=$?; echo "bench rc=$rc"; python -c "
import json; d=json.loads(open('gpurun_out/bench_host.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], json.dumps(d['detail']), json.dumps(d['host_path']))"
[ $rc -ne 0 ] && exit $rc
for V in ${VARIANTS:-}; do
  FARMS_HIP_LIB=build/libfarms_hip_$V.so timeout -k 10 600 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --host-steps 0 > gpurun_out/bench_$V.log 2>&1
  rc=$?; echo "variant $V rc=$rc"; python -c "
import json; d=json.loads(open('gpurun_out/bench_$V.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], json.dumps(d['detail']))"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
