#!/bin/bash
# Fit-mode A/B (FARMS_FIT_MODE 0..3, see csrc/farms_engine.hip launch_fit):
# device-resident bench steps per mode and config, bitwise parity of each mode
# against the default is covered by tests/test_gpu_parity.py.
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
for CFG in ${CFGS:-3 4}; do
  for M in ${MODES:-0 1 2 3}; do
    FARMS_FIT_MODE=$M timeout -k 10 300 python3 bench.py --config $CFG --steps ${STEPS:-6} --warmup 2 --no-cpu-baseline \
      --host-steps 0 > gpurun_out/fitab_c${CFG}_m$M.log 2>&1
    rc=$?; echo "cfg $CFG mode $M rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/fitab_c${CFG}_m$M.log) $(grep -o '"ms_fit_kernel": [0-9.]*' gpurun_out/fitab_c${CFG}_m$M.log) $(grep -o '"ms_pool_kernel": [0-9.]*' gpurun_out/fitab_c${CFG}_m$M.log)"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
