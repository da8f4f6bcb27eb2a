#!/bin/bash
# Round-4 A/B of engine knobs on the device-resident bench step.
#   CFGS   configs to run (default "3 4")
#   COMBOS space-separated combos; each combo is a comma-separated list of
#          VAR=value settings ("-" = defaults), e.g. "FARMS_FIT_MODE=1,FARMS_POOL_GROUP=0 -"
# One log per (config, combo) under gpurun_out/ab4_*.log and a summary line each.
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
for CFG in ${CFGS:-3 4}; do
  for C in ${COMBOS:--}; do
    tag=$(echo "$C" | tr ',=/' '_-_')
    envs=()
    [ "$C" != "-" ] && IFS=',' read -ra envs <<< "$C"
    timeout -k 10 300 env "${envs[@]}" python3 bench.py --config $CFG --steps ${STEPS:-6} --warmup 2 \
      --no-cpu-baseline --host-steps 0 ${BENCH_ARGS:-} > gpurun_out/ab4_c${CFG}_$tag.log 2>&1
    rc=$?
    echo "cfg $CFG [$C] rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab4_c${CFG}_$tag.log) \
$(grep -o '"ms_fit_kernel": [0-9.]*' gpurun_out/ab4_c${CFG}_$tag.log | tail -1) \
$(grep -o '"ms_pool_kernel": [0-9.]*' gpurun_out/ab4_c${CFG}_$tag.log | tail -1)"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
