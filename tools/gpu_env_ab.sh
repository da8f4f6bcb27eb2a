#!/bin/bash
# Environment-knob A/B on one box: for each setting in SETTINGS (space-separated
# VAR=value[,VAR=value] items, "-" for none), tools/lib_ab.py --child steps of
# config CFG in alternation, ROUNDS rounds.  Device-resident step time only.
cd /root/repo
mkdir -p gpurun_out
CFG=${CFG:-3}
OUT=gpurun_out/env_ab_c$CFG.log
for r in $(seq ${ROUNDS:-2}); do
  for S in ${SETTINGS:--}; do
    ENVS=()
    [ "$S" != "-" ] && IFS=, read -ra ENVS <<< "$S"
    env "${ENVS[@]}" timeout -k 10 300 python3 tools/lib_ab.py --child --config $CFG --steps ${STEPS:-4} \
      > gpurun_out/env_ab.tmp 2>&1 || { tail -5 gpurun_out/env_ab.tmp; exit 1; }
    echo "$S $(tail -1 gpurun_out/env_ab.tmp)" | tee -a $OUT
  done
done
