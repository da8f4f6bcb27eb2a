#!/bin/bash
# Device-path A/B: the bench's value under env variants (AB="A=1;B=2", ';' separates; "base" = no change).
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
IFS=';' read -ra CASES <<< "${AB:-base}"
i=0
for C in "${CASES[@]}"; do
  [ "$C" = base ] && C=""
  # PARITY=1: a CPU-baseline sample of CPU_SAMPLE events, and the parity block against it
  CB="--no-cpu-baseline"; [ "${PARITY:-0}" = 1 ] && CB="--cpu-sample ${CPU_SAMPLE:-300000}"
  env $C timeout -k 10 600 python bench.py --steps ${STEPS:-8} --warmup 2 $CB --host-steps 0 ${BENCH_ARGS:-} > gpurun_out/dev_ab_$i.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "case [$C] rc=$rc"; tail -5 gpurun_out/dev_ab_$i.log; exit $rc; }
  echo "case [$C]: $(python -c "
import json; d=json.loads(open('gpurun_out/dev_ab_$i.log').read().strip().splitlines()[-1]); p=d.get('parity') or {}; print(d['value'], d['ms_per_step'], p.get('ok', ''), p.get('valid_mismatch', ''), p.get('scale_mismatch', ''))")"
  i=$((i+1))
done
exit 0
