#!/bin/bash
# Bench lines with the CPU-baseline + parity legs for BASELINE configs 2, 4, 5
# (config 3 is tools/gpu_evidence.sh).
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
for C in ${CONFIGS:-2 4 5}; do
  timeout -k 10 400 python -u bench.py --config $C --host-steps 0 > gpurun_out/r02_bench_c$C.log 2>&1
  rc=$?; echo "config $C rc=$rc"; tail -1 gpurun_out/r02_bench_c$C.log | cut -c1-300
  [ $rc -ne 0 ] && exit $rc
done
exit 0
