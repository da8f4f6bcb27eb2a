#!/bin/bash
# A/B of the host-array path's staging threads (FARMS_HOST_THREADS) on the C3 bench.
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
for T in ${THREADS:-8 16 8 16}; do
  FARMS_HOST_THREADS=$T timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 3 > gpurun_out/ab_host_$T.log 2>&1
  rc=$?; echo "[threads $T] rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['host_path'])" gpurun_out/ab_host_$T.log $T
done
exit 0
