#!/bin/bash
# A/B of bench.py argument sets (AB_ARGS: sets separated by ';') on one box.
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
IFS=';' read -ra SETS <<< "${AB_ARGS:- }"
for A in "${SETS[@]}"; do
  i=$((i+1))
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --host-steps 0 --steps ${STEPS:-5} $A > gpurun_out/abargs_$i.log 2>&1
  rc=$?; echo "[$A] rc=$rc"
  [ $rc -ne 0 ] && { tail -5 gpurun_out/abargs_$i.log; exit $rc; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['detail'])" gpurun_out/abargs_$i.log
done
exit 0
