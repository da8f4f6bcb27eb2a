#!/bin/bash
# A/B of (library, bench arguments) pairs on the bench workload: AB entries
# "lib|args" separated by ';' (lib relative to the package; args may be empty).
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
IFS=';' read -ra SETS <<< "${AB:-build/libfarms_hip.so|}"
for S in "${SETS[@]}"; do
  i=$((i+1))
  L="${S%%|*}"; A="${S#*|}"
  FARMS_HIP_LIB=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline --host-steps 0 --steps ${STEPS:-5} $A > gpurun_out/abmix_$i.log 2>&1
  rc=$?; echo "[$S] rc=$rc"
  [ $rc -ne 0 ] && { tail -5 gpurun_out/abmix_$i.log; exit $rc; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['detail']['ms_fit_sweep'], d['detail']['ms_pool_sweep'])" gpurun_out/abmix_$i.log
done
exit 0
