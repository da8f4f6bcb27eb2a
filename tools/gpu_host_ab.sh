#!/bin/bash
# Host-path A/B: the bench's host legs under env variants (AB="NAME=VAL ..." entries separated by ';'),
# then a kernel trace of two pinned farms_process calls (tools/host_pipeline_tl.py).
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
IFS=';' read -ra CASES <<< "${AB:-base}"
i=0
for C in "${CASES[@]}"; do
  [ "$C" = base ] && C=""
  env $C timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --host-steps 3 > gpurun_out/host_ab_$i.log 2>&1
  rc=$?; echo "case [$C] rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/host_ab_$i.log; exit $rc; }
  python -c "
import json; d=json.loads(open('gpurun_out/host_ab_$i.log').read().strip().splitlines()[-1]); h=d['host_path']; print(d['value'], h['value'], h['ms_per_step'], h['pageable']['value'])"
  i=$((i+1))
done
if [ "${TRACE:-1}" = 1 ]; then
  FARMS_HOST_TRACE=${HT:-1} timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/hosttl -o hosttl -- python3 tools/host_pipeline_tl.py run > gpurun_out/hosttl_run.log 2>&1
  rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
  python3 tools/host_pipeline_tl.py gpurun_out/hosttl/hosttl_kernel_trace.csv 8 > gpurun_out/hosttl_summary.txt; head -12 gpurun_out/hosttl_summary.txt; grep "farms \(host\|enq\)" gpurun_out/hosttl_run.log | tail -${HTN:-40}
fi
exit 0
