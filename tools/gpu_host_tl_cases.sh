#!/bin/bash
# Kernel traces of the host pipeline (tools/host_pipeline_tl.py run) per case: CASES="A=1;B=2" (';' separates).
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
IFS=';' read -ra CS <<< "${CASES:-X=0}"
i=0
for C in "${CS[@]}"; do
  env $C FARMS_HOST_TRACE=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/htl_$i -o t -- python3 tools/host_pipeline_tl.py run > gpurun_out/htl_$i.log 2>&1
  rc=$?; echo "case [$C] rc=$rc"; [ $rc -ne 0 ] && exit $rc
  grep 'farms host' gpurun_out/htl_$i.log | tail -4
  i=$((i+1))
done
exit 0
