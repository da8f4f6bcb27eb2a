#!/bin/bash
# Host-path pipeline cases: one pinned farms_process of the C3 stream per case (tools/host_pipeline_tl.py run),
# with FARMS_HOST_TRACE=1; prints when F, P and the downloads finished. CASES="A=1 B=2;C=3;..." (';' separates cases).
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
IFS=';' read -ra CS <<< "${CASES:-X=0}"
i=0
for C in "${CS[@]}"; do
  env $C FARMS_HOST_TRACE=1 timeout -k 10 120 python3 tools/host_pipeline_tl.py run > gpurun_out/hc_$i.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "case [$C] rc=$rc"; tail -5 gpurun_out/hc_$i.log; exit $rc; }
  echo "case [$C]: $(grep 'farms host' gpurun_out/hc_$i.log | tail -4 | awk '{printf "%s %s %s | ", $4, $5, $3}')"
  i=$((i+1))
done
exit 0
