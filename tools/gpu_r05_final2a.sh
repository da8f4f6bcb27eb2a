#!/bin/bash
# Round-5 evidence on the final build (part 1): the GPU suite, then PMC traffic
# + SQ summaries per BASELINE config, copied into profiles/ so that the bench
# lines of part 2 report them.
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r05_pytest_gpu.log 2>&1 || exit 1
L=gpurun_out/r05_final.log
: > $L
R=r05 CFGS="3 2 4 5" bash tools/gpu_pmc_configs.sh >> $L 2>&1 || exit 2
cp gpurun_out/r05_traffic_c*.json gpurun_out/r05_sq_c*.json profiles/
exit 0
