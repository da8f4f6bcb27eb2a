#!/bin/bash
# Round-5 session 18: paired pooling on by default at fs 7 from 8 scales up
# (C4): the GPU suite, PMC traffic + SQ at C4, the C4 bench line.
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r05_pytest_gpu.log 2>&1 || exit 1
R=r05 CFGS="4" bash tools/gpu_pmc_configs.sh > gpurun_out/r05_pmc_c4.log 2>&1 || exit 2
cp gpurun_out/r05_traffic_c4.json gpurun_out/r05_sq_c4.json profiles/
timeout -k 10 900 python3 -u bench.py --config 4 > gpurun_out/r05_bench_c4.log 2>&1 || exit 3
exit 0
