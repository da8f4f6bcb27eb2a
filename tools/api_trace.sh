#!/bin/bash
# kernel + HIP API trace of a short C2 bench run (host enqueue gaps)
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace -d gpurun_out/r06z_api -o kt --output-format csv -- python3 bench.py --config 2 --steps 2 --warmup 1 --no-cpu-baseline --host-steps 0 > gpurun_out/r06z_api.log 2>&1; echo rc=$?; ls gpurun_out/r06z_api
