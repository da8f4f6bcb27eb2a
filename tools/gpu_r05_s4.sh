#!/bin/bash
# Round-5 session 4: the whole GPU test suite (pair bitmap cap + overflow
# pooling, per-band S2 export); the C3 bench line (scan-width tail); C2/C4
# step times; the C4 N=4 strip rank.  Stops at the first failure.
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
L=gpurun_out/r05_s4.log
: > $L
timeout -k 10 1200 python3 -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r05_pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/r05_pytest_gpu.log >> $L; [ $rc -ne 0 ] && exit 1
timeout -k 10 300 python3 -u bench.py --config 3 --steps 5 --warmup 2 --no-cpu-baseline --host-steps 0 > gpurun_out/r05_bench_c3_s4.log 2>&1 || exit 2
TAG=s4 LIBS="build/libfarms_hip.so" CFGS="2 4" STEPS=5 ROUNDS=1 bash tools/gpu_r05_ab.sh || exit 3
echo "== strips C4 N=4 rank 1" >> $L
timeout -k 10 600 python3 -u tools/strip_rank.py --config 4 --n 4 --ranks 1 --reps 3 >> $L 2>&1 || exit 4
exit 0
