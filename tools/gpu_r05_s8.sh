#!/bin/bash
# Round-5 session 8: DPP-fused row-shift scans and the flat row setup's
# trimmed clamps: GPU parity suite, C3 / C4 A/B against the round-5 final
# build, SQ counters at C3.
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r05_pytest_s8.log 2>&1 || exit 1
L=gpurun_out/r05_ab_s8.log
: > $L
timeout -k 10 600 python3 -u tools/lib_ab.py --config 3 --steps 5 --rounds 2 build/libfarms_hip_r05a.so build/libfarms_hip.so >> $L 2>&1 || exit 2
timeout -k 10 600 python3 -u tools/lib_ab.py --config 4 --steps 4 --rounds 2 build/libfarms_hip_r05a.so build/libfarms_hip.so >> $L 2>&1 || exit 3
SQ_OUT=gpurun_out/r05_sq_s8_c3.json BENCH_ARGS="--config 3" timeout -k 10 600 bash tools/gpu_sq.sh > gpurun_out/r05_sq_s8.out 2>&1 || exit 4
exit 0
