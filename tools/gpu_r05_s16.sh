#!/bin/bash
# Round-5 session 16: k_pool_compact in 1,024-thread blocks: the pooling GPU
# tests, then C3 / C2 A/B against the build before it.
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r05_pytest_s16.log 2>&1 || exit 1
L=gpurun_out/r05_ab_s16.log
: > $L
timeout -k 10 600 python3 -u tools/lib_ab.py --config 3 --steps 5 --rounds 2 build/libfarms_hip_r05b.so build/libfarms_hip.so >> $L 2>&1 || exit 2
timeout -k 10 300 python3 -u tools/lib_ab.py --config 2 --steps 10 --rounds 2 build/libfarms_hip_r05b.so build/libfarms_hip.so >> $L 2>&1 || exit 3
exit 0
