#!/bin/bash
# Round-5 session 9: Gx / Gy divided on two lanes (one division sequence):
# GPU parity suite, C3 A/B against the round-5 final build.
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r05_pytest_s9.log 2>&1 || exit 1
L=gpurun_out/r05_ab_s9.log
: > $L
timeout -k 10 600 python3 -u tools/lib_ab.py --config 3 --steps 5 --rounds 2 build/libfarms_hip_r05a.so build/libfarms_hip.so >> $L 2>&1 || exit 2
exit 0
