#!/bin/bash
# Round-5 session 3: candidate / strip GPU tests on the per-band export; C3
# A/B against the bitmap-cap timing variant; the C4 N=4 strip rank with flat
# stream priorities against the default, and its N=1 reference.
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
L=gpurun_out/r05_s3.log
: > $L
timeout -k 10 900 python3 -u -m pytest tests -x -v -m gpu -k "cand or strip or chunk or gloo or pair" --timeout 300 --timeout-method thread > gpurun_out/r05_pytest_s3.log 2>&1
rc=$?; tail -2 gpurun_out/r05_pytest_s3.log >> $L; [ $rc -ne 0 ] && exit 1
TAG=s3 LIBS="build/libfarms_hip.so build/libfarms_hip_bitcap1k.so" CFGS="3 4" STEPS=5 ROUNDS=2 bash tools/gpu_r05_ab.sh || exit 2
echo "== strips C4 N=4 rank 1, default priorities" >> $L
timeout -k 10 600 python3 -u tools/strip_rank.py --config 4 --n 4 --ranks 1 --reps 3 --halo-cache /tmp/halo --host-times >> $L 2>&1 || exit 3
echo "== strips C4 N=4 rank 1, FARMS_STREAM_PRIO=flat" >> $L
FARMS_STREAM_PRIO=flat timeout -k 10 600 python3 -u tools/strip_rank.py --config 4 --n 4 --ranks 1 --reps 3 --halo-cache /tmp/halo >> $L 2>&1 || exit 4
echo "== N=1 C4 segments" >> $L
timeout -k 10 600 python3 -u tools/strip_rank.py --config 4 --n 1 --ranks 0 --reps 3 --split segments >> $L 2>&1 || exit 5
rm -rf /tmp/halo
exit 0
