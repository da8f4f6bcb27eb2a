#!/bin/bash
# Round-5 session: the strip pipeline with the pooling's import wait skipped
# (against the a2ed55c build), the scan-width tail at C3, then the pair finish /
# mbcnt build and the bitmap-cap timing experiment against a2ed55c, with the
# pooling and strip parity tests first.  Every GPU step under its own limit.
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
L=gpurun_out/r05_strip_ready_ab.log
timeout -k 10 300 python3 -u tools/strip_rank.py --config 4 --n 4 --ranks 1 --reps 3 --host-times --halo-cache /tmp/halo > $L 2>&1 || exit 1
echo "== r05e (before)" >> $L
FARMS_HIP_LIB=aperture-robust-multiscale-optical-flow_amd/build/libfarms_hip_r05e.so timeout -k 10 300 python3 -u tools/strip_rank.py --config 4 --n 4 --ranks 1 --reps 3 --halo-cache /tmp/halo >> $L 2>&1 || exit 2
timeout -k 10 300 python3 -u bench.py --config 3 --steps 3 --warmup 1 --no-cpu-baseline --host-steps 0 > gpurun_out/r05_bench_c3_scan.log 2>&1 || exit 3
TAG=finish TESTS="pair or pool or strip or cand or chunk" LIBS="build/libfarms_hip.so build/libfarms_hip_r05e.so build/libfarms_hip_bitcap1k.so build/libfarms_hip_ring.so" CFGS=3 STEPS=5 ROUNDS=2 bash tools/gpu_r05_ab.sh || exit 4
