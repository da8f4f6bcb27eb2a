#!/bin/bash
# Round-5 session 2: pooling / candidate / strip parity tests on the current
# build; C3 A/B of the current build against a2ed55c (r05e) and the two tuning
# variants (bitmap cap: timing only; ring staging); the C3 scan-width tail;
# then a kernel trace of the C4 N=4 strip step with each stream's hardware
# queue.  Every GPU step under its own limit, stopping at the first failure.
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=s2 TESTS="pair or pool or strip or cand or chunk" LIBS="build/libfarms_hip.so build/libfarms_hip_r05e.so build/libfarms_hip_bitcap1k.so build/libfarms_hip_ring.so" CFGS=3 STEPS=5 ROUNDS=2 bash tools/gpu_r05_ab.sh || exit 1
timeout -k 10 300 python3 -u bench.py --config 3 --steps 3 --warmup 1 --no-cpu-baseline --host-steps 0 > gpurun_out/r05_bench_c3_scan.log 2>&1 || exit 2
timeout -k 10 600 python3 -u tools/strip_rank.py --config 4 --n 4 --ranks 1 --reps 1 --halo-cache /tmp/halo > gpurun_out/r05_strips_q.log 2>&1 || exit 3
timeout -k 10 600 rocprofv3 --kernel-trace -d gpurun_out/kt_strip -o kt --output-format csv -- \
  python3 -u tools/strip_rank.py --config 4 --n 4 --ranks 1 --reps 1 --halo-cache /tmp/halo >> gpurun_out/r05_strips_q.log 2>&1 || exit 4
python3 tools/strip_trace.py gpurun_out/kt_strip/kt_kernel_trace.csv --timeline --label "C4 N=4 strips, rank 1" \
  > gpurun_out/r05_strip_trace_q.txt 2>&1 || exit 5
head -1 gpurun_out/kt_strip/kt_kernel_trace.csv > gpurun_out/r05_kt_header.txt
rm -rf gpurun_out/kt_strip /tmp/halo
exit 0
