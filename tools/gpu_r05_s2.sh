#!/bin/bash
# Round-5 session: the whole GPU test suite on the current build; C3 A/B of the
# current build against the ring-staging and bitmap-cap (timing only) variants;
# the C3 scan-width tail; then a kernel trace of the C4 N=4 strip step with each
# stream's hardware queue.  Every GPU step under its own limit, stopping at the
# first failure.
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
L=gpurun_out/r05_s2.log
: > $L
timeout -k 10 1200 python3 -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r05_pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/r05_pytest_gpu.log >> $L; [ $rc -ne 0 ] && exit 1
TAG=s2 LIBS="build/libfarms_hip.so build/libfarms_hip_ring.so build/libfarms_hip_bitcap1k.so" CFGS=3 STEPS=5 ROUNDS=2 bash tools/gpu_r05_ab.sh || exit 2
timeout -k 10 300 python3 -u bench.py --config 3 --steps 3 --warmup 1 --no-cpu-baseline --host-steps 0 > gpurun_out/r05_bench_c3_scan.log 2>&1 || exit 3
timeout -k 10 600 python3 -u tools/strip_rank.py --config 4 --n 4 --ranks 1 --reps 1 --halo-cache /tmp/halo > gpurun_out/r05_strips_q.log 2>&1 || exit 4
timeout -k 10 600 rocprofv3 --kernel-trace -d gpurun_out/kt_strip -o kt --output-format csv -- \
  python3 -u tools/strip_rank.py --config 4 --n 4 --ranks 1 --reps 1 --halo-cache /tmp/halo >> gpurun_out/r05_strips_q.log 2>&1 || exit 5
python3 tools/strip_trace.py gpurun_out/kt_strip/kt_kernel_trace.csv --timeline --label "C4 N=4 strips, rank 1" \
  > gpurun_out/r05_strip_trace_q.txt 2>&1 || exit 6
head -1 gpurun_out/kt_strip/kt_kernel_trace.csv > gpurun_out/r05_kt_header.txt
rm -rf gpurun_out/kt_strip /tmp/halo
exit 0
