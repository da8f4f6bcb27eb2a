#!/bin/bash
# Round-5 evidence on the final build (part 2): the bench line of every config
# (C3 with its CPU baseline, host path and parity; C2/C4/C5 likewise), the
# rocprofv3 --kernel-trace --stats of the C3 bench command, and serialized
# kernel timelines (FARMS_SERIALIZE=1) at C3 and C4.
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
L=gpurun_out/r05_final.log
for C in 3 2 4 5; do
  timeout -k 10 900 python3 -u bench.py --config $C > gpurun_out/r05_bench_c$C.log 2>&1
  rc=$?; echo "bench c$C rc=$rc" >> $L; [ $rc -ne 0 ] && exit 2
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o kt --output-format csv -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --host-steps 0 > gpurun_out/r05_prof_c3.log 2>&1
rc=$?; echo "rocprof c3 rc=$rc" >> $L; [ $rc -ne 0 ] && exit 3
cp gpurun_out/prof_c3/kt_kernel_stats.csv gpurun_out/r05_kernel_stats.csv
rm -rf gpurun_out/prof_c3
for C in 3 4; do
  BENCH_ARGS="--config $C" bash tools/gpu_serial_tl.sh > gpurun_out/r05_serialized_c$C.txt 2>&1
  rc=$?; echo "serial c$C rc=$rc" >> $L; [ $rc -ne 0 ] && exit 4
  rm -rf gpurun_out/stl_libfarms_hip
done
exit 0
