#!/bin/bash
# Serialized kernel timelines (FARMS_SERIALIZE=1: one stream, no overlap) of the
# bench workload for each library in LIBS: the isolated cost of every kernel.
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
for L in ${LIBS:-build/libfarms_hip.so}; do
  N=$(basename $L .so)
  FARMS_HIP_LIB=$L FARMS_SERIALIZE=1 timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/stl_$N -o kt --output-format csv -- \
     python3 bench.py --no-cpu-baseline --host-steps 0 --steps 1 --warmup 0 ${BENCH_ARGS:-} > gpurun_out/stl_$N.log 2>&1
  rc=$?; echo "[$N] kernel-trace rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  python3 tools/timeline.py gpurun_out/stl_$N/kt_kernel_trace.csv | grep -E "span|busy|k_|rocprim" | head -16
done
exit 0
