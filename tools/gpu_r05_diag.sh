#!/bin/bash
# Round-5 diagnostics on one box, each GPU step under its own time limit,
# stopping at the first failure:
#   1. k_pool phase cycles per valid event (stamps build, tools/pool_stamps.py):
#      C3 concurrent and serialized (FARMS_SERIALIZE=1);
#   2. SERIAL_CFGS (default "3 4"): serialized per-kernel timelines of the bench
#      workload (tools/gpu_serial_tl.sh: one stream, isolated kernel times).
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
LOG=gpurun_out/r05_diag.log
: > $LOG
step() { echo "== $1 rc=$2" | tee -a $LOG; [ "$2" -ne 0 ] && exit "$2"; return 0; }
if [ "${SKIP_STAMPS:-0}" != "1" ]; then
  for C in ${STAMP_CFGS:-3}; do
    timeout -k 10 300 python -u tools/pool_stamps.py --config $C >> $LOG 2>&1
    step stamps_c$C $?
    FARMS_SERIALIZE=1 timeout -k 10 300 python -u tools/pool_stamps.py --config $C >> $LOG 2>&1
    step stamps_serial_c$C $?
  done
fi
for C in ${SERIAL_CFGS:-3 4}; do
  FARMS_SERIALIZE=1 timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/stl_c$C -o kt --output-format csv -- \
     python3 bench.py --no-cpu-baseline --host-steps 0 --steps 1 --warmup 0 --config $C > gpurun_out/stl_c$C.log 2>&1
  step serial_c$C $?
  python3 tools/timeline.py gpurun_out/stl_c$C/kt_kernel_trace.csv > gpurun_out/r05_serialized_c$C.txt 2>&1
  step timeline_c$C $?
  rm -rf gpurun_out/stl_c$C
done
exit 0
