#!/bin/bash
# GPU session step: PMC summaries of the bench workload per BASELINE config
# (HBM traffic: FETCH_SIZE and WRITE_SIZE passes; SQ: one pass of 8 counters),
# each pass its own rocprofv3 run, never combined with a trace domain.  Writes
# gpurun_out/${R}_traffic_c$CFG.json and gpurun_out/${R}_sq_c$CFG.json, which
# bench.py reads (once copied to profiles/) for the lines of that config.
#   CFGS (default "2 3 4 5"), R (round prefix, default r04), BENCH_ARGS
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${R:-r04}
for CFG in ${CFGS:-2 3 4 5}; do
  TRAFFIC_OUT=gpurun_out/${R}_traffic_c$CFG.json BENCH_ARGS="--config $CFG ${BENCH_ARGS:-}" bash tools/gpu_traffic.sh \
    > gpurun_out/${R}_traffic_c$CFG.out 2>&1
  rc=$?; echo "traffic c$CFG rc=$rc"; [ $rc -ne 0 ] && exit $rc
  SQ_OUT=gpurun_out/${R}_sq_c$CFG.json BENCH_ARGS="--config $CFG ${BENCH_ARGS:-}" bash tools/gpu_sq.sh \
    > gpurun_out/${R}_sq_c$CFG.out 2>&1
  rc=$?; echo "sq c$CFG rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
