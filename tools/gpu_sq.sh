#!/bin/bash
# GPU session step: SQ counters of the hot kernels on the bench workload (one
# --pmc pass of 8 SQ counters, never combined with a trace domain).  Writes the
# summary JSON bench.py reports as roofline.issue.
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=${SQ_OUT:-gpurun_out/sq_c3.json}
ARGS="--steps 1 --warmup 0 --no-cpu-baseline --host-steps 0 ${BENCH_ARGS:-}"
CTRS="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD"
timeout -k 10 600 rocprofv3 --pmc $CTRS --kernel-include-regex "k_pool|k_fit|k_chain|k_cand|k_flow" -d gpurun_out/pmc_sq -o pmc \
   --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc_sq.log 2>&1
rc=$?; echo "pmc sq rc=$rc"
[ $rc -ne 0 ] && exit $rc
python3 tools/sq_summary.py gpurun_out/pmc_sq/pmc_counter_collection.csv --label "bench.py $ARGS" > $OUT
rc=$?; echo "sq summary rc=$rc"
exit $rc
