#!/bin/bash
# GPU session step: PMC summaries (HBM traffic, SQ) of one rank-simulated
# x-strip step (tools/strip_rank.py, the pipelined Stepper order), for the
# per-rank rooflines bench.py reports on --split strips lines.  The halo flows
# come from a first, unprofiled run (--halo-cache), so the profiled runs hold
# only the rank's own kernels.
#   CFG (3), N (8), RANK (3: a middle strip), EVENTS (50000000 per GPU)
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=${CFG:-3}; N=${N:-8}; RANK=${RANK:-3}; EVENTS=${EVENTS:-50000000}
ARGS="--config $CFG --n $N --ranks $RANK --events $EVENTS --reps 1 --split strips --halo-cache /tmp/farms_halo"
LABEL="tools/strip_rank.py $ARGS"
timeout -k 10 600 python3 -u tools/strip_rank.py $ARGS > gpurun_out/strip_pmc_prep.log 2>&1
rc=$?; echo "halo prep rc=$rc"; [ $rc -ne 0 ] && exit $rc
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $C --kernel-include-regex "k_pool|k_fit|k_chain|k_cand|k_flow" -d gpurun_out/spmc_$C -o pmc \
     --output-format csv -- python3 tools/strip_rank.py $ARGS > gpurun_out/spmc_$C.log 2>&1
  rc=$?; echo "pmc $C rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
python3 tools/traffic.py gpurun_out/spmc_FETCH_SIZE/pmc_counter_collection.csv \
   gpurun_out/spmc_WRITE_SIZE/pmc_counter_collection.csv --label "$LABEL" > gpurun_out/traffic_c${CFG}_strips.json
rc=$?; echo "traffic rc=$rc"; [ $rc -ne 0 ] && exit $rc
CTRS="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD"
timeout -k 10 600 rocprofv3 --pmc $CTRS --kernel-include-regex "k_pool|k_fit|k_chain|k_cand|k_flow" -d gpurun_out/spmc_sq -o pmc \
   --output-format csv -- python3 tools/strip_rank.py $ARGS > gpurun_out/spmc_sq.log 2>&1
rc=$?; echo "pmc sq rc=$rc"; [ $rc -ne 0 ] && exit $rc
python3 tools/sq_summary.py gpurun_out/spmc_sq/pmc_counter_collection.csv --label "$LABEL" \
   > gpurun_out/sq_c${CFG}_strips.json
rc=$?; echo "sq summary rc=$rc"
exit $rc
