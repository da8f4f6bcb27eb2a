#!/bin/bash
# GPU session step: HBM traffic of the hot kernels on the bench workload, one
# rocprofv3 --pmc pass per counter (FETCH_SIZE and WRITE_SIZE do not fit one
# pass; --pmc is never combined with a trace domain).  Writes the summary JSON
# that bench.py reports as roofline.traffic.
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=${TRAFFIC_OUT:-gpurun_out/traffic_c3.json}
ARGS="--steps 1 --warmup 0 --no-cpu-baseline --host-steps 0 ${BENCH_ARGS:-}"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $C --kernel-include-regex "k_pool|k_fit|k_chain|k_cand|k_flow" -d gpurun_out/pmc_$C -o pmc \
     --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc_$C.log 2>&1
  rc=$?; echo "pmc $C rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
python3 tools/traffic.py gpurun_out/pmc_FETCH_SIZE/pmc_counter_collection.csv \
   gpurun_out/pmc_WRITE_SIZE/pmc_counter_collection.csv --label "bench.py $ARGS" > $OUT
rc=$?; echo "traffic rc=$rc"; cat $OUT
exit $rc
