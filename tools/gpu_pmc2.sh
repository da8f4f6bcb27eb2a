#!/bin/bash
# SQ counters of k_pool for each library in AB_LIBS ("-" = default build), one
# --pmc pass per library (no trace domains), then per-kernel summaries.
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
CTRS=${PMC_CTRS:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"}
i=0
for L in ${AB_LIBS:--}; do
  if [ "$L" = "-" ]; then unset FARMS_HIP_LIB; else export FARMS_HIP_LIB=$L; fi
  timeout -k 10 300 rocprofv3 --pmc $CTRS --kernel-include-regex "${PMC_KERNELS:-k_pool}" -d gpurun_out/pmc2_$i -o pmc \
     --output-format csv -- python3 tools/sweep.py --events ${EVENTS:-10000000} --pool ${POOL:-8192} --batch ${BATCH:-64} \
     --fit ${FIT:-65536} --reps 1 > gpurun_out/pmc2_$i.log 2>&1
  rc=$?; echo "[$L] pmc rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  python3 tools/pmc_summary.py gpurun_out/pmc2_$i/pmc_counter_collection.csv
  i=$((i+1))
done
exit 0
