#!/bin/bash
# PMC counters for the two hot kernels (one pass per counter group; --pmc never
# combined with trace domains).  PMC_SET selects the group.
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
EV=${EVENTS:-5000000}
SET=${PMC_SET:-sq}
case $SET in
  sq)  CTRS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY";;
  mem) CTRS="FETCH_SIZE";;
  wr)  CTRS="WRITE_SIZE";;
  tcc) CTRS="TCC_HIT_sum TCC_MISS_sum";;
  ta)  CTRS="TA_BUSY_avr TA_TA_BUSY_sum SQ_INSTS_SMEM SQ_INSTS_SALU";;
esac
timeout -k 10 500 rocprofv3 --pmc $CTRS --kernel-include-regex "${PMC_KERNELS:-k_pool|k_fit|k_chain}" -d gpurun_out/pmc_$SET -o pmc \
   --output-format csv -- python3 tools/sweep.py --events $EV --pool ${POOL:-32768} --batch ${BATCH:-8} --fit ${FIT:-65536} --reps 1 \
   > gpurun_out/pmc_$SET.log 2>&1
rc=$?; echo "pmc $SET rc=$rc"; exit $rc
