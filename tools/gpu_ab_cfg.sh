#!/bin/bash
# A/B of library builds on configs 3 and 4 (sweep.py, default chunking of each
# config): one line per (library, config). AB_LIBS as in gpu_iter.sh.
cd /root/repo
mkdir -p gpurun_out
for L in ${AB_LIBS:--}; do
  if [ "$L" = "-" ]; then unset FARMS_HIP_LIB; else export FARMS_HIP_LIB=$L; fi
  for C in ${CONFIGS:-3 4}; do
    FS=5; FIT=65536; POOL=8192; BATCH=64
    [ "$C" = "4" ] && { FS=7; FIT=131072; POOL=16384; BATCH=32; }
    timeout -k 10 200 python3 tools/sweep.py --config $C --fs $FS --events 50000000 --pool $POOL --batch $BATCH \
        --fit $FIT --reps 3 > gpurun_out/abc.log 2>&1
    rc=$?; echo "[$L c$C] rc=$rc $(grep fit_chunk gpurun_out/abc.log | cut -c1-120)"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
