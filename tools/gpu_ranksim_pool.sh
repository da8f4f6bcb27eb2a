#!/bin/bash
# N=8 x-strip rank simulations (tools/strip_rank.py, one middle rank) over
# pooling chunk / batch settings: POOLS entries "chunk:batch".
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
for PB in ${POOLS:-0:0}; do
  IFS=: read P B <<< "$PB"
  timeout -k 10 300 python3 -u tools/strip_rank.py --split ${SPLIT:-strips} --n 8 --ranks ${RANKS:-3} --pool $P --batch $B \
     --reps 1 > gpurun_out/ranksim_pool_${P}_${B}.log 2>&1
  rc=$?; echo "[$PB] rc=$rc"; grep '"rank"' gpurun_out/ranksim_pool_${P}_${B}.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
