#!/bin/bash
# N=8 rank simulations on one GPU (tools/strip_rank.py), ranks 0, 3 and 7 of each split.
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
for SPLIT in ${SPLITS:-strips segments}; do
  timeout -k 10 600 python3 -u tools/strip_rank.py --split $SPLIT --n ${N:-8} --ranks ${RANKS:-0,3,7} ${SIM_ARGS:-} \
    > gpurun_out/ranksim_${SPLIT}_n${N:-8}.log 2>&1
  rc=$?; echo "ranksim $SPLIT rc=$rc"; tail -4 gpurun_out/ranksim_${SPLIT}_n${N:-8}.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
