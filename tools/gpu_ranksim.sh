#!/bin/bash
# N=8 rank simulations on one GPU (tools/strip_rank.py): x-strips with the
# flow-halo exchange and temporal segments, three ranks each.
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
for SPLIT in ${SPLITS:-strips segments}; do
  timeout -k 10 500 python3 -u tools/strip_rank.py --split $SPLIT --n 8 --ranks ${RANKS:-0,3,7} > gpurun_out/ranksim_${SPLIT}_n8.log 2>&1
  rc=$?; echo "ranksim $SPLIT rc=$rc"; tail -4 gpurun_out/ranksim_${SPLIT}_n8.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
