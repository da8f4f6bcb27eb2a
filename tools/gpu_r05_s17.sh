#!/bin/bash
# Round-5 session 17: paired pooling beside the fs-7 fit on the final build
# (band-contiguous slots), C4 and C5, FARMS_POOL_PAIRS=1 against the default.
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
L=gpurun_out/r05_ab_pairs_fs7_final.log
: > $L
for r in 1 2; do
  for C in 4 5; do
    echo "== C$C default" >> $L
    timeout -k 10 600 python3 -u tools/lib_ab.py --config $C --steps 4 --rounds 1 build/libfarms_hip.so >> $L 2>&1 || exit 1
    echo "== C$C FARMS_POOL_PAIRS=1" >> $L
    FARMS_POOL_PAIRS=1 timeout -k 10 600 python3 -u tools/lib_ab.py --config $C --steps 4 --rounds 1 build/libfarms_hip.so >> $L 2>&1 || exit 2
  done
done
exit 0
