#!/bin/bash
# Round-5 session 15: work-order tile edge A/B at C3 on the final build
# (FARMS_TILE_SHIFT 2 / 3 (default) / 4), alternating.
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
L=gpurun_out/r05_ab_tile_c3.log
: > $L
for r in 1 2; do
  for S in 3 2 4; do
    echo "== FARMS_TILE_SHIFT=$S" >> $L
    FARMS_TILE_SHIFT=$S timeout -k 10 300 python3 -u tools/lib_ab.py --config 3 --steps 4 --rounds 1 build/libfarms_hip.so >> $L 2>&1 || exit 1
  done
done
exit 0
