#!/bin/bash
# Round-4 multi-GPU evidence on one box (each step under its own limit, the
# first failure ends the script):
#   1. rank simulations at N=4 of BASELINE config 4 (fs 7, 50M events per GPU),
#      x-strips (edge rank 0, middle rank 1) and temporal segments (ranks 0, 3)
#      -> gpurun_out/ranksim_{strips,segments}_n4_c4.log
#   2. PMC summaries of one rank-simulated x-strip step (C3, N=8, middle rank 3)
#      -> gpurun_out/traffic_c3_strips.json, sq_c3_strips.json
#   3. N=2 rehearsals (two ranks on device 0 over gloo) of both splits at C3,
#      5M events per rank: the per-rank measurement fields of an N>1 line
#      -> gpurun_out/rehearsal_{segments,strips}_n2_c3.log
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${SKIP_RANKSIM:-0}" != "1" ]; then
  timeout -k 10 900 python3 -u tools/strip_rank.py --config 4 --split strips --n 4 --ranks 0,1 \
    > gpurun_out/ranksim_strips_n4_c4.log 2>&1
  rc=$?; echo "ranksim strips n4 c4 rc=$rc"; tail -1 gpurun_out/ranksim_strips_n4_c4.log; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 900 python3 -u tools/strip_rank.py --config 4 --split segments --n 4 --ranks 0,3 \
    > gpurun_out/ranksim_segments_n4_c4.log 2>&1
  rc=$?; echo "ranksim segments n4 c4 rc=$rc"; tail -1 gpurun_out/ranksim_segments_n4_c4.log; [ $rc -ne 0 ] && exit $rc
fi
if [ "${SKIP_SPMC:-0}" != "1" ]; then
  bash tools/gpu_strip_pmc.sh > gpurun_out/strip_pmc.out 2>&1
  rc=$?; echo "strip pmc rc=$rc"; [ $rc -ne 0 ] && exit $rc
  cp gpurun_out/traffic_c3_strips.json profiles/r04_traffic_c3_strips.json
  cp gpurun_out/sq_c3_strips.json profiles/r04_sq_c3_strips.json
fi
STAGES=rehearse CFG=3 N=2 bash tools/gpu_r04.sh
exit $?
