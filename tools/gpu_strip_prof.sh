#!/bin/bash
# Where a middle x-strip's step goes: rank 3 of 8 at C3 (tools/strip_rank.py) under
# a kernel trace, then the pooling-chunk sweep (POOLS, 0 = the engine default).
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/strip_prof -o strip -- \
  python3 -u tools/strip_rank.py --split strips --n 8 --ranks 3 --reps 1 ${SIM_ARGS:-} \
  > gpurun_out/strip_prof.log 2>&1 || exit $?
tail -2 gpurun_out/strip_prof.log
for P in ${POOLS:-0 4096 2048}; do
  timeout -k 10 300 python3 -u tools/strip_rank.py --split strips --n 8 --ranks 3 --pool $P ${SIM_ARGS:-} \
    > gpurun_out/strip_pool_$P.log 2>&1 || exit $?
  tail -2 gpurun_out/strip_pool_$P.log
done
exit 0
