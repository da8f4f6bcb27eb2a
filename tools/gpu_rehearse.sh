#!/bin/bash
# Multi-rank rehearsal on the one-GPU box: N ranks (gloo for the bench's
# collectives, every rank on device 0) through bench.py, per split mode.
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
N=${N:-2}
for SPLIT in ${SPLITS:-segments strips}; do
  FARMS_BENCH_DEVICE=0 FARMS_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 \
     --nproc-per-node $N --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus $N --steps 2 --warmup 1 \
     --events ${REH_EVENTS:-10000000} --split $SPLIT > gpurun_out/rehearsal_${SPLIT}_n$N.log 2>&1
  rc=$?; echo "rehearsal $SPLIT n=$N rc=$rc"; grep metric gpurun_out/rehearsal_${SPLIT}_n$N.log | tail -1
  [ $rc -ne 0 ] && exit $rc
done
exit 0
