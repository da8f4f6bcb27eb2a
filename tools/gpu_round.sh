#!/bin/bash
# GPU session: full test suite (gpu marker), 1-GPU bench, 2-rank strip rehearsal
# on the one GPU (gloo), rocprofv3 kernel-trace summary.
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -q -m gpu -rA > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log
[ $rc -ne 0 ] && exit $rc
if [ "${REHEARSE:-1}" = "1" ]; then
  FARMS_BENCH_DEVICE=0 FARMS_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 \
     --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 \
     --events ${REH_EVENTS:-20000000} > gpurun_out/bench_n2_rehearsal.log 2>&1
  rc=$?; echo "rehearsal rc=$rc"; grep metric gpurun_out/bench_n2_rehearsal.log | tail -1
  [ $rc -ne 0 ] && exit $rc
fi
if [ "${PROFILE:-1}" = "1" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
      python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1
  rc=$?; echo "rocprof rc=$rc"
fi
exit $rc
