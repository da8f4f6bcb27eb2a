#!/bin/bash
# One-GPU bench lines for the other BASELINE configs (2: 320x320 fs 5; 4: 1280x720
# fs 7; 5: 1280x720 fs 7, 3 scales), then an N=2 rehearsal of both multi-GPU
# splits on the one GPU (gloo).
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
for C in ${CONFIGS:-2 4 5}; do
  timeout -k 10 400 python bench.py --config $C --no-cpu-baseline > gpurun_out/bench_c$C.log 2>&1
  rc=$?; echo "bench config $C rc=$rc"; tail -1 gpurun_out/bench_c$C.log
  [ $rc -ne 0 ] && exit $rc
done
if [ "${REHEARSE:-1}" = "1" ]; then
  bash tools/gpu_rehearse.sh
  rc=$?; [ $rc -ne 0 ] && exit $rc
fi
exit 0
