#!/bin/bash
# x-strip pipeline check and A/B: the strip / multirank GPU tests and the
# range-check tests, then rank 3 of 8 at C3 (tools/strip_rank.py) for each
# "sets:pool_chunk" case in CASES (FARMS_PHASE_SETS; pool chunk 0 = default).
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_strips.py tests/test_multirank.py tests/test_gpu_parity.py -m gpu -x -v \
  -k "strip or multirank or segment or halo or sensor or empty" --timeout 300 \
  --timeout-method thread > gpurun_out/strip_tests.log 2>&1 || { tail -30 gpurun_out/strip_tests.log; exit 1; }
tail -2 gpurun_out/strip_tests.log
for C in ${CASES:-2:0 3:0 2:8192}; do
  S=${C%%:*}; P=${C##*:}
  FARMS_PHASE_SETS=$S timeout -k 10 300 python3 -u tools/strip_rank.py --split strips --n 8 --ranks 3 --pool $P \
    ${SIM_ARGS:-} > gpurun_out/strip_s${S}_p$P.log 2>&1 || exit $?
  echo "sets $S"; tail -1 gpurun_out/strip_s${S}_p$P.log
done
exit 0
