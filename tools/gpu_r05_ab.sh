#!/bin/bash
# Round-5 A/B session on one box, every GPU step under its own time limit,
# stopping at the first failure (no retries):
#   TESTS="<pytest -k expression>"  gpu tests of that selection first (optional)
#   LIBS="build/a.so build/b.so"     builds compared by tools/lib_ab.py (ABAB)
#   CFGS="3 4"                        configs of the A/B (default 3)
#   STEPS=5                           timed steps per child
# Logs: gpurun_out/r05_ab_<tag>.log (TAG, default "ab").
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-ab}
LOG=gpurun_out/r05_ab_${TAG}.log
: > $LOG
step() { echo "== $1 rc=$2" | tee -a $LOG; [ "$2" -ne 0 ] && exit "$2"; return 0; }
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -k "$TESTS" --timeout 300 --timeout-method thread \
    > gpurun_out/r05_pytest_${TAG}.log 2>&1
  rc=$?; tail -3 gpurun_out/r05_pytest_${TAG}.log | tee -a $LOG
  step pytest $rc
fi
for C in ${CFGS:-3}; do
  if [ -n "${LIBS:-}" ]; then
    timeout -k 10 900 python -u tools/lib_ab.py --config $C --steps ${STEPS:-5} --rounds ${ROUNDS:-2} $LIBS >> $LOG 2>&1
    step lib_ab_c$C $?
  fi
done
exit 0
