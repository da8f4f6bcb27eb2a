#!/bin/bash
# Round-5 session 10: the x-strip pipeline with the asynchronous exchange
# (fit of b + 2 issued before the exchange of b + 1 is waited for; three
# workspace sets): the strip / multirank GPU tests, then the C4 N=4 middle
# strip rank against N=1.
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_strips.py tests/test_multirank.py -m gpu -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/r05_pytest_s10.log 2>&1 || exit 1
L=gpurun_out/r05_strips_s10.log
: > $L
timeout -k 10 600 python3 -u tools/strip_rank.py --config 4 --n 4 --ranks 1 --reps 3 --halo-cache /tmp/halo --host-times >> $L 2>&1 || exit 2
timeout -k 10 600 python3 -u tools/strip_rank.py --config 4 --n 1 --ranks 0 --reps 3 --split segments >> $L 2>&1 || exit 3
rm -rf /tmp/halo
exit 0
