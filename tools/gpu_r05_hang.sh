#!/bin/bash
# Round-5: the fixed idle-half descriptor: the strip guard sequence + phase-2
# repro, rank 1 of the C3 strip step, the 2-rank strip step, then the pooling /
# candidate / strip / multirank GPU tests.  Stops at the first failure.
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
L=gpurun_out/r05_hang.log
echo "== sequence repro" > $L
timeout -k 10 200 python3 -u tools/pool_phase2_repro.py --strip-first >> $L 2>&1
rc=$?; echo "rc=$rc" >> $L; [ $rc -ne 0 ] && exit $rc
echo "== strips rank 1 (one process)" >> $L
timeout -k 10 300 python3 -u tools/strip_rank.py --config 3 --n 2 --ranks 1 --events 120000 --reps 1 >> $L 2>&1
rc=$?; echo "rc=$rc" >> $L; [ $rc -ne 0 ] && exit $rc
echo "== 2 processes, strips" >> $L
timeout -k 10 200 python3 -u tools/strips_hip_ranks.py >> $L 2>&1
rc=$?; echo "rc=$rc" >> $L; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python3 -u -m pytest tests -x -v -m gpu -k "pair or pool or strip or cand or chunk or gloo or multirank" --timeout 150 --timeout-method thread > gpurun_out/r05_pytest_hangfix.log 2>&1
rc=$?; tail -3 gpurun_out/r05_pytest_hangfix.log >> $L; exit $rc
