#!/bin/bash
# Round-3 GPU session: gpu test suite, smoke, bench N=1, and N=2 rehearsals on
# the one-GPU box (both ranks on device 0, gloo for the collectives) whose
# parity block crosses the rank boundary.  Every GPU step has its own time
# limit; a failed step ends the script (no retries).
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
STAGES=${STAGES:-tests smoke bench rehearse}
for S in $STAGES; do
  case $S in
  tests)
    timeout -k 10 1500 python -u -m pytest tests -v -m gpu -rA --timeout 400 --timeout-method thread \
      > gpurun_out/pytest_gpu.log 2>&1
    rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log ;;
  smoke)
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
    rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log ;;
  bench)
    timeout -k 10 600 python bench.py --steps ${STEPS:-10} --warmup 2 ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
    rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-600 ;;
  rehearse)
    for SPLIT in ${SPLITS:-segments strips}; do
      FARMS_BENCH_DEVICE=0 FARMS_DIST_BACKEND=gloo timeout -k 10 600 python bench.py --gpus ${N:-2} --steps 2 \
        --warmup 1 --events ${REH_EVENTS:-5000000} --split $SPLIT ${REH_ARGS:-} \
        > gpurun_out/rehearsal_${SPLIT}_n${N:-2}.log 2>&1
      rc=$?; echo "rehearsal $SPLIT rc=$rc"; grep -o '"parity".*' gpurun_out/rehearsal_${SPLIT}_n${N:-2}.log | cut -c1-900
      [ $rc -ne 0 ] && break
    done ;;
  prof)
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
      python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --host-steps 0 ${BENCH_ARGS:-} > gpurun_out/prof.log 2>&1
    rc=$?; echo "rocprof rc=$rc"; tail -1 gpurun_out/prof.log | cut -c1-300 ;;
  ranksim)  # N=8 rank simulations (tools/strip_rank.py): strips ranks 0, 3, 7; segments rank 3
    timeout -k 10 500 python3 -u tools/strip_rank.py --split strips --n 8 --ranks ${RANKS:-0,3,7} \
      > gpurun_out/ranksim_strips_n8.log 2>&1
    rc=$?; echo "ranksim strips rc=$rc"; tail -1 gpurun_out/ranksim_strips_n8.log
    [ $rc -ne 0 ] && exit $rc
    timeout -k 10 300 python3 -u tools/strip_rank.py --split segments --n 8 --ranks 3 \
      > gpurun_out/ranksim_segments_n8.log 2>&1
    rc=$?; echo "ranksim segments rc=$rc"; tail -1 gpurun_out/ranksim_segments_n8.log ;;
  ab)  # device-resident C3 step for each "pool_chunk:pool_batch" in AB_CASES
    for C in ${AB_CASES:-8192:64 4096:64 4096:128}; do
      timeout -k 10 300 python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --host-steps 0 \
        --pool-chunk ${C%%:*} --pool-batch ${C##*:} > gpurun_out/ab_${C/:/_}.log 2>&1
      rc=$?; echo "ab $C rc=$rc"; grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_${C/:/_}.log
      [ $rc -ne 0 ] && break
    done ;;
  *) echo "unknown stage $S"; rc=2 ;;
  esac
  [ $rc -ne 0 ] && exit $rc
done
exit 0
