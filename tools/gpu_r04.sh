#!/bin/bash
# Round-4 GPU session: stages run in order, each GPU step under its own time
# limit; a failed step ends the script (no retries).
#   tests     gpu test suite            smoke    __graft_entry__.smoke()
#   bench     bench.py N=1 (BENCH_ARGS) benchpool the same with --prof pool (overhead A/B)
#   rehearse  N=2 ranks on device 0 over gloo, SPLITS
#   traffic   PMC FETCH/WRITE passes of CFG -> gpurun_out/traffic_c$CFG.json
#   sq        PMC SQ pass of CFG        -> gpurun_out/sq_c$CFG.json
#   prof      rocprofv3 --kernel-trace --stats of CFG
#   ranksim   tools/strip_rank.py, N / SPLITS / RANKS / CFG
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=${CFG:-3}
STAGES=${STAGES:-tests smoke bench}
for S in $STAGES; do
  case $S in
  tests)
    timeout -k 10 1500 python -u -m pytest tests -v -m gpu -rA --timeout 400 --timeout-method thread ${PYTEST_ARGS:-} \
      > gpurun_out/pytest_gpu.log 2>&1
    rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log ;;
  smoke)
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
    rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log ;;
  bench)
    timeout -k 10 600 python bench.py --config $CFG --steps ${STEPS:-10} --warmup 2 ${BENCH_ARGS:-} \
      > gpurun_out/bench_c$CFG.log 2>&1
    rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_c$CFG.log | cut -c1-700 ;;
  benchpool)
    timeout -k 10 600 python bench.py --config $CFG --steps ${STEPS:-10} --warmup 2 --prof pool --no-cpu-baseline \
      --host-steps 0 ${BENCH_ARGS:-} > gpurun_out/benchpool_c$CFG.log 2>&1
    rc=$?; echo "benchpool rc=$rc"; grep -o '"ms_per_step": [0-9.]*' gpurun_out/benchpool_c$CFG.log ;;
  rehearse)
    for SPLIT in ${SPLITS:-segments strips}; do
      FARMS_BENCH_DEVICE=0 FARMS_DIST_BACKEND=gloo timeout -k 10 600 python bench.py --config $CFG --gpus ${N:-2} \
        --steps 2 --warmup 1 --events ${REH_EVENTS:-5000000} --split $SPLIT ${REH_ARGS:-} \
        > gpurun_out/rehearsal_${SPLIT}_n${N:-2}_c$CFG.log 2>&1
      rc=$?; echo "rehearsal $SPLIT rc=$rc"; tail -1 gpurun_out/rehearsal_${SPLIT}_n${N:-2}_c$CFG.log | cut -c1-900
      [ $rc -ne 0 ] && break
    done ;;
  traffic)
    TRAFFIC_OUT=gpurun_out/traffic_c$CFG.json BENCH_ARGS="--config $CFG ${BENCH_ARGS:-}" bash tools/gpu_traffic.sh \
      > gpurun_out/traffic_c$CFG.out 2>&1
    rc=$?; echo "traffic rc=$rc" ;;
  sq)
    SQ_OUT=gpurun_out/sq_c$CFG.json BENCH_ARGS="--config $CFG ${BENCH_ARGS:-}" bash tools/gpu_sq.sh \
      > gpurun_out/sq_c$CFG.out 2>&1
    rc=$?; echo "sq rc=$rc" ;;
  prof)
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c$CFG -o run --output-format csv -- \
      python3 bench.py --config $CFG --steps 2 --warmup 1 --no-cpu-baseline --host-steps 0 ${BENCH_ARGS:-} \
      > gpurun_out/prof_c$CFG.log 2>&1
    rc=$?; echo "rocprof rc=$rc"; tail -1 gpurun_out/prof_c$CFG.log | cut -c1-300 ;;
  ranksim)
    for SPLIT in ${SPLITS:-strips segments}; do
      timeout -k 10 600 python3 -u tools/strip_rank.py --config $CFG --split $SPLIT --n ${N:-8} --ranks ${RANKS:-0,3,7} \
        ${SIM_ARGS:-} > gpurun_out/ranksim_${SPLIT}_n${N:-8}_c$CFG.log 2>&1
      rc=$?; echo "ranksim $SPLIT rc=$rc"; tail -2 gpurun_out/ranksim_${SPLIT}_n${N:-8}_c$CFG.log
      [ $rc -ne 0 ] && break
    done ;;
  *) echo "unknown stage $S"; rc=2 ;;
  esac
  [ $rc -ne 0 ] && exit $rc
done
exit 0
