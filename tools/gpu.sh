#!/bin/bash
# One GPU session step per call, each under its own time limit; chain steps
# with && in the gpurun command so that the first failure ends the session:
#   tools/gpu.sh TAG pytest [PYTEST ARGS...]    GPU tests (default: the whole -m gpu suite)
#   tools/gpu.sh TAG smoke                      __graft_entry__.smoke()
#   tools/gpu.sh TAG bench [BENCH ARGS...]      one bench.py line
#   tools/gpu.sh TAG ab CONFIG STEPS LIB...     tools/lib_ab.py: builds side by side, alternating
#   tools/gpu.sh TAG stats [BENCH ARGS...]      rocprofv3 --kernel-trace --stats of a bench run
#   tools/gpu.sh TAG serial [BENCH ARGS...]     FARMS_SERIALIZE=1 kernel timeline (no overlap)
#   tools/gpu.sh TAG trace [BENCH ARGS...]      kernel trace of one bench step, tools/trace_gaps.py summary
#   tools/gpu.sh TAG sq [BENCH ARGS...]         one --pmc pass of 8 SQ counters -> TAG_sq.json
#   tools/gpu.sh TAG traffic [BENCH ARGS...]    FETCH_SIZE / WRITE_SIZE passes -> TAG_traffic.json
#   tools/gpu.sh TAG ranksim [strip_rank.py ARGS...]
# Outputs go to gpurun_out/TAG_<step>.*  (copied into profiles/ when kept).
# FARMS_HIP_LIB (env) picks another engine build for every step.
cd /root/repo || exit 9
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; STEP=$2; shift 2
O=gpurun_out/${TAG}_${STEP}
PROF_ARGS="--steps 1 --warmup 0 --no-cpu-baseline --host-steps 0"
KREGEX="k_pool|k_fit|k_chain|k_cand|k_flow"
case $STEP in
pytest)
  [ $# -eq 0 ] && set -- tests
  timeout -k 10 ${PYTEST_LIMIT:-1000} python3 -u -m pytest "$@" -m gpu -x -v --timeout ${TEST_TIMEOUT:-300} \
    --timeout-method thread > $O.log 2>&1
  rc=$?; tail -3 $O.log ;;
smoke)
  timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O.log 2>&1
  rc=$?; tail -2 $O.log ;;
bench)
  timeout -k 10 ${BENCH_LIMIT:-600} python3 -u bench.py "$@" > $O.log 2>&1
  rc=$?; tail -1 $O.log | cut -c1-600 ;;
ab)
  CFG=$1; K=$2; shift 2
  timeout -k 10 ${AB_LIMIT:-900} python3 -u tools/lib_ab.py --config $CFG --steps $K "$@" > $O.log 2>&1
  rc=$?; cat $O.log | tail -12 ;;
stats)
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O -o kt --output-format csv -- \
    python3 bench.py --no-cpu-baseline "$@" > $O.log 2>&1
  rc=$?; tail -1 $O.log | cut -c1-300 ;;
serial)
  FARMS_SERIALIZE=1 timeout -k 10 400 rocprofv3 --kernel-trace -d $O -o kt --output-format csv -- \
    python3 bench.py $PROF_ARGS "$@" > $O.log 2>&1
  rc=$?
  if [ $rc -eq 0 ]; then python3 tools/timeline.py $O/kt_kernel_trace.csv > $O.txt; rc=$?; grep -E "span|busy|k_|rocprim" $O.txt | head -20 || true; fi ;;
trace)
  timeout -k 10 400 rocprofv3 --kernel-trace -d $O -o kt --output-format csv -- \
    python3 bench.py $PROF_ARGS "$@" > $O.log 2>&1
  rc=$?
  if [ $rc -eq 0 ]; then python3 tools/trace_gaps.py $O/kt_kernel_trace.csv --call ${CALL:-0} > $O.txt; rc=$?; head -40 $O.txt; fi ;;
sq)
  CTRS="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD"
  timeout -s KILL 600 rocprofv3 --pmc $CTRS --kernel-include-regex "$KREGEX" -d $O -o pmc --output-format csv -- \
    python3 bench.py $PROF_ARGS "$@" > $O.log 2>&1
  rc=$?
  if [ $rc -eq 0 ]; then python3 tools/sq_summary.py $O/pmc_counter_collection.csv --label "bench.py $PROF_ARGS $*" > $O.json; rc=$?; fi ;;
traffic)
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 600 rocprofv3 --pmc $C --kernel-include-regex "$KREGEX" -d ${O}_$C -o pmc --output-format csv -- \
      python3 bench.py $PROF_ARGS "$@" > ${O}_$C.log 2>&1
    rc=$?; [ $rc -ne 0 ] && break
  done
  if [ $rc -eq 0 ]; then python3 tools/traffic.py ${O}_FETCH_SIZE/pmc_counter_collection.csv \
    ${O}_WRITE_SIZE/pmc_counter_collection.csv --label "bench.py $PROF_ARGS $*" > $O.json; rc=$?; fi ;;
ranksim)
  timeout -k 10 600 python3 -u tools/strip_rank.py "$@" > $O.log 2>&1
  rc=$?; tail -6 $O.log ;;
*)
  echo "unknown step $STEP"; exit 9 ;;
esac
echo "[$TAG $STEP] rc=$rc"
exit $rc
