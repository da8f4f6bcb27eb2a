#!/bin/bash
# Candidate build A/B on one box: the default (k_cand on time-ordered streams)
# against FARMS_CAND=chain, alternating processes (tools/lib_ab.py --child, device-
# resident steps), after the candidate-build parity tests; then a kernel trace of
# the default with the pooling stream's gaps (tools/pool_gaps.py).
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=${CFG:-3}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 240 --timeout-method thread \
  -k "${TESTS:-candidate_builds or chunking or streaming or serial or unsorted}" > gpurun_out/pt_cand.log 2>&1
rc=$?; tail -2 gpurun_out/pt_cand.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for m in default chain; do
    if [ $m = default ]; then unset FARMS_CAND; else export FARMS_CAND=$m; fi
    timeout -k 10 300 python3 tools/lib_ab.py --child --config $CFG --steps ${STEPS:-4} > gpurun_out/ab_$m.tmp 2>&1 || exit $?
    echo "$m $(tail -1 gpurun_out/ab_$m.tmp)" | tee -a gpurun_out/cand_ab_c$CFG.log
  done
done
unset FARMS_CAND
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tl -o tl -- python3 tools/lib_ab.py --child --config $CFG --steps 1 \
  > gpurun_out/tl.log 2>&1 || exit $?
python3 tools/pool_gaps.py $(find gpurun_out/tl -name "*.db" | head -1) > gpurun_out/gaps_c$CFG.txt 2>&1
rc=$?; rm -rf gpurun_out/tl; head -24 gpurun_out/gaps_c$CFG.txt; tail -1 gpurun_out/gaps_c$CFG.txt
exit $rc
