#!/bin/bash
# Round-4 evidence on the final build, one box, every GPU step under its own
# time limit, stopping at the first failure (no retries):
#   PMC traffic + SQ summaries of the bench workload of C3, C4, C2, C5 (copied
#   into profiles/ on the box so that the bench lines read them), the gpu test
#   suite, smoke, the bench lines of C3 (with the CPU baseline and the host
#   path), C4, C2, C5, a rocprofv3 --kernel-trace --stats summary of the C3
#   bench command, and the N=2 rehearsals of both splits (gloo, one GPU).
#   ONLY_PMC=1: the PMC passes only; SKIP_PMC=1 / SKIP_TESTS=1: skip those.
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
R=r04
step() { echo "== $1 rc=$2"; [ "$2" -ne 0 ] && exit "$2"; return 0; }
if [ "${SKIP_PMC:-0}" != "1" ]; then
  CFGS="${PMC_CFGS:-3 4 2 5}" R=$R bash tools/gpu_pmc_configs.sh > gpurun_out/final_pmc.out 2>&1
  step pmc $?
  cp gpurun_out/${R}_traffic_c*.json gpurun_out/${R}_sq_c*.json profiles/
  [ "${ONLY_PMC:-0}" = "1" ] && { rm -rf gpurun_out/pmc_*; exit 0; }
fi
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 1200 python -u -m pytest tests -v -m gpu -rA --timeout 400 --timeout-method thread \
    > gpurun_out/${R}_pytest_gpu.log 2>&1
  step pytest $?
  tail -1 gpurun_out/${R}_pytest_gpu.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${R}_smoke.log 2>&1
  step smoke $?
fi
timeout -k 10 600 python -u bench.py --config 3 > gpurun_out/${R}_bench_c3.log 2>&1
step bench_c3 $?
for C in 4 2 5; do
  timeout -k 10 600 python -u bench.py --config $C --host-steps 0 > gpurun_out/${R}_bench_c$C.log 2>&1
  step bench_c$C $?
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
  python3 bench.py --config 3 --steps 2 --warmup 1 --no-cpu-baseline --host-steps 0 > gpurun_out/prof.log 2>&1
step rocprof $?
cp "$(find gpurun_out/prof -name '*kernel_stats.csv' | head -1)" gpurun_out/${R}_kernel_stats.csv
rm -rf gpurun_out/prof
for SPLIT in segments strips; do
  FARMS_BENCH_DEVICE=0 FARMS_DIST_BACKEND=gloo timeout -k 10 600 python bench.py --config 3 --gpus 2 --steps 2 \
    --warmup 1 --events 5000000 --split $SPLIT > gpurun_out/${R}_rehearsal_${SPLIT}_n2.log 2>&1
  step rehearsal_$SPLIT $?
done
rm -rf gpurun_out/pmc_*
exit 0
