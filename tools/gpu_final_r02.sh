#!/bin/bash
# Round-2 closing evidence on one box, each GPU step under its own limit, stopping
# at the first failure: the smoke, the evidence set (gpu suite, PMC traffic, SQ,
# bench, kernel stats), the other configs' bench lines, and N=8 rank simulations.
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_evidence.sh || exit $?
bash tools/gpu_configs_r02.sh || exit $?
if [ "${RANKSIM:-1}" = "1" ]; then
  bash tools/gpu_ranksim.sh || exit $?
fi
exit 0
