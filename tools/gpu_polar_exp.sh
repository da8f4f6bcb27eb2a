#!/bin/bash
# Round-4 experiment: k_true_polar on the chain stream.
#   A: the events that mark a super-chunk's records final (ev_pool / gpool,
#      the host path's download trigger, w.done) stay on the pooling stream,
#      recorded before k_true_polar runs -- the round-3 arrangement;
#   B: the same launch placement with those events recorded after
#      k_true_polar on the chain stream.
# Both builds come from the current engine by /tmp/tp/mk.py-style patches
# (built in the container as build/libfarms_hip_polar{A,B}.so).  The bitwise
# host-path, chunking and pipeline tests run once per build; test failures are
# the expected outcome for A (exit 1 continues), anything else stops.
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
for V in A B; do
  FARMS_HIP_LIB=build/libfarms_hip_polar$V.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -v -m gpu \
    -k "host_path or chunking or streaming" --timeout 300 --timeout-method thread > gpurun_out/polar_$V.log 2>&1
  rc=$?; echo "variant $V pytest rc=$rc"; tail -3 gpurun_out/polar_$V.log
  [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
done
exit 0
