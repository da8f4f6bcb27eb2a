#!/bin/bash
# Round-5 breakdown of the x-strip step at BASELINE config 4 (N = 4, the middle
# rank 1: two halos) against the N = 1 step, each under a rocprofv3 kernel
# trace (tools/strip_trace.py splits the traced steps into phases).  The halo
# flows are fitted once and cached on the box (/tmp, not gpurun_out: 400 MB),
# so that the traced run holds only the rank's own kernels.
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
LOG=gpurun_out/r05_strips_c4.log
: > $LOG
step() { echo "== $1 rc=$2" | tee -a $LOG; [ "$2" -ne 0 ] && exit "$2"; return 0; }
if [ "${SKIP_STRIP:-0}" != "1" ]; then
timeout -k 10 600 python3 -u tools/strip_rank.py --config 4 --n 4 --ranks 1 --reps 2 --halo-cache /tmp/halo \
  >> $LOG 2>&1
step strip_rank $?
timeout -k 10 600 rocprofv3 --kernel-trace -d gpurun_out/kt_strip -o kt --output-format csv -- \
  python3 -u tools/strip_rank.py --config 4 --n 4 --ranks 1 --reps 1 --halo-cache /tmp/halo >> $LOG 2>&1
step trace_strip $?
python3 tools/strip_trace.py gpurun_out/kt_strip/kt_kernel_trace.csv --timeline --label "C4 N=4 strips, rank 1" \
  > gpurun_out/r05_strip_trace_c4.txt 2>&1
step analyse_strip $?
fi
timeout -k 10 600 rocprofv3 --kernel-trace -d gpurun_out/kt_n1 -o kt --output-format csv -- \
  python3 -u tools/strip_rank.py --config 4 --n 1 --ranks 0 --reps 1 --split segments >> $LOG 2>&1
step trace_n1 $?
python3 tools/strip_trace.py gpurun_out/kt_n1/kt_kernel_trace.csv --timeline --label "C4 N=1" \
  > gpurun_out/r05_n1_trace_c4.txt 2>&1
step analyse_n1 $?
rm -rf gpurun_out/kt_strip gpurun_out/kt_n1 /tmp/halo
exit 0
