#!/bin/bash
# hipGraph experiment on the C++-only driver (tools/graph_bench.cpp, ROCm 7.2
# runtime): config 3 with the sweeps enqueued directly, then captured into a
# graph per call (FARMS_GRAPH=1); the scale hash must agree.
cd /root/repo
mkdir -p gpurun_out
B=aperture-robust-multiscale-optical-flow_amd/build
timeout -k 10 300 $B/graph_bench 3 5 5 > gpurun_out/graph_bench_direct.log 2>&1
rc=$?; echo "direct rc=$rc"; tail -1 gpurun_out/graph_bench_direct.log
[ $rc -ne 0 ] && exit $rc
FARMS_GRAPH=1 timeout -k 10 300 $B/graph_bench 3 5 5 > gpurun_out/graph_bench_graph.log 2>&1
rc=$?; echo "graph rc=$rc"; grep "farms graph" gpurun_out/graph_bench_graph.log | tail -2; tail -1 gpurun_out/graph_bench_graph.log
exit $rc
