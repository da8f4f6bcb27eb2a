#!/bin/bash
# hipGraph capture-cost probe (tools/graph_capture_probe.hip), default stack size.
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 180 aperture-robust-multiscale-optical-flow_amd/build/graph_capture_probe ${LIMIT_MS:-4000} > gpurun_out/graph_probe.log 2>&1
rc=$?; echo "graph probe rc=$rc"; tail -4 gpurun_out/graph_probe.log
exit $rc
