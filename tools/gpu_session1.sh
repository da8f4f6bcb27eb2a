#!/bin/bash
# Round session: gpu tests + bench + kernel-trace stats (gpu_round.sh), then the
# PMC traffic passes (gpu_traffic.sh).  Stops at the first failure.
cd /root/repo
REHEARSE=${REHEARSE:-0} bash tools/gpu_round.sh && bash tools/gpu_traffic.sh
