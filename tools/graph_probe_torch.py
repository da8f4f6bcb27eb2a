"""Runs tools/graph_capture_probe.hip's probe inside a process that imported
torch first, so the probe binds PyTorch's bundled HIP runtime (as the engine
does under Python) instead of /opt/rocm's."""
import ctypes
import os
import sys

import torch

lib = ctypes.CDLL(os.path.join(os.path.dirname(__file__), "..", "aperture-robust-multiscale-optical-flow_amd",
                               "build", "libgraph_probe.so"))
lib.graph_probe_run.argtypes = [ctypes.c_double]
print("torch", torch.__version__, flush=True)
sys.exit(lib.graph_probe_run(float(sys.argv[1]) if len(sys.argv) > 1 else 3000.0))
