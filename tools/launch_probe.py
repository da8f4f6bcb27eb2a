"""Runs tools/launch_probe.hip's probe under the HIP runtime the engine binds:
`python tools/launch_probe.py torch` imports torch first (its bundled runtime), plain: /opt/rocm's."""
import ctypes
import os
import sys

if len(sys.argv) > 1 and sys.argv[1] == "torch":
    import torch  # noqa: F401
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "build", "liblaunch_probe.so"))
sys.stdout.flush()
sys.exit(lib.launch_probe(int(os.environ.get("ITERS", "2000"))))
