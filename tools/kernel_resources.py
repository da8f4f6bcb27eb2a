#!/usr/bin/env python3
"""Register / LDS / scratch use of the gfx950 kernels in build/libfarms_hip.so
(reads the code object's metadata notes; tuning aid)."""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = sys.argv[1] if len(sys.argv) > 1 and sys.argv[1] else os.path.join(ROOT, "aperture-robust-multiscale-optical-flow_amd/build/libfarms_hip.so")
pat = sys.argv[2] if len(sys.argv) > 2 else r"k_"
with tempfile.TemporaryDirectory() as d:
    fat, co = os.path.join(d, "fat.bin"), os.path.join(d, "g.co")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", lib, os.devnull], check=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
    notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True).stdout
cur = {}
rows = []
for line in notes.splitlines():
    if line.startswith("  - ."):  # a new kernel record
        if cur:
            rows.append(cur)
        cur = {}
    m = re.match(r"(?:  - |    )\.(\w+):\s+(.*)", line)
    if m:
        cur[m.group(1)] = m.group(2)
if cur:
    rows.append(cur)
for r in rows:
    name = r.get("name", "")
    if not re.search(pat, name) or "rocprim" in name:
        continue
    short = re.search(r"(k_\w+?)(?:ILi(\d+)E)?E", name)
    nm = f"{short.group(1)}<{short.group(2)}>" if short and short.group(2) else (short.group(1) if short else name)
    print(f"{nm:22s} vgpr {r.get('vgpr_count', '?'):>4s} agpr {r.get('agpr_count', '?'):>3s} sgpr {r.get('sgpr_count', '?'):>4s} "
          f"lds {r.get('group_segment_fixed_size', '?'):>6s} scratch {r.get('private_segment_fixed_size', '?'):>5s} "
          f"spill {r.get('vgpr_spill_count', '?')}")
