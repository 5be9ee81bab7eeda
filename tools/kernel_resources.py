"""Print VGPR/SGPR/LDS/scratch per kernel of a gfx950 code object
(`hipcc --cuda-device-only --no-gpu-bundle-output -c X.hip -o X.co`).
Usage: python tools/kernel_resources.py X.co [substring ...]"""
import re
import subprocess
import sys

LLVM = "/opt/rocm/lib/llvm/bin"
notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", sys.argv[1]], capture_output=True,
                       text=True).stdout
keys = ["vgpr_count", "agpr_count", "sgpr_count", "group_segment_fixed_size",
        "private_segment_fixed_size", "vgpr_spill_count"]
recs, cur = [], None
for line in notes.splitlines():
    m = re.match(r"\s+-?\s*\.(\w+):\s+(.*)", line)
    if not m:
        continue
    k, v = m.group(1), m.group(2).strip()
    if k == "name":
        cur = {"name": v}
        recs.append(cur)
    elif cur is not None and k in keys:
        cur[k] = v
subs = sys.argv[2:]
for r in recs:
    dem = subprocess.run(["c++filt", r["name"]], capture_output=True, text=True).stdout.strip()
    if subs and not any(s in dem for s in subs):
        continue
    print(f"{dem[:70]:70s} " + " ".join(f"{k.split('_')[0]}={r.get(k, '-')}" for k in keys))
