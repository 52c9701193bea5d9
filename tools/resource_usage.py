"""Per-kernel register / scratch / occupancy table from hipcc's kernel-resource-usage remarks."""
import re
import subprocess
import sys
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# usage: resource_usage.py [source.hip] [extra hipcc flags]; default mgx_api.hip; mgx_pgs.hip gets
# its own per-TU flags (native.SOURCE_FLAGS)
args = sys.argv[1:]
name = args.pop(0) if args and args[0].endswith(".hip") else "mgx_api.hip"
src = os.path.join(ROOT, "mujoco_gymnasium_environments_amd", "csrc", name)
sys.path.insert(0, ROOT)
from mujoco_gymnasium_environments_amd.native import SOURCE_FLAGS  # noqa: E402
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c", "-o", "/tmp/_ru.o", src,
       "-Rpass-analysis=kernel-resource-usage"] + SOURCE_FLAGS.get(name, []) + args
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"remark: (.*?): (.*?) \[-Rpass", line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2).strip()
    if k == "Function Name":
        cur = v
        rows[cur] = {}
    elif cur:
        rows[cur][k] = v
keys = ["VGPRs", "AGPRs", "ScratchSize [bytes/lane]", "Occupancy [waves/SIMD]", "SGPRs Spill", "VGPRs Spill", "LDS Size [bytes/block]"]
for name, r in rows.items():
    short = re.sub(r"^_Z\d+", "", name)[:40]
    print(f"{short:42s} " + " ".join(f"{k.split()[0]}={r.get(k, '?')}" for k in keys))
