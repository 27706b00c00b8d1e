"""VGPRs, AGPRs, scratch (register spills) and occupancy of every kernel of csrc/geobpe.hip for
gfx950, from the compiler's resource-usage remarks (device-only compile, nothing written).

  python tools/kernel_resources.py [filter] [-- extra hipcc flags]"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
argv = sys.argv[1:]
extra = argv[argv.index("--") + 1:] if "--" in argv else []
flt = argv[0] if argv and argv[0] != "--" else ""
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only", "-c", "-o",
       "/dev/null", "-Rpass-analysis=kernel-resource-usage", *extra, os.path.join(ROOT, "pt-bpe_amd/csrc/geobpe.hip")]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = {}, None
for ln in out.splitlines():
    m = re.search(r"Function Name: (\S+)", ln)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+([A-Za-z ]+?)(?: \[[^]]*\])?: (\d+)", ln)
    if m and cur:
        rows[cur][m.group(1).strip()] = int(m.group(2))
for k, v in sorted(rows.items()):
    if "k_" in k and flt in k:
        print(f"{k[:64]:64s} vgpr {v.get('VGPRs', 0):4d} agpr {v.get('AGPRs', 0):3d} "
              f"scratch {v.get('ScratchSize', 0):4d} B/lane (vgpr spill {v.get('VGPRs Spill', 0)}, sgpr spill "
              f"{v.get('SGPRs Spill', 0)})  occ {v.get('Occupancy', 0)}  lds {v.get('LDS Size', 0)}")
