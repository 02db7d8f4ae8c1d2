#!/usr/bin/env python3
"""Per-kernel register / LDS / scratch usage from a hipcc --save-temps .s (amdhsa metadata).

    python tools/kstats.py /tmp/logreg-hip-amdgcn-amd-amdhsa-gfx950.s [name-filter]
"""
import re
import subprocess
import sys

src = open(sys.argv[1]).read()
flt = sys.argv[2] if len(sys.argv) > 2 else ""
meta = src[src.find("amdhsa.kernels:"):]
for blk in re.split(r"\n\s+- \.", meta)[1:]:
    f = dict(re.findall(r"\.(\w+):\s+([^\n]+)", "." + blk))
    name = f.get("name", "?")
    if flt and flt not in name:
        continue
    try:
        dem = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
    except OSError:
        dem = name
    print(f"vgpr {f.get('vgpr_count','?'):>4} agpr {f.get('agpr_count','?'):>4} sgpr {f.get('sgpr_count','?'):>4} "
          f"lds {f.get('group_segment_fixed_size','?'):>6} scratch {f.get('private_segment_fixed_size','?'):>4}  {dem[:110]}")
