#!/usr/bin/env python3
"""Per-kernel register/LDS/scratch usage from a hipcc --cuda-device-only -S listing.

    python tools/kmeta.py file.s [substring]
"""
import re
import sys

src = open(sys.argv[1]).read()
pat = sys.argv[2] if len(sys.argv) > 2 else ""
meta = src[src.index("amdhsa.kernels:"):]
for ent in re.split(r"\n  - ", meta)[1:]:
    name = re.search(r"\.name:\s+(\S+)", ent)
    if not name or pat not in name.group(1):
        continue
    get = lambda k: (re.search(re.escape(k) + r":\s+(\d+)", ent) or [None, "?"])[1]
    print(f"{name.group(1)[:90]:90s} sgpr {get('.sgpr_count'):>4} vgpr {get('.vgpr_count'):>4} agpr {get('.agpr_count'):>3} "
          f"spill s/v {get('.sgpr_spill_count')}/{get('.vgpr_spill_count')} lds {get('.group_segment_fixed_size')} "
          f"scratch {get('.private_segment_fixed_size')}")
