#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output into markdown for profiles/.

    python tools/prof_summary.py stats  <run_kernel_stats.csv>          # per-kernel time
    python tools/prof_summary.py pmc    <dir with set*/run_counter_collection.csv>

The PMC mode averages every counter per kernel over its dispatches (counters
are per-dispatch totals) and adds derived ratios when the inputs exist:
TCC hit rate, HBM read/write bytes per dispatch (EA requests x 64 B), VALU /
VMEM / LDS instruction mix.
"""
from __future__ import annotations

import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(name: str) -> str:
    name = name.replace('"', "").replace("pga::(anonymous namespace)::", "").replace("void ", "")
    name = re.sub(r"\(.*\)$", "", name)
    return name[:90]


def stats(path: str) -> str:
    rows = list(csv.DictReader(open(path)))
    out = ["| kernel | calls | avg us | min us | max us | % time |", "|---|---|---|---|---|---|"]
    for r in rows:
        out.append(f"| `{short(r['Name'])}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | "
                   f"{float(r['MinNs']) / 1e3:.1f} | {float(r['MaxNs']) / 1e3:.1f} | {float(r['Percentage']):.2f} |")
    return "\n".join(out)


def pmc(d: str) -> str:
    acc = defaultdict(lambda: defaultdict(list))
    meta = {}
    for f in sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            meta[k] = (r["Grid_Size"], r["Workgroup_Size"], r["VGPR_Count"], r["SGPR_Count"], r["LDS_Block_Size"],
                       r["Scratch_Size"])
    out = []
    for k, cs in sorted(acc.items(), key=lambda kv: -len(next(iter(kv[1].values())))):
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        g, wg, vgpr, sgpr, lds, scr = meta[k]
        out.append(f"### `{k}`\n\ngrid {g}, workgroup {wg}, VGPR {vgpr}, SGPR {sgpr}, LDS {lds} B, scratch {scr} B\n")
        out.append("| counter | avg per dispatch |\n|---|---|")
        for c in sorted(avg):
            out.append(f"| {c} | {avg[c]:.4g} |")
        der = []
        if "TCC_HIT_sum" in avg and "TCC_MISS_sum" in avg and avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"] > 0:
            der.append(f"L2 hit rate {avg['TCC_HIT_sum'] / (avg['TCC_HIT_sum'] + avg['TCC_MISS_sum']):.1%}")
        # fabric bytes from the request-size split when the pass collected it
        # (an L2 read request is 32, 64 or 128 B, a write 32 or 64 B); else
        # the request count at 64 B, a lower bound for 128-B row reads
        if "TCC_EA0_RDREQ_sum" in avg:
            n = avg["TCC_EA0_RDREQ_sum"]
            if "TCC_EA0_RDREQ_128B_sum" in avg and "TCC_EA0_RDREQ_64B_sum" in avg:
                b128, b64 = avg["TCC_EA0_RDREQ_128B_sum"], avg["TCC_EA0_RDREQ_64B_sum"]
                rd = 128 * b128 + 64 * b64 + 32 * max(0.0, n - b128 - b64)
                der.append(f"fabric read {rd / 1e6:.1f} MB ({b128 / max(n, 1):.1%} of requests 128 B)")
            else:
                der.append(f"fabric read >= {n * 64 / 1e6:.1f} MB (requests x 64 B)")
        if "TCC_EA0_WRREQ_sum" in avg:
            n = avg["TCC_EA0_WRREQ_sum"]
            if "TCC_EA0_WRREQ_64B_sum" in avg:
                w64 = avg["TCC_EA0_WRREQ_64B_sum"]
                der.append(f"fabric write {(64 * w64 + 32 * max(0.0, n - w64)) / 1e6:.1f} MB")
            else:
                der.append(f"fabric write ≈ {n * 64 / 1e6:.1f} MB (requests x 64 B)")
        if "SQ_INSTS_VALU" in avg and "SQ_WAVES" in avg and avg["SQ_WAVES"]:
            der.append(f"VALU insts/wave {avg['SQ_INSTS_VALU'] / avg['SQ_WAVES']:.0f}")
        if "SQ_WAIT_ANY" in avg and "SQ_WAVE_CYCLES" in avg and avg["SQ_WAVE_CYCLES"]:
            der.append(f"wave cycles waiting {avg['SQ_WAIT_ANY'] / avg['SQ_WAVE_CYCLES']:.1%}")
        if der:
            out.append("\nDerived: " + "; ".join(der) + "\n")
        out.append("")
    return "\n".join(out)


if __name__ == "__main__":
    mode, path = sys.argv[1], sys.argv[2]
    print(stats(path) if mode == "stats" else pmc(path))
