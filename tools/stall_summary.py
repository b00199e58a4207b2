"""Per-kernel stall / issue account of a 1-stream headline wave from the counter
groups of tools/diag_stall_step.sh (one rocprofv3 --pmc run per group).

    python tools/stall_summary.py <diag_stall_step OUTDIR> [name-filter]

Per kernel (name + grid), averaged over its dispatches:
  kcyc     GRBM_GUI_ACTIVE / 8 XCDs per dispatch (kernel cycles)
  MHz      effective clock = kcyc / dispatch time (when the CSV carries timestamps)
  valu     VALU busy = SQ_ACTIVE_INST_VALU * 4 / 1024 SIMDs / kcyc (the fraction of the
           SIMDs' issue cycles spent issuing VALU; MI355X_MICROARCH.md 'rocprofv3 PMC slots')
  wait / winst / act
           SQ_WAIT_ANY, SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES (disjoint)
  VALU/VMEM/LDS per wave
           SQ_INSTS_* / SQ_WAVES
  L2hit    TCC_HIT / (TCC_HIT + TCC_MISS)
"""
import collections
import csv
import glob
import re
import sys


def short(name, grid):
    m = re.search(r"(\w+)<([^()]*)>", name)
    n = f"{m.group(1)}<{m.group(2)}>" if m else name.split("(")[0]
    return f"{n} grid {grid}"


def main(root, filt=""):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for f in sorted(glob.glob(f"{root}/p*/**/*counter_collection.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"], r.get("Grid_Size", "?"))
            if filt and filt not in k:
                continue
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            if r.get("Start_Timestamp") and r.get("End_Timestamp") and r["Counter_Name"] == "GRBM_GUI_ACTIVE":
                dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    mean = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in vals.items()}
    rows = []
    for k, m in mean.items():
        g = m.get("GRBM_GUI_ACTIVE")
        if not g:
            continue
        kc = g / 8
        wc = m.get("SQ_WAVE_CYCLES") or 0
        waves = m.get("SQ_WAVES") or 0
        hit, miss = m.get("TCC_HIT_sum"), m.get("TCC_MISS_sum")
        t = sum(dur[k]) / len(dur[k]) if dur.get(k) else None
        rows.append((kc, k, {
            "kcyc": kc / 1e3,
            "MHz": kc / t / 1e6 if t else None,
            "valu": m.get("SQ_ACTIVE_INST_VALU", 0) * 4 / 1024 / kc,
            "wait": m.get("SQ_WAIT_ANY", 0) / wc if wc else None,
            "winst": m.get("SQ_WAIT_INST_ANY", 0) / wc if wc else None,
            "act": m.get("SQ_ACTIVE_INST_ANY", 0) / wc if wc else None,
            "valu/w": m.get("SQ_INSTS_VALU", 0) / waves if waves else None,
            "vmem/w": (m.get("SQ_INSTS_VMEM_RD", 0) + m.get("SQ_INSTS_VMEM_WR", 0)) / waves if waves else None,
            "lds/w": m.get("SQ_INSTS_LDS", 0) / waves if waves else None,
            "L2hit": hit / (hit + miss) if hit is not None and miss else None,
        }))
    rows.sort(reverse=True)
    cols = ["kcyc", "MHz", "valu", "wait", "winst", "act", "valu/w", "vmem/w", "lds/w", "L2hit"]
    print(f"{'kernel':72s} " + " ".join(f"{c:>7s}" for c in cols))
    for _, k, d in rows:
        print(f"{k[:72]:72s} " + " ".join(f"{d[c]:7.2f}" if isinstance(d[c], float) else f"{'-':>7s}" for c in cols))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
