"""Per-step kernel table of the headline bench from a rocprofv3 kernel trace.

    python tools/step_table.py gpurun_out/prof/bench STEPS

Takes the LAST `STEPS` ct-mult steps of the trace (a step starts at the
tensor-prologue INTT row pass), so the roofline-loop launches are excluded.
Kernels are keyed by (short name, grid) so the NTT of the ModUp digits, of conv
and of acc_P show up as separate rows.
"""
import csv
import glob
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"(\w+)<([^()]*)>", name)
    return f"{m.group(1)}<{m.group(2)}>" if m else name.split("(")[0]


def main(d, steps):
    f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    # a step starts at the tensor-prologue INTT row pass (EPI 2) and ends at its
    # ModDown-finish row pass (EPI 1, or 6..9 with the fused inner product);
    # round-3 kernels carry a trailing lazy-schedule parameter
    starts = [i for i, r in enumerate(rows) if re.search(r"true, false, true, 2(, \d)?>", r["Kernel_Name"])]
    first = starts[-steps]
    last = max(i for i, r in enumerate(rows) if re.search(r"false, false, true, [16789](, \d)?>", r["Kernel_Name"]))
    agg = defaultdict(lambda: [0, 0.0, 0, 0])
    for r in rows[first:last + 1]:
        k = (short(r["Kernel_Name"]), int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]))
        a = agg[k]
        a[0] += 1
        a[1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        a[2], a[3] = int(r["VGPR_Count"]), int(r["LDS_Block_Size"])
    span = (int(rows[last]["End_Timestamp"]) - int(rows[first]["Start_Timestamp"])) / 1e6 / steps
    tot = sum(a[1] for a in agg.values()) / steps
    print(f"{'kernel':52s} {'grid':>9s} {'vgpr':>5s} {'ms/step':>8s} {'share':>6s}")
    for (name, grid), a in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{name:52s} {grid:9d} {a[2]:5d} {a[1] / steps:8.3f} {a[1] / steps / tot:6.1%}")
    print(f"kernel sum {tot:.3f} ms/step; wall span {span:.3f} ms/step")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 5)
