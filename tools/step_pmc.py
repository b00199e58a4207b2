"""Per-kernel PMC account of one headline wave (bench.py --streams 1): HBM bytes
(FETCH_SIZE x2 gfx950 correction + WRITE_SIZE), VALU instructions, and the
kernel's effective GB/s from its trace duration.

    python tools/step_pmc.py gpurun_out/pmcstep gpurun_out/pmcstepf gpurun_out/pmcstepw
"""
import collections
import csv
import glob
import re
import sys


def short(name):
    m = re.search(r"(\w+)<([^()]*)>", name)
    return f"{m.group(1)}<{m.group(2)}>" if m else name.split("(")[0]


def load(d):
    out = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)  # dispatches per kernel key
    for f in glob.glob(f"{d}/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            k = (short(r["Kernel_Name"]), r["Grid_Size"])
            out[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add((f, r["Dispatch_Id"]))
    return out, collections.Counter({k: len(v) for k, v in disp.items()})


def main(valu_dir, fetch_dir, write_dir):
    v, nv = load(valu_dir)
    f, nf = load(fetch_dir)
    w, nw = load(write_dir)
    rows = []
    for k in v:
        if "fill_kernel" in k[0]:
            continue
        n = max(nv[k], 1)
        grbm = v[k]["GRBM_GUI_ACTIVE"] / n / 8
        fetch = f[k]["FETCH_SIZE"] / max(nf[k], 1) * 1024 * 2
        write = w[k]["WRITE_SIZE"] / max(nw[k], 1) * 1024
        valu = v[k]["SQ_INSTS_VALU"] / n
        busy = v[k]["SQ_ACTIVE_INST_VALU"] / n * 4 / 1024 / grbm if grbm else 0
        rows.append((k[0], int(k[1]), n, grbm, (fetch + write) / 1e6, valu / 1e6, busy))
    print(f"{'kernel':52s} {'grid':>9s} {'n':>3s} {'kcyc/disp':>10s} {'HBM MB':>8s} {'VALU M':>7s} {'valu_busy':>9s}")
    for r in sorted(rows, key=lambda r: -r[3] * r[2]):
        print(f"{r[0]:52s} {r[1]:9d} {r[2]:3d} {r[3] / 1e3:10.1f} {r[4]:8.1f} {r[5]:7.2f} {r[6]:9.2f}")


if __name__ == "__main__":
    main(*sys.argv[1:4])
