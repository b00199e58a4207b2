"""SQ_INSTS_VALU per ct-mult of one op, summed over the kernels of its calls,
from rocprofv3 --pmc 'SQ_INSTS_VALU SQ_WAVES' runs of tools/op_bench.py
(tools/gpu_steps.sh valu=V1,V2,...; one directory per library variant).

    python tools/valu_count.py ROOT V1 [V2 ...] [--batch 128]

Per kernel (name + grid): dispatches per call, waves, VALU instructions per
wave and per ct-mult; the total per ct-mult, and each variant against the
first.  Calls are counted by the inverse row pass with the tensor prologue
(PRO_TENSOR / PRO_TENSOR2, one per call; BFV: the BEHZ floor / HPS scaling); the input fills and the context's
table uploads (everything before the first fill) are excluded.
"""
import collections
import csv
import glob
import re
import sys

# one dispatch per op call: the CKKS tensor prologue (PRO_TENSOR / PRO_TENSOR2),
# the BFV floor (BEHZ) or the HPS scaling
TENSOR = re.compile(r"ntt_pass<\d+, 8, 4, 16, true, false, (true|false), [25](, \d)?>|behz_floor_kernel|hps_scale_kernel")


def short(name, grid):
    m = re.search(r"(\w+)<([^()]*)>", name)
    n = f"{m.group(1)}<{m.group(2)}>" if m else name.split("(")[0]
    return f"{n} grid {grid}"


def account(d, batch):
    f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
    if not f:
        raise SystemExit(f"no counter_collection.csv under {d}")
    rows = list(csv.DictReader(open(f[0])))
    rows.sort(key=lambda r: int(r.get("Dispatch_Id") or 0))
    first_fill = next((int(r["Dispatch_Id"]) for r in rows if "fill_kernel" in r["Kernel_Name"]), 0)
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    calls = set()
    for r in rows:
        n = r["Kernel_Name"]
        did = int(r["Dispatch_Id"])
        if "fill_kernel" in n or did < first_fill or "copyBuffer" in n:
            continue
        k = short(n, r.get("Grid_Size", "?"))
        per[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(did)
        if TENSOR.search(n):
            calls.add(did)
    nc = max(1, len(calls))
    out = {}
    for k, cs in per.items():
        valu, waves = cs.get("SQ_INSTS_VALU", 0.0), cs.get("SQ_WAVES", 0.0)
        out[k] = {"disp_per_call": len(disp[k]) / nc, "valu_per_wave": valu / waves if waves else 0.0,
                  "valu_per_ct": valu / nc / batch}
    return out, nc


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    batch = int(sys.argv[sys.argv.index("--batch") + 1]) if "--batch" in sys.argv else 128
    if "--batch" in sys.argv:
        args.remove(str(batch))
    root, vs = args[0], args[1:]
    accs = {}
    for v in vs:
        accs[v], nc = account(f"{root}/{v}", batch)
        tot = sum(x["valu_per_ct"] for x in accs[v].values())
        print(f"== {v}: {nc} calls of {batch} ct-mults, {tot / 1e6:.3f} M VALU instructions per ct-mult")
        for k, x in sorted(accs[v].items(), key=lambda kv: -kv[1]["valu_per_ct"]):
            print(f"   {x['valu_per_ct'] / 1e6:8.3f} M/ct  {x['valu_per_wave']:8.0f}/wave  {x['disp_per_call']:4.1f}/call  {k[:90]}")
    if len(vs) > 1:
        t0 = sum(x["valu_per_ct"] for x in accs[vs[0]].values())
        for v in vs[1:]:
            t = sum(x["valu_per_ct"] for x in accs[v].values())
            print(f"{v} against {vs[0]}: {t / 1e6:.3f} / {t0 / 1e6:.3f} M per ct-mult = {t / t0:.4f} ({100 * (t / t0 - 1):+.1f}%)")


if __name__ == "__main__":
    main()
