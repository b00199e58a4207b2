"""Per-kernel time and HBM bytes of the headline op (CKKS mul+relin at the metric
config, waves of 128) from three rocprofv3 runs of tools/op_bench.py ckks_mul:
a kernel trace, a FETCH_SIZE pass and a WRITE_SIZE pass (tools/gpu_steps.sh
steppmc).  Writes profiles/step_traffic.json, which bench.py puts into its
line as the `step` block.

    python tools/step_summary.py TRACE_DIR FETCH_DIR WRITE_DIR OUT_DIR [CALL_REGEX WORKLOAD]

(another op: CALL_REGEX names the kernel launched once per call, e.g.
"behz_floor" for bfv_mul; profiles/step_traffic.json is then left alone)

A call of op_bench is one wave (128 ct-mults); calls are counted by the
PRO_TENSOR inverse row pass (one per call).  HBM bytes follow
MI355X_MICROARCH.md: FETCH_SIZE (KB) x 1024 x 2 (gfx950 reports half of a wide
streaming read), WRITE_SIZE (KB) x 1024.  The input fills (fill_kernel) are
excluded, and so are the context's table uploads (the runtime's copyBuffer blits
that run before the first fill: fhe_ctx_create, not the op loop).
"""
import collections
import csv
import glob
import json
import os
import re
import sys

TENSOR = re.compile(r"true, false, true, [25](, \d)?>")  # PRO_TENSOR or PRO_TENSOR2


def short(name):
    m = re.search(r"(\w+)<([^()]*)>", name)
    return f"{m.group(1)}<{m.group(2)}>" if m else name.split("(")[0]


def trace(d, TENSOR=TENSOR):
    f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
    per, calls = collections.defaultdict(lambda: [0, 0.0]), 0
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    first_fill = next((int(r["Start_Timestamp"]) for r in rows if "fill_kernel" in r["Kernel_Name"]), 0)
    for r in rows:
        n = r["Kernel_Name"]
        if "fill_kernel" in n or int(r["Start_Timestamp"]) < first_fill:
            continue
        calls += bool(TENSOR.search(n))
        k = (short(n), int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"]))
        per[k][0] += 1
        per[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    return per, calls


def counters(d, name, scale, TENSOR=TENSOR):
    out, calls, seen = collections.defaultdict(float), 0, set()
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            if r["Counter_Name"] != name or "fill_kernel" in n:
                continue
            key = (f, r["Dispatch_Id"])
            if TENSOR.search(n) and key not in seen:
                calls += 1
            seen.add(key)
            out[(short(n), int(r["Grid_Size"]))] += float(r["Counter_Value"]) * scale
    return out, calls


def main(tdir, fdir, wdir, dst, marker=None, workload=None):
    mk = re.compile(marker) if marker else TENSOR
    per, calls = trace(tdir, mk)
    fetch, fc = counters(fdir, "FETCH_SIZE", 1024 * 2, mk)
    write, wc = counters(wdir, "WRITE_SIZE", 1024, mk)
    wave = 128
    rows = []
    for k, (cnt, ms) in per.items():
        b = fetch.get(k, 0.0) / max(fc, 1) + write.get(k, 0.0) / max(wc, 1)
        t = ms / calls
        rows.append({"kernel": k[0], "grid": k[1], "launches_per_wave": cnt / calls, "ms_per_wave": round(t, 4),
                     "hbm_MB_per_wave": round(b / 1e6, 1), "TBps": round(b / (t * 1e-3) / 1e12, 3) if t else None})
    rows.sort(key=lambda r: -r["ms_per_wave"])
    tot_ms = sum(r["ms_per_wave"] for r in rows)
    tot_b = sum(r["hbm_MB_per_wave"] for r in rows) * 1e6
    res = {
        "source": os.path.relpath(dst, os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
        "workload": workload or "tools/op_bench.py ckks_mul --batch 128 (N=2^16, L=12, K=4, dnum=3), one stream",
        "wave": wave, "calls_traced": calls, "calls_counted": [fc, wc],
        "kernel_ms_per_wave": round(tot_ms, 4),
        "hbm_bytes_per_wave": round(tot_b),
        "hbm_bytes_per_ct_mult": round(tot_b / wave),
        "kernel_TBps": round(tot_b / (tot_ms * 1e-3) / 1e12, 3),
        "dominant": rows[0] if rows else None,
        "kernels": rows,
        "note": "FETCH_SIZE x 2 (gfx950 half-count of wide streaming reads), WRITE_SIZE as is; fill kernels and the context's setup uploads excluded",
    }
    os.makedirs(dst, exist_ok=True)
    json.dump(res, open(os.path.join(dst, "step_summary.json"), "w"), indent=1)
    top = os.path.join(os.path.dirname(dst.rstrip("/")), "step_traffic.json")
    if not marker:
      json.dump({k: res[k] for k in ("source", "workload", "wave", "kernel_ms_per_wave", "hbm_bytes_per_ct_mult",
                                     "kernel_TBps", "dominant")}, open(top, "w"), indent=1)
    print(f"{'kernel':52s} {'grid':>9s} {'n/wave':>6s} {'ms':>7s} {'MB':>8s} {'TB/s':>6s}")
    for r in rows:
        print(f"{r['kernel']:52s} {r['grid']:9d} {r['launches_per_wave']:6.2f} {r['ms_per_wave']:7.3f} "
              f"{r['hbm_MB_per_wave']:8.1f} {r['TBps'] or 0:6.2f}")
    print(f"total {tot_ms:.3f} ms/wave, {tot_b / 1e9:.3f} GB/wave, {tot_b / wave / 1e6:.1f} MB/ct-mult")


if __name__ == "__main__":
    main(*sys.argv[1:7])
