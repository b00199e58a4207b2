"""Average kernel time per variant from rocprofv3 --stats runs (tools/gpu_cmd_kp.sh).

    python tools/kstat_cmp.py OUT var... [--filter SUBSTR ...]
"""
import csv
import sys


def main():
    args = sys.argv[1:]
    out, rest = args[0], args[1:]
    flt = []
    if "--filter" in rest:
        i = rest.index("--filter")
        rest, flt = rest[:i], rest[i + 1:]
    stats = {}
    for v in rest:
        stats[v] = {}
        for r in csv.DictReader(open(f"{out}/{v}/run_kernel_stats.csv")):
            n = r["Name"]
            n = n.replace("(anonymous namespace)::", "").replace("void ", "")
            n = n.split("(")[0]
            stats[v][n] = float(r["AverageNs"]) / 1e3
    names = sorted(stats[rest[0]], key=lambda n: -stats[rest[0]][n])
    print(f"{'kernel (avg us)':60s} " + " ".join(f"{v:>9s}" for v in rest))
    for n in names:
        if flt and not any(f in n for f in flt):
            continue
        print(f"{n[:60]:60s} " + " ".join(f"{stats[v].get(n, float('nan')):9.1f}" for v in rest))


if __name__ == "__main__":
    main()
