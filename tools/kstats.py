"""Per-kernel time table from a rocprofv3 --kernel-trace --stats output dir.

    python tools/kstats.py DIR [steps]
"""
import csv
import glob
import re
import sys


def short(name):
    m = re.search(r"(\w+)<([^()]*)>", name)
    return f"{m.group(1)}<{m.group(2)}>" if m else name.split("(")[0]


def main(d, steps=None):
    f = glob.glob(f"{d}/**/*kernel_stats.csv", recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"{'kernel':60s} {'calls':>6s} {'avg_us':>9s} {'total_ms':>9s} {'pct':>6s}" +
          (f" {'ms/step':>8s}" if steps else ""))
    for r in rows:
        t = float(r["TotalDurationNs"])
        line = (f"{short(r['Name'])[:60]:60s} {r['Calls']:>6s} {float(r['AverageNs'])/1e3:9.1f} "
                f"{t/1e6:9.3f} {100*t/tot:6.1f}")
        if steps:
            line += f" {t/1e6/steps:8.3f}"
        print(line)


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else None)
