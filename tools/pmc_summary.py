"""Summarise rocprofv3 --pmc CSVs: per kernel, mean counter value per dispatch.

    python tools/pmc_summary.py <dir-with-pass-subdirs> [name-filter]
"""
import collections
import csv
import glob
import re
import sys


def short(name):
    m = re.search(r"(\w+)<([^()]*)>", name)
    if m:
        return f"{m.group(1)}<{m.group(2)}>"
    return name.split("(")[0]


def main(root, filt=""):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(f"{root}/*/run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            name = short(r["Kernel_Name"])
            if filt and filt not in name:
                continue
            agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for name, cs in agg.items():
        print(name)
        for cn, vals in sorted(cs.items()):
            print(f"   {cn:30s} {sum(vals)/len(vals):16.1f}  (n={len(vals)})")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
