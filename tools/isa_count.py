#!/usr/bin/env python3
"""Static instruction mix of one kernel in a device assembly file
(hipcc --cuda-device-only -S): counts per mnemonic, issue slots (a 64-bit
multiply-add, v_mul_lo/hi_u32 and v_lshl_add_u64 issue at half rate,
DESIGN.md §4), memory and branch counts.
  tools/isa_count.py FILE.s KERNEL_REGEX [--top N]"""
import re
import sys
from collections import Counter

HALF = ("v_mad_u64_u32", "v_mul_lo_u32", "v_mul_hi_u32", "v_lshl_add_u64", "v_mad_i64_i32", "v_mul_u32_u24")


def body(path, pat):
    lines = open(path).read().split("\n")
    rx = re.compile(pat)
    start = None
    for i, ln in enumerate(lines):
        if start is None and re.match(r"^_Z\S*:", ln) and rx.search(ln.split(":")[0]):
            start, name = i, ln.split(":")[0]
        elif start is not None and ln.startswith(".Lfunc_end"):
            return name, lines[start:i + 1]
    raise SystemExit(f"no kernel matching {pat}")


def main():
    path, pat = sys.argv[1], sys.argv[2]
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 25
    name, b = body(path, pat)
    ops = Counter()
    for ln in b:
        t = ln.strip()
        if not t or t.startswith((";", ".", "_")) or t.endswith(":"):
            continue
        ops[t.split()[0]] += 1
    valu = {k: v for k, v in ops.items() if k.startswith("v_")}
    half = sum(v for k, v in valu.items() if k.startswith(HALF))
    nvalu = sum(valu.values())
    vmem = sum(v for k, v in ops.items() if k.startswith(("global_", "buffer_")))
    lds = sum(v for k, v in ops.items() if k.startswith("ds_"))
    salu = sum(v for k, v in ops.items() if k.startswith("s_"))
    br = sum(v for k, v in ops.items() if k.startswith(("s_cbranch", "s_branch")))
    print(f"{name}\n  VALU {nvalu} (half-rate {half}; issue slots {nvalu + half}), VMEM {vmem}, LDS {lds}, "
          f"SALU {salu}, branches {br}")
    for k, v in sorted(valu.items(), key=lambda kv: -kv[1])[:top]:
        print(f"    {v:6d} {k}")


if __name__ == "__main__":
    main()
