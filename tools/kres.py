"""Per-kernel register / scratch / occupancy summary of a built library's gfx950
code objects (llvm-objdump --offloading + llvm-readelf --notes).

    python tools/kres.py herdsman_amd/lib/libherdsman_fhe.so [name-filter]
"""
import glob
import os
import re
import shutil
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def main(lib, filt=""):
    tmp = tempfile.mkdtemp()
    try:
        src = os.path.join(tmp, os.path.basename(lib))
        shutil.copy(lib, src)
        subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", src], cwd=tmp, capture_output=True, check=True)
        for co in sorted(glob.glob(src + ".*gfx950*")):
            notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True).stdout
            for blk in notes.split("  - .agpr_count")[1:]:
                g = lambda k: (re.search(rf"\.{k}:\s+(\S+)", blk) or [None, "?"])[1]
                name = g("name")
                if filt and filt not in name:
                    continue
                v = int(g("vgpr_count"))
                lds = g("group_segment_fixed_size")
                occ = min(8, 512 // (((v + 7) // 8) * 8)) if v else 8
                print(f"{name[:90]:90s} vgpr {v:4d} (waves/SIMD by VGPR {occ}) spill {g('vgpr_spill_count')} "
                      f"scratch {g('private_segment_fixed_size')} lds {lds}")
    finally:
        shutil.rmtree(tmp)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
