#!/usr/bin/env python3
"""Per-kernel register / spill / LDS use of a built object (gfx950 code object notes).
Usage: python3 tools/kres.py <obj.o> [name-substring]"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"


def notes(obj):
    with tempfile.TemporaryDirectory() as d:
        fb, co = os.path.join(d, "f.fatbin"), os.path.join(d, "k.co")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", obj, os.path.join(d, "h")], check=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fb}",
                        f"--targets={TARGET}", f"--output={co}"], check=True)
        return subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True, text=True).stdout


def main():
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    keys = ("sgpr_count", "sgpr_spill_count", "vgpr_count", "vgpr_spill_count", "private_segment_fixed_size")
    for b in notes(sys.argv[1]).split("  - ."):
        m = re.search(r"\.name:\s+(\S+)", b)
        if not m or sub not in m.group(1) or ".sgpr_count" not in b:
            continue
        vals = {k: (re.search(r"\." + k + r":\s+(\S+)", b) or [None, None])[1] for k in keys}
        print(m.group(1), vals)


if __name__ == "__main__":
    main()
