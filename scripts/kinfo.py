#!/usr/bin/env python3
"""Register / scratch / spill summary of the gfx950 kernels in a built .so or .o (code-object notes).
Usage: scripts/kinfo.py <lib.so|obj.o> [name-substring ...]"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def code_objects(path):
    tmp = tempfile.mkdtemp()
    src = path
    if path.endswith(".so"):
        src = os.path.join(tmp, "fatbin")
        subprocess.check_call([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={src}", path,
                               os.path.join(tmp, "copy.so")])
    else:  # a hipcc -c object: the bundle sits in .hip_fatbin as well
        src = os.path.join(tmp, "fatbin")
        subprocess.check_call([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={src}", path,
                               os.path.join(tmp, "copy.o")])
    data = open(src, "rb").read()
    starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
    for i, st in enumerate(starts):
        part = os.path.join(tmp, f"b{i}")
        open(part, "wb").write(data[st:starts[i + 1] if i + 1 < len(starts) else len(data)])
        co = part + ".co"
        subprocess.check_call([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={part}",
                               "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"])
        yield co


def main():
    path, keys = sys.argv[1], sys.argv[2:]
    for co in code_objects(path):
        out = subprocess.check_output([f"{LLVM}/llvm-readobj", "--notes", co], text=True)
        for blk in out.split(".name:")[1:]:
            name = blk.split("\n")[0].strip()
            if keys and not any(k in name for k in keys):
                continue

            def g(k):
                m = re.search(r"\." + k + r":\s+(\d+)", blk)
                return m.group(1) if m else "?"
            print(f"{name[:70]:70s} vgpr {g('vgpr_count'):>3} sgpr {g('sgpr_count'):>3} scratch "
                  f"{g('private_segment_fixed_size'):>4} spill v {g('vgpr_spill_count')} s {g('sgpr_spill_count')}")


if __name__ == "__main__":
    main()
