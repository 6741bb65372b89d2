#!/usr/bin/env python3
"""ISA summary of a kernel in a HIP object (diagnostic, CPU only): for each backward branch (a loop)
the instruction mix of its body -- VALU, SALU, readlane / writelane (SGPR spill traffic), scratch.
usage: isa_loops.py <file.o> <kernel-name-substring>"""
import collections
import re
import subprocess
import sys
import tempfile
import os

LLVM = "/opt/rocm/lib/llvm/bin"


def disasm(obj):
    tmp = tempfile.mkdtemp()
    fb = os.path.join(tmp, "fatbin")
    subprocess.check_call([os.path.join(LLVM, "llvm-objcopy"), f"--dump-section=.hip_fatbin={fb}", obj,
                           os.path.join(tmp, "copy.o")])
    data = open(fb, "rb").read()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    starts = [m.start() for m in re.finditer(re.escape(magic), data)] + [len(data)]
    text = []
    for i in range(len(starts) - 1):
        part = os.path.join(tmp, f"b{i}")
        open(part, "wb").write(data[starts[i]:starts[i + 1]])
        co = part + ".co"
        subprocess.check_call([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o",
                               f"--input={part}", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"])
        text.append(subprocess.check_output([os.path.join(LLVM, "llvm-objdump"), "-d", co], text=True))
    return "\n".join(text)


def main():
    obj, name = sys.argv[1], sys.argv[2]
    asm = disasm(obj)
    func, body = None, []
    for line in asm.splitlines():
        m = re.match(r"^([0-9a-f]+) <(\S+)>:$", line)
        if m:
            if func and name in func:
                break
            func, body = m.group(2), []
        elif func and line.startswith("\t"):
            m2 = re.search(r"// ([0-9A-F]+):", line)
            body.append((int(m2.group(1), 16) if m2 else None, line.strip()))
    addr = {a: i for i, (a, _) in enumerate(body) if a is not None}
    print(func, len(body), "instructions")
    for i, (a, ins) in enumerate(body):
        m = re.match(r"s_cbranch_\w+|s_branch", ins)
        t = re.search(r"<\S+\+0x([0-9a-f]+)>", ins)
        if not m or not t:
            continue
        base = body[0][0]
        tgt = base + int(t.group(1), 16) - 0  # offsets are relative to the function start
        # find the function start address: first instruction's address minus its offset (0)
        j = addr.get(tgt)
        if j is None or j >= i:
            continue
        c = collections.Counter()
        for _, x in body[j:i + 1]:
            op = x.split()[0]
            if op.startswith("v_readlane") or op.startswith("v_writelane"):
                c["lane_rw"] += 1
            if op.startswith("scratch_"):
                c["scratch"] += 1
            if op.startswith("v_"):
                c["valu"] += 1
            elif op.startswith("s_nop"):
                c["nop"] += 1
            elif op.startswith("s_"):
                c["salu"] += 1
            elif op.startswith(("global_", "buffer_", "flat_")):
                c["vmem"] += 1
            elif op.startswith("ds_"):
                c["lds"] += 1
        print(f"loop [{j}, {i}] len {i - j + 1}: {dict(c)}")


if __name__ == "__main__":
    main()
