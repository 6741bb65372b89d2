#!/usr/bin/env python3
"""Does the voxel-update loop of the frame kernels touch scratch? (tests/test_isa.py's check, on any
built .so / .o). Usage: scripts/loopscratch.py <lib.so|obj.o>"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import test_isa  # noqa: E402

test_isa.LIB = sys.argv[1]
funcs = test_isa._functions(test_isa._disassemble())
for name, body in funcs.items():
    if not name.startswith(("_ZN4tsdf7k_frame", "_ZN4tsdf9k_frame_g", "_ZN4tsdf13k_integrate_t", "_ZN4tsdf14k_integrate_vg")):
        continue
    for j, i in test_isa._loops(body):
        ops = [x.split()[0] for x in body[j:i + 1]]
        if i - j < 4000 and ops.count("global_load_dwordx4") >= 3 and "v_rcp_f32_e32" in ops:
            sc = sum(o.startswith("scratch_") for o in ops)
            rl = sum(o.startswith("v_readlane") for o in ops)
            print(f"{name[:40]:40s} loop {i - j:5d} instrs, scratch {sc}, readlane {rl}")
