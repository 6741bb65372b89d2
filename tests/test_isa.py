"""Codegen pins of the in-kernel hand-offs: the last-arriver pattern
(csrc/tsdf_resolve.h arrive_last) orders a workgroup's published records before its arrival with a
raw s_waitcnt vmcnt(0) and a workgroup barrier, relying on the agent-scope (sc1) stores being counted
in vmcnt -- not on a release fence, whose gfx950 form (buffer_wbl2 sc1: an L2 writeback per
workgroup) costs the frame. These checks read the gfx950 code object of the built library and assert
that every arrival atomic of the frame kernels is preceded by a barrier with no global store between
the two, and that a vmcnt(0) wait precedes that barrier; and that the publishing stores and the last
arriver's loads carry the agent-scope bit (sc1). CPU only (llvm-objdump on the built .so)."""
import os
import re
import shutil
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "disinfect-slam_amd", "libdisinfect_tsdf.so")
LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _disassemble():
    if not os.path.exists(LIB) or not os.path.exists(os.path.join(LLVM, "llvm-objdump")):
        pytest.skip("library or llvm tools absent")
    tmp = tempfile.mkdtemp()
    try:
        fb = os.path.join(tmp, "fatbin")
        subprocess.check_call([os.path.join(LLVM, "llvm-objcopy"), f"--dump-section=.hip_fatbin={fb}", LIB,
                               os.path.join(tmp, "copy.so")])
        data = open(fb, "rb").read()
        starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
        text = []
        for i, st in enumerate(starts):
            part = os.path.join(tmp, f"b{i}")
            with open(part, "wb") as f:
                f.write(data[st:starts[i + 1] if i + 1 < len(starts) else len(data)])
            co = part + ".co"
            subprocess.check_call([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o",
                                   f"--input={part}", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                                   f"--output={co}"])
            text.append(subprocess.check_output([os.path.join(LLVM, "llvm-objdump"), "-d", co], text=True))
        return "\n".join(text)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def _functions(asm):
    funcs, name = {}, None
    for line in asm.splitlines():
        m = re.match(r"^[0-9a-f]+ <(\S+)>:$", line)
        if m:
            name = m.group(1)
            funcs[name] = []
        elif name and line.startswith("\t"):
            funcs[name].append(line.strip())
    return funcs


def test_arrivals_follow_a_drained_barrier():
    funcs = _functions(_disassemble())
    frame = {n: body for n, body in funcs.items()
             if "k_ingest_dda" in n or "k_integrate_t" in n or "k_integrate_vg" in n}
    assert len(frame) >= 8, sorted(funcs)[:20]
    checked = 0
    for name, body in frame.items():
        for i, ins in enumerate(body):
            # the arrivals: returning 64-bit adds on the counters (first level, then the top counter)
            if not (ins.startswith("global_atomic_add_x2") and ins.split("//")[0].rstrip().endswith("sc0")):
                continue
            j = max(k for k in range(i) if body[k].startswith("s_barrier"))
            between = body[j + 1:i]
            assert not any(b.startswith(("global_store", "flat_store", "buffer_store")) for b in between), \
                (name, between)
            window = body[max(0, j - 60):j]
            assert any(re.match(r"s_waitcnt\b.*vmcnt\(0\)", w) for w in window), (name, window[-10:])
            checked += 1
    assert checked >= 16


def test_publication_is_agent_scope():
    """st_co / ld_co: the new-key list, the candidate records and the arrival counters' readers use
    sc1 (agent scope) so the last arriver on another XCD reads them from the coherent level."""
    funcs = _functions(_disassemble())
    ing = next(b for n, b in funcs.items() if n.startswith("_ZN4tsdf12k_ingest_ddaILi1024"))
    integ = next(b for n, b in funcs.items() if n.startswith("_ZN4tsdf13k_integrate_tILb0ELb0"))
    assert any(i.startswith("global_store_dwordx2") and "sc1" in i for i in ing)   # nk_list entries
    assert any(i.startswith("global_load_dwordx2") and "sc1" in i for i in ing)    # resolver prologue
    assert any(i.startswith("global_store_dwordx2") and "sc1" in i for i in integ)  # candidate records
    # k_integrate_vg: the view-grid cells its grid workgroups write are written through (the carving's
    # last arriver clears some of them after every arrival: its stores must be the cells' last writes)
    vg = next(b for n, b in funcs.items() if n.startswith("_ZN4tsdf14k_integrate_vg"))
    assert any(i.startswith("global_store_dword ") and "sc1" in i for i in vg)


def _kframe():
    funcs = _functions(_disassemble())
    names = [n for n in funcs if n.startswith("_ZN4tsdf7k_frame")]
    assert names, sorted(funcs)[:20]
    return funcs[names[0]]


def _addr(ins):
    m = re.search(r"//\s*([0-9A-F]+):", ins)
    return int(m.group(1), 16) if m else None


def test_k_frame_flags_follow_a_drained_barrier():
    """k_frame (the pipelined frame, tsdf_fuse.hip): workgroup 0 publishes the carving and then the
    allocation (the combined fast path: both after one drain) with one flag per XCD (publish_flags: an agent-scope atomic exchange, the kernel's only
    global_atomic_swap_x2). Every flag must follow a workgroup barrier with no global store or atomic
    between them, and a vmcnt(0) wait must come before that barrier (drain_barrier): the table /
    free-stack / new-key / rtag writes the flags publish are complete when another XCD sees the tag."""
    body = _kframe()
    # (non-returning: a returning swap, sc0, is a bucket lock of the hash-level resolver path)
    swaps = [i for i, ins in enumerate(body) if ins.startswith("global_atomic_swap_x2")
             and not ins.split("//")[0].rstrip().endswith("sc0")]
    assert len(swaps) >= 2, "carving and allocation flags"
    for i in swaps:
        j = max(k for k in range(i) if body[k].startswith("s_barrier"))
        # (the head's fast path publishes the carving and the allocation after one drain: the other
        # flag's swaps may sit between the barrier and this one)
        between = [b for k, b in enumerate(body[j + 1:i], j + 1) if k not in swaps]
        assert not any(b.startswith(("global_store", "flat_store", "buffer_store", "global_atomic"))
                       for b in between), between
        window = body[max(0, j - 40):j]
        assert any(re.match(r"s_waitcnt\b.*vmcnt\(0\)", w) for w in window), window[-10:]


def test_k_frame_hand_offs_are_agent_scope():
    """The carving / allocation outputs other XCDs read in the same launch are written through (sc1):
    table entries as three sc1 dwords (store_ent_co), never a plain 16-bit offset store (store_off);
    new-key-list / fresh-list / candidate records as sc1 dwordx2. Every flag poll (a loop with
    s_sleep: wait_tag, the fresh workgroups, the deferred blocks) reads with an sc1 load or an atomic,
    never a plain load (it would be served from this CU's L1 / the XCD's L2 forever)."""
    body = _kframe()
    assert not any(ins.startswith("global_store_short") for ins in body), "plain store_off in k_frame"
    def addr(x):  # the address operands of a global store (vaddr, saddr / off)
        ops = x.split("//")[0].split()[1:]
        return (ops[0].rstrip(","), ops[2].rstrip(",")) if len(ops) >= 3 else None

    ok = 0
    sc1 = [i for i, x in enumerate(body) if x.startswith("global_store_dword ") and "sc1" in x]
    for i in sc1:
        a = body[i]
        if "offset:" in a.split("//")[0]:
            continue
        near = [body[k] for k in sc1 if i < k <= i + 6 and addr(body[k]) == addr(a)]
        if any("offset:4 " in x for x in near) and any("offset:8 " in x for x in near):
            ok += 1
    assert ok >= 1, "store_ent_co (3 sc1 dwords) not found"
    assert sum(1 for ins in body if ins.startswith("global_store_dwordx2") and "sc1" in ins) >= 6
    polls = 0
    for i, ins in enumerate(body):
        if not ins.startswith("s_sleep"):
            continue
        # the loop around the sleep: the next backward branch
        here = _addr(ins)
        for k in range(i + 1, min(len(body), i + 80)):
            m = re.match(r"s_c?branch\S*\s+(-?\d+)", body[k])
            if not m:
                continue
            off = int(m.group(1))
            off = off - 65536 if off >= 32768 else off
            tgt = _addr(body[k]) + 4 + 4 * off
            if tgt > here:
                continue
            loop = [x for x in body if _addr(x) is not None and tgt <= _addr(x) <= _addr(body[k])]
            loads = [x for x in loop if x.startswith(("global_load", "buffer_load", "flat_load"))]
            atomics = [x for x in loop if x.startswith("global_atomic")]
            assert loads or atomics, loop[:12]
            assert all("sc1" in x for x in loads), [x for x in loads if "sc1" not in x]
            polls += 1
            break
    assert polls >= 3, polls


def _loops(body):
    """(first, last) instruction indices of every backward branch's loop body."""
    addrs = []
    for x in body:
        m = re.search(r"// ([0-9A-F]+):", x)
        addrs.append(int(m.group(1), 16) if m else None)
    base = addrs[0]
    idx = {a: i for i, a in enumerate(addrs) if a is not None}
    for i, x in enumerate(body):
        if re.match(r"s_cbranch_\w+|s_branch", x):
            t = re.search(r"<\S+\+0x([0-9a-f]+)>", x)
            j = idx.get(base + int(t.group(1), 16)) if t and base is not None else None
            if j is not None and j < i:
                yield j, i


def test_update_loops_keep_their_state_in_registers():
    """The voxel-update loops of k_integrate_t and k_frame (three 16-B pool loads, the reciprocal
    estimates) keep their state in registers: a spilled value there is re-read for every block (round 4:
    the __shfl_xor lane addresses of the carve minimum and an indexed band-start array were spilled, 100s
    of scratch accesses per iteration, and made the update ~30 % slower). Since round 6 the loops carry
    the semantic update's exact float chain at 6 waves per SIMD (80 VGPRs); a few loop-invariant
    reloads remain (<= 12 scratch instructions in an iteration of 1,500-2,800 -- measured: 0-12, the
    interleaved semantic pass, same speed as the 0-5 of the pair-by-pair form), nothing more.
    k_raycast uses no scratch at all."""
    funcs = _functions(_disassemble())
    seen = set()
    for name, body in funcs.items():
        kern = next((k for k in ("_ZN4tsdf7k_frame", "_ZN4tsdf9k_frame_g", "_ZN4tsdf13k_integrate_t",
                                 "_ZN4tsdf14k_integrate_vg") if name.startswith(k)), None)
        if kern:
            for j, i in _loops(body):
                ops = [x.split()[0] for x in body[j:i + 1]]
                if i - j < 4000 and ops.count("global_load_dwordx4") >= 3 and "v_rcp_f32_e32" in ops:
                    seen.add(kern)
                    assert sum(o.startswith("scratch_") for o in ops) <= 12, (name, j, i)
        if name.startswith("_ZN4tsdf9k_raycast"):
            assert not any(x.startswith("scratch_") for x in body), name
    assert seen == {"_ZN4tsdf7k_frame", "_ZN4tsdf9k_frame_g", "_ZN4tsdf13k_integrate_t",
                    "_ZN4tsdf14k_integrate_vg"}, seen


def test_frame_kernels_make_no_calls():
    """Every device function of the frame kernels is inlined: a real call (s_swappc) passes the
    kernel's EngineDev by reference, so the kernel first copies it (240 B per lane) to scratch and
    the callee reads every field from there (round 4: pipe_update grew past the inliner's threshold
    and the k_frame update ran from scratch)."""
    funcs = _functions(_disassemble())
    kernels = [n for n in funcs if n.startswith(("_ZN4tsdf7k_frame", "_ZN4tsdf9k_frame_g", "_ZN4tsdf13k_integrate_t",
                                                 "_ZN4tsdf14k_integrate_vg", "_ZN4tsdf12k_ingest_dda",
                                                 "_ZN4tsdf9k_raycast"))]
    assert kernels
    for name in kernels:
        assert not any(x.startswith("s_swappc") for x in funcs[name]), name
