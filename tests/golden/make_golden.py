#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/ (run from the repo root, CPU only).

1. kat_reference.json -- the known-answer vectors the reference's own tests hold for this path,
   transcribed as data: utils/tests/voxel_hash_test.cu (Single :56-92, Multiple :94-126,
   Collision :128-180) and utils/tests/voxel_mem_test.cu (Test1 :38-90). They are the only golden
   facts the reference ships; the reference itself is CUDA + Eigen + OpenCV and
   cannot be built or run here, so no reference-generated integrate output exists.
2. integrate_48x36.npz -- a small synthetic stream (inputs stored verbatim: rgb, depth, ht, lt,
   poses, intrinsics) and the CPU oracle's outputs after every frame (per-frame counters) and at
   the end (active hash entries, free-block stack, voxel state of every live block, raycast images,
   Query result). Pins the oracle against drift (tests/test_golden.py) and gives the GPU tests a
   fixed target that needs no oracle call (tests/test_gpu_golden.py). "Parity unpinned" applies:
   these outputs are the restatement's, not the reference's.
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "disinfect-slam_amd"))

# ---- 1. reference KATs (data only) ----
KAT = {
    "source": "utils/tests/voxel_hash_test.cu, utils/tests/voxel_mem_test.cu (yuzhou42/disinfect-slam)",
    "num_bucket": 1 << 21,
    "hash": [  # voxel_hash_test.cu:133-135: three block keys that land in the last bucket
        {"key": [33, 180, 42], "bucket": (1 << 21) - 1},
        {"key": [61, 16, 170], "bucket": (1 << 21) - 1},
        {"key": [63, 171, 45], "bucket": (1 << 21) - 1},
    ],
    "collision": {  # voxel_hash_test.cu:128-180: block_pos[0..3] -- three keys of the last bucket
        # and {0, 0, 0} -- go to ONE Allocate<<<1, 4>>> launch (all four keys), three times
        # (:139, :145, :151), with ResetLocks after each; the active count is 2, 3, 4 (:143, :149,
        # :155) whatever order the four threads run in. Then the first voxel of each block gets
        # rgb = weight = i (:157-161) and is retrieved (:171-179).
        "keys": [[33, 180, 42], [61, 16, 170], [63, 171, 45], [0, 0, 0]],
        "launches": 3,
        "active_after_each": [2, 3, 4],
        "assign_rgbw": [[i, i, i, i] for i in range(4)],
    },
    "single": {  # voxel_hash_test.cu:56-92
        "allocate": [1, 1, 1], "retrieve_point": [8, 8, 8], "expect_block": [1, 1, 1],
        "empty_point": [0, 0, 0], "expect_empty_weight": 0,
        "assign": [[[0, 0, i], [i, i, i, i]] for i in range(8)],
    },
    "multiple": {"n": 128},  # voxel_hash_test.cu:94-126: diagonal blocks (i, i, i), voxel (i,i,i,i)
    "mem_pool": {  # voxel_mem_test.cu:38-90: acquire -> init weight 0; set weight; release
        "num_blocks_log2": 12, "init_weight": 0, "init_tsdf": -1.0, "init_prob": 0.5,
    },
}


def make_integrate(touch="complement", nframes=6, bits=11):
    from _oracle import OracleGrid
    from tsdf_amd import synth

    W, H, voxel, trunc = 48, 36, 0.02, 0.08
    cam = synth.camera(W, H, synth.TUM_FR1)
    ora = OracleGrid(voxel, trunc, bits)
    rgb, depth, ht, lt, q, t, stats = [], [], [], [], [], [], []
    for f in range(nframes):
        fr = synth.render(cam, 3 * f, touch=touch)
        ora.integrate(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], 4.0, cam.K, fr["q"], fr["t"])
        s = ora.stats()
        assert not s["pool_exhausted"], (touch, f)
        stats.append([s["last_num_visible"], s["last_num_updated"], s["last_num_deleted"],
                      s["active_blocks"]])
        rgb.append(fr["rgb"]); depth.append(fr["depth"]); ht.append(fr["ht"]); lt.append(fr["lt"])
        q.append(fr["q"]); t.append(fr["t"])
    d = ora.dump()
    live = np.flatnonzero(d["entry_idx"] >= 0)
    idx = d["entry_idx"][live]
    blk = lambda a: a.reshape(-1, 512, *a.shape[1:])[idx]
    rq, rt = q[-1], t[-1]
    rgba, normal = ora.raycast(cam.K, W, H, rq, rt, 4.0)
    query = ora.query(None)
    out = dict(
        W=W, H=H, voxel=voxel, trunc=trunc, num_block_bits=bits, max_depth=4.0, touch=touch,
        K=np.asarray(cam.K, np.float32),
        rgb=np.stack(rgb), depth=np.stack(depth), ht=np.stack(ht), lt=np.stack(lt),
        q=np.stack(q).astype(np.float32), t=np.stack(t).astype(np.float32),
        stats=np.asarray(stats, np.int64),
        live_entry=live.astype(np.int32), live_pos=d["entry_pos"][live], live_idx=idx,
        heap=d["heap"], free=np.int32(d["free"]),
        tsdf=blk(d["tsdf"]), prob=blk(d["prob"]), rgbw=blk(d["rgbw"]),
        rgba=rgba, normal=normal, query_count=np.int64(query.shape[0]),
        query_sha256=np.frombuffer(hashlib.sha256(np.ascontiguousarray(query)).digest(), np.uint8),
        query_head=query[:2048],
    )
    ora.close()
    return out


# 3. the semantic streams: ht / lt as two independent channels over (0, 1] with the
#    extremes 1e-6, 1 - 1e-6, the largest float below 1 and 1; and uint16 / 65535 PNG maps with exact
#    zeros (lt only, and both channels: the reference's 0 / 0 NaN), 40 frames so that much of the
#    surface reaches the weight cap (40)
SEMANTIC = {"independent": "integrate_48x36_independent.npz", "u16": "integrate_48x36_u16.npz",
            "u16z": "integrate_48x36_u16z.npz"}

# 4. sem_math_digests.json -- the oracle's logf / expf (oracle/ora_math.c) digested over every input
#    bit pattern in chunks of 2^24 (ora_math_digest), the target of the GPU restatement's exhaustive
#    check (tests/test_gpu_numerics.py); kind 2 (the update's p and 1 - p) over [0, 1] and the NaNs.
CHUNK = 1 << 24


def sem_chunks(kind):
    if kind in (0, 1):
        return [(i * CHUNK, (i + 1) * CHUNK) for i in range(256)]
    one = 0x3F800001
    out = [(lo, min(lo + CHUNK, one)) for lo in range(0, one, CHUNK)]
    return out + [(0x7F800001, 0x80000000), (0xFF800001, 0x100000000)]


def _digest(args):
    from _oracle import lib
    L = lib()
    kind, lo, hi = args
    return str(L.ora_math_digest(kind, lo, hi))


def make_sem_digests():
    from multiprocessing import Pool
    out = {}
    with Pool(min(8, os.cpu_count() or 1)) as pool:
        for kind in (0, 1, 2):
            ch = sem_chunks(kind)
            dig = pool.map(_digest, [(kind, lo, hi) for lo, hi in ch])
            out[str(kind)] = [[lo, hi, d] for (lo, hi), d in zip(ch, dig)]
    return out


def main():
    json.dump(KAT, open(os.path.join(HERE, "kat_reference.json"), "w"), indent=1)
    g = make_integrate()
    np.savez_compressed(os.path.join(HERE, "integrate_48x36.npz"), **g)
    print("live blocks", g["live_entry"].size, "query voxels", int(g["query_count"]),
          "stats", g["stats"].tolist())
    for touch, name in SEMANTIC.items():
        g = make_integrate(touch, nframes=40, bits=12)
        np.savez_compressed(os.path.join(HERE, name), **g)
        w = g["rgbw"][..., 3]
        print(touch, "live blocks", g["live_entry"].size, "weight-40 voxels", int((w == 40).sum()),
              "NaN prob", int(np.isnan(g["prob"]).sum()), "prob 0 / 1", int((g["prob"] == 0).sum()),
              int((g["prob"] == 1).sum()))
    if "--digests" in sys.argv:
        json.dump(make_sem_digests(), open(os.path.join(HERE, "sem_math_digests.json"), "w"))


if __name__ == "__main__":
    main()
