# Diagnostic (GPU box): a ShardGroup vs the unsharded engine, frame by frame; prints the first
# frame whose per-frame counters or index differ and what differs.
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "disinfect-slam_amd")]
import numpy as np
import torch
import tsdf_amd
from tsdf_amd import synth
G = int(sys.argv[1]) if len(sys.argv) > 1 else 2
split = (sys.argv[2] != "0") if len(sys.argv) > 2 else True
W, H, vox, tr = 96, 72, 0.01, 0.04
cam = synth.camera(W, H, synth.TUM_FR1)
torch.cuda.init()
full = tsdf_amd.Engine(vox, tr, max_width=W, max_height=H, num_block_bits=13)
grp = tsdf_amd.ShardGroup(G, vox, tr, max_width=W, max_height=H, num_block_bits=13, split=split)
for f in range(6):
    fr = synth.render(cam, 2 * f)
    pose = tsdf_amd.SE3(fr["q"], fr["t"])
    full.integrate(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], cam.K, pose, 4.0)
    grp.integrate(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], cam.K, pose, 4.0, count=True)
    fs = full.stats(); ss = grp.stats()
    keys = ("last_num_visible", "last_num_alloc", "last_num_deleted", "last_num_new_keys", "active_blocks", "last_num_updated", "status")
    print(f, {k: (fs[k], [s[k] for s in ss]) for k in keys}, "exchanged", grp.keys_exchanged, grp.cands_exchanged)
    df = full.dump(pool=False)
    focc = df["entry_idx"] >= 0
    for i, e in enumerate(grp.engines):
        d = e.dump(pool=False)
        occ = d["entry_idx"] >= 0
        if not np.array_equal(occ, focc):
            extra = np.flatnonzero(occ & ~focc); miss = np.flatnonzero(focc & ~occ)
            print("  shard", i, "extra entries", extra[:8], d["entry_pos"][extra[:8]].tolist(), "idx", d["entry_idx"][extra[:8]].tolist())
            print("  shard", i, "missing entries", miss[:8], df["entry_pos"][miss[:8]].tolist())
        else:
            bad = np.flatnonzero(np.any(d["entry_pos"][occ] != df["entry_pos"][focc], axis=1))
            if bad.size: print("  shard", i, "entry content differs at", np.flatnonzero(occ)[bad[:8]])
