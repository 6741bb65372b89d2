# Diagnostic (GPU box): drive two shard engines' phases by hand with host syncs between them.
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "disinfect-slam_amd")]
import numpy as np
import torch
import tsdf_amd
from tsdf_amd import synth
W, H, vox, tr, G, cap = 96, 72, 0.01, 0.04, 2, 16384
sync = sys.argv[1] == "1"
cam = synth.camera(W, H, synth.TUM_FR1)
torch.cuda.init()
st = torch.cuda.current_stream().cuda_stream
engs = [tsdf_amd.Engine(vox, tr, max_width=W, max_height=H, num_block_bits=13, shard_index=i, shard_count=G,
                        stream=st) for i in range(G)]
sb = tsdf_amd.Engine.shard_slot_bytes(cap)
keys = torch.zeros((G, sb), dtype=torch.uint8, device="cuda")
cands = torch.zeros((G, sb), dtype=torch.uint8, device="cuda")
hdr = lambda t: t[:, 8:12].contiguous().view(torch.int32).flatten().tolist()
fr = synth.render(cam, 0)
pose = tsdf_amd.SE3(fr["q"], fr["t"])
for i, e in enumerate(engs):
    e.integrate_shard_begin(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], cam.K, pose, 4.0, i, G, keys[i], cap)
    if sync: torch.cuda.synchronize(); print("after begin", i, "key headers", hdr(keys))
for i, e in enumerate(engs):
    e.integrate_shard_update(keys, cap, cands[i], cap)
    if sync: torch.cuda.synchronize(); print("after update", i, "new keys", e.stats()["last_num_new_keys"])
for e in engs:
    e.integrate_shard_end(cands, cap)
torch.cuda.synchronize()
print("final", hdr(keys), [e.stats()["last_num_new_keys"] for e in engs], [e.stats()["active_blocks"] for e in engs])
