# Sharded raycast composite (tsdf_render_blocks -> gather -> tsdf_import_blocks -> tsdf_raycast) on
# one GPU, G shard engines in-process, at the bench geometry (640x480, 5 mm, 3 cm truncation, 120
# orbit frames). Prints one JSON line: per-phase ms of the composite next to the unsharded raycast,
# records per shard, and whether the images are equal. GPU box: python3 scripts/render_composite_timing.py [G]
import json
import sys
import time

sys.path[:0] = ['disinfect-slam_amd', 'tests']
import numpy as np
import torch

import tsdf_amd
from tsdf_amd import synth

G = int(sys.argv[1]) if len(sys.argv) > 1 else 8
W, H, N = 640, 480, 120
cam = synth.camera(W, H, synth.TUM_FR1)
fr = synth.render_torch(cam, list(range(N + 1)), device='cuda')
K = tsdf_amd.CameraIntrinsics(*[float(v) for v in cam.K])
poses = [tsdf_amd.SE3(fr['q'][i], fr['t'][i]) for i in range(N + 1)]
mk = lambda **kw: tsdf_amd.Engine(0.005, 0.03, max_width=W, max_height=H, **kw)
full = mk()
group = tsdf_amd.ShardGroup(G, 0.005, 0.03, max_width=W, max_height=H, num_block_bits=18,
                            key_cap=32768 // G, cand_cap=16384 // G)
shards = group.engines
replica = mk()
for i in range(N):
    full.integrate(fr['rgb'][i], fr['depth'][i], fr['ht'][i], fr['lt'][i], K, poses[i], 4.0)
    group.integrate(fr['rgb'][i], fr['depth'][i], fr['ht'][i], fr['lt'][i], K, poses[i], 4.0)
torch.cuda.synchronize()
pose = poses[N]
rgba = torch.zeros((H, W, 4), dtype=torch.uint8, device='cuda')
normal = torch.zeros_like(rgba)


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        out = fn()
    torch.cuda.synchronize()
    return 1e3 * (time.perf_counter() - t) / reps, out


ms_full, _ = timed(lambda: full.raycast(K, W, H, pose, 4.0, rgba=rgba, normal=normal))
ms_pack = []
parts = []
for e in shards:
    ms, p = timed(lambda e=e: e.render_blocks(K, W, H, pose, 4.0, device=True))
    ms_pack.append(ms)
    parts.append(p)
allrecs = torch.cat(parts)
ms_reset, _ = timed(replica.reset)
ms_import, _ = timed(lambda: replica.import_blocks(allrecs, replace=True))
ms_rc, _ = timed(lambda: replica.raycast(K, W, H, pose, 4.0, rgba=rgba, normal=normal))
exp = full.raycast(K, W, H, pose, 4.0)
got = replica.raycast(K, W, H, pose, 4.0)
print(json.dumps({
    "shards": G, "frames": N, "active_blocks_unsharded": full.stats()["active_blocks"],
    "records_per_shard": [int(p.shape[0]) for p in parts], "records_total": int(allrecs.shape[0]),
    "record_bytes_total": int(allrecs.numel()),
    "ms_raycast_unsharded": round(ms_full, 4), "ms_render_blocks_per_shard_max": round(max(ms_pack), 4),
    "ms_full_reset": round(ms_reset, 4), "ms_replica_import_replace": round(ms_import, 4),
    "ms_replica_raycast": round(ms_rc, 4),
    "images_equal": bool(np.array_equal(exp[0], got[0]) and np.array_equal(exp[1], got[1])),
}))
for e in [full, replica] + shards:
    e.close()
