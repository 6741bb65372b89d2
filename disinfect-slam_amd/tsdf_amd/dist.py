"""Multi-GPU plumbing of the TSDF engine: one process per GPU (torch.distributed.run).

 - streams mode (weak scaling): rank r integrates its own camera stream into its own volume; no
   data-path collective;
 - sharded mode (strong scaling, SURVEY 8e option 1): every rank sees the same frames, runs the
   whole DDA and owns the blocks whose 4^3 brick hashes to it (tsdf_block_owner); no data-path
   collective; a whole-volume Query is the union of the shards;
 - routed mode (strong scaling, SURVEY 8e option 2): same ownership, but rank r runs the DDA only
   over its slice of pixel-tile rows and routes the keys other ranks own with one all-to-all per
   frame (route_exchange: RCCL over xGMI on the GPU box).

The functions here are backend-agnostic (RCCL "nccl" on the GPU box, "gloo" in the CPU tests).
"""
from __future__ import annotations

import os


def env_rank_world():
    """(rank, local_rank, world_size) from the torch.distributed.run environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))


def shard_of(mode: str, rank: int, world: int):
    """(shard_index, shard_count) of this rank's engine."""
    return (rank, world) if (mode in ("sharded", "routed") and world > 1) else (0, 1)


def route_exchange(outbox, inbox):
    """Routed frames: inbox slot s <- rank s's outbox slot <this rank> (all-to-all, equal splits).

    outbox / inbox: contiguous (world, slot_bytes) tensors (tsdf_route_buffer_bytes in all). On the
    GPU box this is one RCCL all-to-all ordered on the current stream (the engine's stream), so the
    frame stays asynchronous; without a process group it is the identity (one shard)."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        inbox.copy_(outbox)
        return inbox
    dist.all_to_all_single(inbox, outbox)
    return inbox


def stream_offset(mode: str, rank: int, world: int, stride: int = 240) -> int:
    """First frame of this rank's camera stream (streams mode: a third of an orbit apart)."""
    return rank * stride if (mode == "streams" and world > 1) else 0


def units(mode: str, steps: int, world: int) -> int:
    """Frames integrated by the whole job in `steps` timed steps."""
    return steps * (world if mode == "streams" else 1)


def max_over_ranks(value: float, device=None) -> float:
    """MAX of a per-rank float over all ranks (identity without an initialised process group)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(value)
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(values, device=None):
    """Element-wise SUM of a list of per-rank numbers over all ranks."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return [float(v) for v in values]
    t = torch.tensor(list(values), dtype=torch.float64, device=device)
    dist.all_reduce(t)
    return [float(v) for v in t.tolist()]


def gather_block_sets(positions, device=None):
    """All-gather every rank's live block positions (N x 3 int16 numpy) -> list per rank."""
    import numpy as np
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return [np.asarray(positions)]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, np.asarray(positions))
    return out


def gather_query(voxels, device=None):
    """Whole-volume Query of a sharded volume: every rank passes its shard's
    tsdf_query result, all ranks get the union -- an all-gather of the counts, then one padded
    all-gather of the (x, y, z, tsdf) rows (RCCL on the GPU box, gloo in the CPU tests). Shards own
    disjoint blocks, so the union is the unsharded Query as a set of voxels; rows come rank by
    rank, each rank's in its own entry order."""
    import numpy as np
    import torch
    import torch.distributed as dist
    arr = np.ascontiguousarray(np.asarray(voxels).view(np.float32).reshape(-1, 4))
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return arr
    world = dist.get_world_size()
    n = torch.tensor([arr.shape[0]], dtype=torch.int64, device=device)
    counts = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(counts, n)
    counts = [int(c.item()) for c in counts]
    cap = max(max(counts), 1)
    mine = torch.zeros((cap, 4), dtype=torch.float32, device=device)
    if arr.shape[0]:
        mine[:arr.shape[0]] = torch.from_numpy(arr).to(mine.device)
    allrows = torch.empty((world * cap, 4), dtype=torch.float32, device=device)
    dist.all_gather_into_tensor(allrows, mine)
    allrows = allrows.cpu().numpy()
    return np.concatenate([allrows[r * cap:r * cap + counts[r]] for r in range(world)])


def gather_rows(rows, device=None):
    """All-gather-v of a 2-D tensor / array of rows (same row width and dtype on every rank): an
    all-gather of the counts, then one padded all-gather of the rows, concatenated rank by rank.
    Returns a tensor on `device` (the rows' own device by default)."""
    import numpy as np
    import torch
    import torch.distributed as dist
    t = rows if isinstance(rows, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(rows))
    if device is not None:
        t = t.to(device)
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return t
    world = dist.get_world_size()
    n = torch.tensor([t.shape[0]], dtype=torch.int64, device=t.device)
    counts = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(counts, n)
    counts = [int(c.item()) for c in counts]
    cap = max(max(counts), 1)
    mine = torch.zeros((cap,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    mine[:t.shape[0]] = t
    allrows = torch.empty((world * cap,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    dist.all_gather_into_tensor(allrows, mine)
    return torch.cat([allrows[r * cap:r * cap + counts[r]] for r in range(world)])


def render_sharded(engine, replica, K, width, height, cam_T_world, max_depth, device=True,
                   rgba=None, normal=None):
    """Raycast of a spatially sharded volume (SURVEY.md 8e raycast composite): every
    rank packs the blocks of its shard that this camera's rays can read (tsdf_render_blocks), the
    records are all-gathered (RCCL over xGMI on the GPU box), and `replica` -- a scratch engine of
    the same voxel size / truncation with room for them -- imports the union and renders it with
    the unchanged raycast kernel. Every rank gets the image the unsharded volume renders.
    Returns (rgba, normal) as numpy (H, W, 4) uint8, or the given device tensors rgba / normal."""
    recs = engine.render_blocks(K, width, height, cam_T_world, max_depth, device=device)
    allrecs = gather_rows(recs)
    replica.import_blocks(allrecs if device else allrecs.numpy(), replace=True)
    return replica.raycast(K, width, height, cam_T_world, max_depth, rgba=rgba, normal=normal)


def mesh_sharded(engine, replica, bounds=None, missing_tsdf=0.99, min_weight=0, device=True,
                 out=None):
    """Marching cubes of a spatially sharded volume: a shard's own extraction misses the cells that
    straddle another owner's blocks, so every rank packs all its live blocks (tsdf_pack_blocks),
    the records are all-gathered, `replica` imports the union -- the whole unsharded volume -- and
    extracts there (tsdf_extract_mesh with bounds). Same triangles as the unsharded mesh, in the
    replica's entry order."""
    recs = engine.pack_blocks(None, device=device)
    allrecs = gather_rows(recs)
    replica.import_blocks(allrecs if device else allrecs.numpy(), replace=True)
    return replica.extract_mesh(bounds, missing_tsdf, min_weight, out=out)
