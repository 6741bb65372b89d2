"""Multi-GPU plumbing of the TSDF engine: one process per GPU (torch.distributed.run).

 - streams mode (weak scaling): rank r integrates its own camera stream into its own volume; no
   data-path collective;
 - sharded modes (strong scaling): ONE stream into ONE volume spatially sharded over
   the ranks by 4^3-block bricks. Every rank keeps the whole hash index and the voxels of its own
   bricks, and a frame is three engine calls around two all-gathers (integrate_sharded): the new
   block keys (each rank runs the DDA over its band of pixel-tile rows; "routed") and the
   space-carving candidates. With split=False ("sharded") every rank runs the whole DDA and only
   the candidates are exchanged. Either way the union of the ranks is the unsharded volume, block
   for block and voxel for voxel.

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


def all_gather_slots(slot, out):
    """out (world, slot_bytes) <- every rank's slot (world x slot_bytes u8), rank order: one
    all-gather, RCCL over xGMI on the GPU box, ordered on the current stream (no host sync).
    Without a process group (one rank) it is a copy."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        out.view(-1)[:slot.numel()].copy_(slot.view(-1))
        return out
    if slot.is_cuda and dist.get_backend() == "gloo":  # CPU-backend tests: stage through the host
        host = torch.empty(out.numel(), dtype=out.dtype)
        dist.all_gather_into_tensor(host, slot.view(-1).cpu())
        out.view(-1).copy_(host)
        return out
    dist.all_gather_into_tensor(out.view(-1), slot.view(-1))
    return out


class ShardBuffers:
    """Exchange slots of one rank's sharded engine (tsdf_shard_slot_bytes each)."""

    def __init__(self, engine, world, key_cap=16384, cand_cap=16384, device=None):
        import torch
        dev = device if device is not None else f"cuda:{engine.device}"
        self.key_cap, self.cand_cap = key_cap, cand_cap
        kb, cb = engine.shard_slot_bytes(key_cap), engine.shard_slot_bytes(cand_cap)
        self.keys_out = torch.zeros(kb, dtype=torch.uint8, device=dev)
        self.keys_in = torch.zeros((world, kb), dtype=torch.uint8, device=dev)
        self.cands_out = torch.zeros(cb, dtype=torch.uint8, device=dev)
        self.cands_in = torch.zeros((world, cb), dtype=torch.uint8, device=dev)


def integrate_sharded(engine, bufs, rgb, depth, ht, lt, K, cam_T_world, max_depth, split=True):
    """One frame of a spatially sharded volume on this rank (tsdf_integrate_shard_*):
    begin (DDA over this rank's band of tile rows when split) -> all-gather of the key slots ->
    update -> all-gather of the carve-candidate slots -> end. Asynchronous on the current stream."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        rank, world = dist.get_rank(), dist.get_world_size()
    else:
        rank, world = 0, 1
    try:
        _integrate_sharded(engine, bufs, rgb, depth, ht, lt, K, cam_T_world, max_depth, split, rank, world)
    except Exception:
        # a failed exchange (e.g. a collective timeout) must not leave the engine mid-frame
        engine.integrate_shard_abort()
        raise


def _integrate_sharded(engine, bufs, rgb, depth, ht, lt, K, cam_T_world, max_depth, split, rank, world):
    if split:
        engine.integrate_shard_begin(rgb, depth, ht, lt, K, cam_T_world, max_depth, rank, world,
                                     bufs.keys_out, bufs.key_cap)
        all_gather_slots(bufs.keys_out, bufs.keys_in)
        engine.integrate_shard_update(bufs.keys_in, bufs.key_cap, bufs.cands_out, bufs.cand_cap)
    else:
        engine.integrate_shard_begin(rgb, depth, ht, lt, K, cam_T_world, max_depth)
        engine.integrate_shard_update(None, bufs.key_cap, bufs.cands_out, bufs.cand_cap)
    all_gather_slots(bufs.cands_out, bufs.cands_in)
    engine.integrate_shard_end(bufs.cands_in, bufs.cand_cap)


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
