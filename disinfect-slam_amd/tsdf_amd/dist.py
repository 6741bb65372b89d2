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


def integrate_sharded(engine, bufs, rgb, depth, ht, lt, K, cam_T_world, max_depth, split=True, graph=None):
    """One frame of a spatially sharded volume on this rank (tsdf_integrate_shard_*):
    begin (DDA over this rank's band of tile rows when split) -> all-gather of the key slots ->
    update -> all-gather of the carve-candidate slots -> end. Asynchronous on the current stream.
    graph: the engine's ShardFrameGraph (Engine.shard_frame_graph): the three phases as its captured
    segments, the all-gathers between them as here (RCCL calls cannot be recorded into the engine's
    graphs across the C ABI)."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        rank, world = dist.get_rank(), dist.get_world_size()
    else:
        rank, world = 0, 1
    try:
        if graph is not None:
            graph.begin(rgb, depth, ht, lt, K, cam_T_world, max_depth, bufs.keys_out, bufs.keys_in, bufs.key_cap,
                        bufs.cands_out, bufs.cands_in, bufs.cand_cap)
            if graph.split:
                all_gather_slots(bufs.keys_out, bufs.keys_in)
            graph.update(bufs.keys_in, bufs.cands_out)
            all_gather_slots(bufs.cands_out, bufs.cands_in)
            graph.end(bufs.cands_in)
            return
        _integrate_sharded(engine, bufs, rgb, depth, ht, lt, K, cam_T_world, max_depth, split, rank, world)
    except Exception:
        # a failed exchange (e.g. a collective timeout) must not leave the engine mid-frame; the
        # caller sees the original error even if the abort itself fails
        try:
            engine.integrate_shard_abort()
        except Exception:
            pass
        raise


def integrate_sharded_pipe(engine, bufs, rgb, depth, ht, lt, K, cam_T_world, max_depth):
    """One pipelined sharded frame on this rank (tsdf_integrate_shard_pipe): ONE
    all-gather per frame -- this call's carve candidates (bufs.cands_out) into every rank's inbox
    (bufs.cands_in, read by the next call). depth None: one step of completing the pending frames.
    Returns True while more steps are needed (flush_sharded_pipe loops)."""
    try:
        pend = engine.integrate_shard_pipe(rgb, depth, ht, lt, K, cam_T_world, max_depth, bufs.cands_in,
                                           bufs.cands_out, bufs.cand_cap)
        all_gather_slots(bufs.cands_out, bufs.cands_in)
    except Exception:
        # as integrate_sharded: the pending pipelined frames are dropped (STATUS_SHARD_ABORTED), the
        # caller sees the original error
        try:
            engine.integrate_shard_abort()
        except Exception:
            pass
        raise
    return pend


def flush_sharded_pipe(engine, bufs):
    """Complete this rank's pipelined sharded frames (every rank calls it: each step exchanges)."""
    while integrate_sharded_pipe(engine, bufs, None, None, None, None, None, None, 4.0):
        pass


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


def band_rows(height: int, world: int):
    """Row boundaries of a sharded render's image bands: rank r renders rows [rows[r], rows[r + 1])."""
    return [height * r // world for r in range(world + 1)]


def exchange_groups(counts, recs):
    """All-to-all-v of grouped rows (tsdf_render_bands / tsdf_pack_halo output): the counts[d] rows
    of group d go to rank d. Returns (the rows this rank received, concatenated in source-rank order;
    the received counts per source). RCCL on the GPU box (device tensors), gloo through the host.
    Without a process group the rows are this rank's own group 0."""
    import numpy as np
    import torch
    import torch.distributed as dist
    t = recs if isinstance(recs, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(recs))
    counts = [int(c) for c in counts]
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return t[:counts[0]], [counts[0]]
    world = dist.get_world_size()
    host = t.is_cuda and dist.get_backend() == "gloo"
    cdev = torch.device("cpu") if (host or not t.is_cuda) else t.device
    send_n = torch.tensor(counts, dtype=torch.int64, device=cdev)
    recv_n = torch.empty(world, dtype=torch.int64, device=cdev)
    dist.all_to_all_single(recv_n, send_n)
    rcounts = [int(c) for c in recv_n.tolist()]
    row = int(t[0].numel()) if t.dim() > 1 else 1
    src = t.cpu() if host else t
    out = torch.empty((sum(rcounts),) + tuple(t.shape[1:]), dtype=t.dtype, device=src.device)
    dist.all_to_all_single(out.view(-1), src.contiguous().view(-1), [c * row for c in rcounts],
                           [c * row for c in counts])
    return (out.to(t.device) if host else out), rcounts


# bytes this rank moved in the last sharded render / mesh (the bench reports them per frame)
last_exchange = {}


def render_sharded(engine, replica, K, width, height, cam_T_world, max_depth, device=True,
                   rgba=None, normal=None):
    """Raycast of a spatially sharded volume that divides the work: rank r renders the
    image rows of band r. Every rank packs, per band, the blocks of its shard that the band's rays
    can read (tsdf_render_bands) and sends band b's records to rank b (an all-to-all over xGMI on the
    GPU box); rank r imports what it received into `replica` (a scratch engine of the same voxel
    size / truncation) and renders its rows with the unchanged raycast kernel (tsdf_raycast_rows),
    then the bands are all-gathered. Every rank gets the image the unsharded volume renders, bit for
    bit. Returns (rgba, normal): numpy (H, W, 4) u8, or the given device tensors filled."""
    import numpy as np
    import torch
    import torch.distributed as dist
    rank, world = ((dist.get_rank(), dist.get_world_size())
                   if dist.is_available() and dist.is_initialized() else (0, 1))
    rows = band_rows(height, world)
    counts, recs = engine.render_bands(K, width, height, cam_T_world, max_depth, rows, device=device)
    mine, _ = exchange_groups(counts, recs)
    replica.import_blocks(mine if device else mine.numpy(), replace=True)
    r0, nr = rows[rank], rows[rank + 1] - rows[rank]
    maxr = max(rows[i + 1] - rows[i] for i in range(world))
    dev = torch.device("cuda", torch.cuda.current_device())
    band = torch.zeros((2, maxr, width, 4), dtype=torch.uint8, device=dev)
    replica.raycast_rows(K, width, height, cam_T_world, max_depth, r0, nr, rgba=band[0], normal=band[1])
    if world > 1:
        allb = torch.empty((world,) + tuple(band.shape), dtype=torch.uint8, device=dev)
        if dist.get_backend() == "gloo":
            hb = torch.empty(allb.shape, dtype=torch.uint8)
            dist.all_gather_into_tensor(hb.view(-1), band.cpu().view(-1))
            allb.copy_(hb)
        else:
            dist.all_gather_into_tensor(allb.view(-1), band.view(-1))
    else:
        allb = band[None]
    img = torch.cat([allb[i, :, :rows[i + 1] - rows[i]] for i in range(world)], dim=1)  # (2, H, W, 4)
    last_exchange.update(render_records_sent=int(recs.shape[0]), render_records_received=int(mine.shape[0]),
                         render_bytes_sent=int(recs.shape[0]) * 6160, render_bytes_received=int(mine.shape[0]) * 6160,
                         render_band_bytes=int(band.numel()), render_rows=nr)
    if rgba is not None:
        rgba.copy_(img[0])
        if normal is not None:
            normal.copy_(img[1])
        return rgba, normal
    out = img.cpu().numpy()
    return np.ascontiguousarray(out[0]), np.ascontiguousarray(out[1])


def mesh_sharded(engine, replica, bounds=None, missing_tsdf=0.99, min_weight=0, device=True,
                 out=None):
    """Marching cubes of a spatially sharded volume that divides the work: each rank meshes the
    cells of its own blocks. Its cells read one sample into every neighbouring block, so every rank
    sends each of its blocks to the owners of the block's 26 neighbours (tsdf_pack_halo, an
    all-to-all); rank r imports its own blocks plus the halo it received into `replica` and extracts
    the triangles of its own blocks there (tsdf_extract_mesh_owned). The triangles are all-gathered:
    the same set as the unsharded mesh (rank by rank, each in its replica's entry order). Returns an
    (n, 3, 3) float32 numpy array, or a device tensor view when `out` is given."""
    import torch
    import torch.distributed as dist
    rank, world = ((dist.get_rank(), dist.get_world_size())
                   if dist.is_available() and dist.is_initialized() else (0, 1))
    own = engine.pack_blocks(None, device=device)
    if world > 1:
        counts, halo = engine.pack_halo(device=device)
        got, _ = exchange_groups(counts, halo)
        sent = int(halo.shape[0])
    else:
        got, sent = own[:0], 0
    recs = torch.cat([torch.as_tensor(own), torch.as_tensor(got).to(torch.as_tensor(own).device)])
    replica.import_blocks(recs if device else recs.numpy(), replace=True)
    tris = replica.extract_mesh(bounds, missing_tsdf, min_weight, out=out,
                                owner=(rank, world) if world > 1 else None)
    last_exchange.update(mesh_halo_records_sent=sent, mesh_halo_records_received=int(got.shape[0]),
                         mesh_own_records=int(own.shape[0]))
    rows = tris.reshape(-1, 9)
    allrows = gather_rows(rows, device=rows.device if isinstance(rows, torch.Tensor) else None)
    if out is not None:
        n = int(allrows.shape[0])
        out.view(-1)[:9 * n].copy_(allrows.reshape(-1).to(out.device))
        return out.view(-1)[:9 * n].view(-1, 3, 3)
    return allrows.cpu().numpy().reshape(-1, 3, 3) if isinstance(allrows, torch.Tensor) else allrows
