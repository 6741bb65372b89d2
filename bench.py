#!/usr/bin/env python3
"""bench.py -- TSDF integrate frames/s on MI355X (BASELINE.json metric), one JSON line on rank 0.

Workload (N=1): BASELINE.json configs[2] (C3) -- synthetic 640x480 depth + per-pixel high/low-touch
probability maps (the segmentation/inference output shape), fused TSDF + RGB + semantic integrate
into a 5 mm voxel-hash volume (3 cm truncation, 4 m max depth, TUM fr1 intrinsics). One step = one
TSDFGrid::Integrate of one frame (voxel_tsdf.cu:347-375): DDA block allocation, visibility, fused
update, space carving. All frames are rendered on the GPU and resident in HBM before timing starts.

N>1 (torch.distributed.run, one rank per GPU) -- default --mode routed: ONE camera stream into ONE
volume spatially sharded over the ranks. Every rank keeps the whole hash
index and the voxels of its own 4^3-block bricks; rank r runs the block-allocation DDA over its band
of pixel-tile rows, the frame's new keys and the carve candidates are all-gathered over RCCL, and
each rank updates only its own blocks. value = frames / max rank time, scaling "strong"; the volume
is the single-GPU volume block for block. --mode sharded: the same with every rank running the whole
DDA (no key exchange). --mode streams: each rank integrates its own camera stream into its own volume
(a multi-camera rig; weak scaling, no data-path collective). At N>1 the line carries the streams run
as a labelled "secondary" object measured in the same job (--secondary none to skip).

roofline: SURVEY.md 8d. The frame-level fraction B_read * frames/s / (N * 8 TB/s) with
B_read = 15 W H (frame) + N_vis * 6156 B (voxel state + metadata of every visible block), and the
same with the updated voxels' writes; and the kernel-level entry of the fused update kernel
k_integrate: algorithmic bytes per launch N_vis * 6156 + N_upd * 12 + 15 W H (N_vis, N_upd counted
on device) / the kernel's average duration from HIP start/stop events bound to its dispatches on the
engine stream. traffic: HBM bytes per launch from a rocprofv3 --pmc pass (FETCH_SIZE x2 + WRITE_SIZE,
MI355X_MICROARCH.md gfx950 corrections) of THIS command over the same timed-window launches,
accepted only when that pass integrated the same frames (equal N_vis / N_upd sums); otherwise null.
The two resolvers run inside the ingest / update kernels' last-arriving workgroups: their device-clock
spans are reported in "device_us_per_frame".
cpu_baseline: the single-threaded CPU oracle (oracle/tsdf_oracle.c, a restatement of the reference
kernels incl. its full-table visibility scan) on the first frames of this same stream (the GPU
frames copied to the host), from an empty map.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "disinfect-slam_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
BLOCK_READ_BYTES = 512 * 12 + 12  # voxel state + metadata of one visible block
PMC_FILE = os.path.join(ROOT, "profiles", "pmc_integrate_r6.json")
# SQ counters of k_raycast (rocprofv3 --pmc passes of `bench.py --loop c5`, scripts/profile_kernel_sq.sh)
RAYCAST_SQ_FILE = os.path.join(ROOT, "profiles", "r5_raycast_sq.json")
VALU_PEAK_WAVE_INSTR = 256 * 4 * 2.4e9 / 2  # wave64 VALU instructions/s: 1024 SIMDs, 2 cycles each


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=300)
    p.add_argument("--warmup", type=int, default=30)
    p.add_argument("--width", type=int, default=640)
    p.add_argument("--height", type=int, default=480)
    p.add_argument("--voxel", type=float, default=0.005)
    p.add_argument("--trunc", type=float, default=0.03)
    p.add_argument("--max-depth", type=float, default=4.0)
    p.add_argument("--depth-only", action="store_true", help="config C2: ht = lt = NULL (ones)")
    p.add_argument("--mode", choices=("routed", "sharded", "streams"), default="routed",
                   help="N>1: routed (sharded volume, DDA split by tile rows, keys exchanged), sharded "
                        "(sharded volume, whole-frame DDA on every rank), streams (one volume per rank)")
    p.add_argument("--secondary", choices=("streams", "none"), default="streams",
                   help="N>1: also measure the streams mode in the same job (labelled secondary)")
    p.add_argument("--loop", choices=("c3", "c5"), default="c3",
                   help="c5: BASELINE config C5 -- integrate + raycast of the frame's camera every frame, "
                        "marching cubes of the whole volume every 30 frames (eager chain)")
    p.add_argument("--graph", action="store_true",
                   help="frames through the graph-captured frame (one hipGraph launch per frame)")
    p.add_argument("--graph-batch", type=int, default=None,
                   help="with --graph: frames per graph launch (tsdf_graph_create_batch; the launch's fixed "
                        "cost paid once per batch). Default 16 for the C3 loop (19.6k vs 16.6k frames/s at "
                        "1), 8 for C5 (7.2k vs 6.76k at 1 and 6.95k at 16; DESIGN.md 4 round 6)")
    p.add_argument("--shard", default=None, metavar="G",
                   help="single-GPU rehearsal of the routed sharded volume: G shard engines on this GPU "
                        "exchanging their slots with device copies; reports the per-shard frame time")
    p.add_argument("--key-cap", type=int, default=0,
                   help="sharded modes: key records per rank per frame (0 = 32768 / G)")
    p.add_argument("--cand-cap", type=int, default=0,
                   help="sharded modes: carve-candidate records per rank per frame (0 = 16384 / G)")
    p.add_argument("--cpu-frames", type=int, default=-1, help="oracle sample size (-1 = auto)")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--native-group", action="store_true",
                   help="with --shard G: the library-owned group (tsdf_group_*) instead of tsdf_amd.ShardGroup")
    p.add_argument("--no-cpp-loop", action="store_true",
                   help="skip the C++ timed loop over the C ABI (disinfect-slam_amd/bench_main) that the "
                        "single-GPU C3 line runs after its own loop (the host enqueue floor without Python)")
    p.add_argument("--broadcast-frames", dest="broadcast_frames", action="store_true", default=None,
                   help="sharded modes: rank 0 broadcasts every frame to the other ranks inside the timed "
                        "loop (one camera feeding the node) -- the default with the nccl backend")
    p.add_argument("--no-broadcast-frames", dest="broadcast_frames", action="store_false",
                   help="sharded modes: every rank holds the stream; the broadcast is timed beside the line")
    p.add_argument("--backend", choices=("nccl", "gloo"), default="nccl",
                   help="process-group backend for N > 1: nccl (RCCL over xGMI, one GPU per rank) or gloo "
                        "(a rehearsal of the multi-rank code path; ranks may share a GPU, exchanges staged "
                        "through the host -- not a performance number)")
    p.add_argument("--host-frames", choices=("pageable", "pinned"), default=None,
                   help="single GPU: frames in host memory (the reference API's cv::Mat inputs), passed as "
                        "TSDF_MEM_HOST -- the engine uploads each frame (voxel_tsdf.cu:358-365) on its upload "
                        "stream beside the previous frames' kernels; the line reports the upload alone too")
    p.add_argument("--block-bits", type=int, default=18)
    p.add_argument("--event-every", type=int, default=0,
                   help="HIP-event-time the frame kernel on every n-th timed frame (a dispatch with bound "
                        "events runs ~1 us slower, so the loop samples); 0 = steps // 5 clamped to [1, 16] "
                        "(at least 5 timed launches)")
    p.add_argument("--no-events", action="store_true",
                   help="diagnostic: no HIP events in the timed loop (kernel roofline then from the "
                        "device clock)")
    p.add_argument("--no-defer", action="store_true",
                   help="C5 loop: immediate tsdf_raycast / tsdf_graph_create instead of tsdf_raycast_deferred / "
                        "tsdf_graph_create_deferred (the raycast then runs in its own launch instead of "
                        "beside the next frame's ingest)")
    a = p.parse_args()
    if a.graph_batch is None:
        a.graph_batch = 16 if a.loop != "c5" else 8
    return a


def workload_name(a):
    W, H = a.width, a.height
    if (W, H) == (640, 480):
        w = "C2: 640x480 depth-only" if a.depth_only else "C3: 640x480 depth + ht/lt semantic"
    else:
        w = f"{W}x{H} depth{'' if a.depth_only else ' + ht/lt semantic'}"
    if a.loop == "c5":
        w = "C5: " + w + ", raycast every frame, marching cubes every 30 frames"
    if a.host_frames:
        w += f", {a.host_frames} host frames (TSDF_MEM_HOST: uploaded by the engine every frame)"
    return (w + f", {a.voxel * 1000:g} mm voxel, {a.trunc * 100:g} cm truncation, {a.max_depth:g} m "
            f"max depth, {'TUM fr1' if W <= 640 else 'L515 full-res'} intrinsics, orbit 1 cm + 0.5 deg/frame")


class Run:
    """One timed configuration on this rank: engines, the per-frame step, the timed loop."""

    def __init__(self, a, mode, rank, world, dev, cam, frames, K, poses, dist):
        import torch
        import tsdf_amd
        from tsdf_amd import dist as tdist
        self.a, self.mode, self.world, self.dist, self.dev = a, mode, world, dist, dev
        self.frames, self.K, self.poses = frames, K, poses
        # the frames are inputs already resident in HBM: split them into per-frame views (and the poses
        # into their C structs) once, so the timed loop's host time is the engine's enqueue, not
        # torch's tensor indexing
        self.frame_views = {k: (list(v.unbind(0)) if hasattr(v, "unbind") else v) for k, v in frames.items()}
        for p_ in poses:
            p_._c()
        self.sharded = mode in ("routed", "sharded") and world > 1
        si, sc = (rank, world) if self.sharded else (0, 1)
        self.shard_index, self.shard_count = si, sc
        self.stream = torch.cuda.current_stream()
        self.eng = tsdf_amd.Engine(a.voxel, a.trunc, max_width=a.width, max_height=a.height,
                                   num_block_bits=a.block_bits, device=torch.cuda.current_device(),
                                   shard_index=si, shard_count=sc, stream=self.stream)
        self.bufs = None
        if self.sharded:  # exchange slots (RCCL all-gathers on this stream)
            self.bufs = tdist.ShardBuffers(self.eng, sc, a.key_cap or max(1024, 32768 // sc),
                                           a.cand_cap or max(1024, 16384 // sc), device=dev)
        self.graph = None
        self.replica = None
        self.mesh_tris = []
        W, H = a.width, a.height
        self.rgba = self.normal = None
        if a.loop == "c5":
            self.rgba = torch.zeros((H, W, 4), dtype=torch.uint8, device=dev)
            self.normal = torch.zeros_like(self.rgba)
            self.mesh_buf = torch.empty(9 * (8 << 20), dtype=torch.float32, device=dev)
            if self.sharded:  # raycast / mesh composite of the sharded volume through a replica engine
                self.replica = tsdf_amd.Engine(a.voxel, a.trunc, max_width=W, max_height=H,
                                               num_block_bits=a.block_bits, device=torch.cuda.current_device(),
                                               stream=self.stream)
        self.sgraph = None
        if a.graph:
            if self.sharded:  # a shard's frame as three captured segments around the exchanges
                split = mode == "routed"
                self.sgraph = self.eng.shard_frame_graph(W, H, rank if split else 0, world if split else 1)
            else:
                rw, rh = (W, H) if a.loop == "c5" else (0, 0)
                self.graph = self.eng.frame_graph(W, H, rw, rh, deferred=bool(rw) and not a.no_defer,
                                                  batch=a.graph_batch)

    def step(self, i):
        from tsdf_amd import dist as tdist
        a, fr, K, pose = self.a, self.frame_views, self.K, self.poses[i]
        ht = None if a.depth_only else fr["ht"][i]
        lt = None if a.depth_only else fr["lt"][i]
        c5 = a.loop == "c5"
        if self.graph is not None:
            self.graph.frame(fr["rgb"][i], fr["depth"][i], ht, lt, K, pose, a.max_depth,
                             K if c5 else None, pose if c5 else None, self.rgba, self.normal)
        elif self.sharded:
            if a.broadcast_frames:  # the camera's frame reaches every rank from rank 0 (in the timed region)
                for t in (fr["rgb"][i], fr["depth"][i], ht, lt):
                    if t is not None:
                        self.dist.broadcast(t, src=0)
            if self.mode == "sharded" and self.sgraph is None:  # pipelined: one exchange per frame
                tdist.integrate_sharded_pipe(self.eng, self.bufs, fr["rgb"][i], fr["depth"][i], ht, lt, K, pose,
                                             a.max_depth)
            else:
                tdist.integrate_sharded(self.eng, self.bufs, fr["rgb"][i], fr["depth"][i], ht, lt, K, pose,
                                        a.max_depth, split=self.mode == "routed", graph=self.sgraph)
            if c5:
                self.flush()  # (the render reads the volume as of this frame)
                tdist.render_sharded(self.eng, self.replica, K, a.width, a.height, pose, a.max_depth,
                                     rgba=self.rgba, normal=self.normal)
        else:
            self.eng.integrate(fr["rgb"][i], fr["depth"][i], ht, lt, K, pose, a.max_depth)
            if c5:  # deferred: launched with the next frame's ingest (k_render_ingest), or by the flush
                self.eng.raycast(K, a.width, a.height, pose, a.max_depth, rgba=self.rgba, normal=self.normal,
                                 deferred=not a.no_defer)
        if c5 and (i + 1) % 30 == 0:  # marching cubes of the whole volume, on device
            if self.replica is not None:
                n = tdist.mesh_sharded(self.eng, self.replica, None, 0.99, 0, out=self.mesh_buf).shape[0]
            else:
                n = self.eng.extract_mesh(None, 0.99, 0, out=self.mesh_buf).shape[0]
            self.mesh_tris.append(int(n))

    def flush(self):
        """Complete the pending frames (pipelined single volume: tsdf_flush; pipelined sharded frames:
        the exchange protocol's steps)."""
        from tsdf_amd import dist as tdist
        if self.sharded and self.mode == "sharded" and self.sgraph is None:
            tdist.flush_sharded_pipe(self.eng, self.bufs)
        else:
            self.eng.flush()

    def timed(self):
        """warmup, then exactly `steps` timed frames between barrier + synchronize; returns the
        max-over-ranks elapsed seconds and this rank's profile of the timed window."""
        import torch
        from tsdf_amd import dist as tdist
        a = self.a
        for i in range(a.warmup):
            self.step(i)
        self.flush()
        torch.cuda.synchronize()
        if self.dist:
            self.dist.barrier()
        # start/stop events bound to every event_every-th k_integrate dispatch (hipExtLaunchKernel):
        # the kernel's own begin/end timestamps, nothing added to the stream; the device-clock spans
        # and the N_vis / N_upd sums cover every timed frame
        every = a.event_every or max(1, min(16, a.steps // 5))
        self.eng.profile_begin(integrate_only=True, every=(1 << 30) if a.no_events else every,
                               kernel_events=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(a.warmup, a.warmup + a.steps):
            self.step(i)
        # pipelined frames: the last frames' updates / carvings are enqueued here, inside the timed region
        self.flush()
        t_enq = time.perf_counter()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        if self.dist:
            self.dist.barrier()
        prof = self.eng.profile_end()
        self.host_enqueue_ms = (t_enq - t0) / a.steps * 1e3
        return tdist.max_over_ranks(t1 - t0, device=self.dev), prof

    def raycast_timing(self, reps=50):
        """k_raycast's C5 work alone: `reps` back-to-back raycasts of the last timed frame's camera
        into the final volume, bracketed by events on the engine stream (the whole tsdf_raycast call:
        view grid + bitmaps + k_raycast). Returns microseconds per call."""
        import torch
        a = self.a
        pose = self.poses[a.warmup + a.steps - 1]
        for _ in range(3):
            self.eng.raycast(self.K, a.width, a.height, pose, a.max_depth, rgba=self.rgba, normal=self.normal)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            self.eng.raycast(self.K, a.width, a.height, pose, a.max_depth, rgba=self.rgba, normal=self.normal)
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / reps

    def close(self):
        if self.graph is not None:
            self.graph.close()
        if self.sgraph is not None:
            self.sgraph.close()
        if self.replica is not None:
            self.replica.close()
        self.eng.close()


PIX_RECORD_BYTES = 20  # pixA {depth, range, logf ht, logf lt} + pixC rgb, written once per pixel


def pipe_fraction(prof):
    """Share of the frames whose update ran in a pipelined frame launch (k_frame: the update beside
    the previous frame's carving and the next frame's ingest)."""
    return prof.get("pipelined", 0) / max(prof.get("calls", 0), 1)


def kernel_roofline(a, prof, n_frames, pmc):
    """The frame kernel: SURVEY.md 8(d) algorithmic bytes of ONE frame / its average launch duration
    (this rank). Pipelined frames (k_frame: every launch of the timed window runs one frame's update,
    carving and allocation and the next frame's ingest): N_vis * 6156 + N_upd * 12 + 15 W H (12 W H
    depth-only). Unpipelined frames (k_integrate, e.g. the C5 loop, whose raycast reads every frame's
    finished volume): N_vis * 6156 + N_upd * 12 -- the frame image is read by k_ingest_dda, not by this
    kernel. What the launch moves beyond that (the pixel records, table probes, the occupancy bitmap)
    is implementation traffic: roofline.traffic (rocprofv3 PMC). The duration is the mean over the
    HIP start/stop events bound to the kernel's own dispatches; where none exist (graph-launched
    frames) it is the timed-window kernel-trace mean of this same command committed under profiles/
    (scripts/profile_integrate.sh), else unknown. Returns (read, write bytes, seconds, kind)."""
    W, H = a.width, a.height
    img_bytes = ((12 if a.depth_only else 15) * W * H) if pipe_fraction(prof) > 0 else 0
    alg_read = prof["sum_visible"] * BLOCK_READ_BYTES / n_frames + img_bytes
    alg_write = prof["sum_updated"] * 12 / n_frames
    t, kind = None, "no kernel duration (no dispatch events and no committed trace of this command)"
    if prof["frames"] > 0 and not a.no_events:
        t = prof["ms_integrate"] / prof["frames"] / 1e3
        kind = "HIP events bound to the frame kernel's dispatch (hipExtLaunchKernel), engine stream"
    elif pmc is not None and pmc.get("trace_kernel_avg_us"):
        t = pmc["trace_kernel_avg_us"] * 1e-6
        kind = ("rocprofv3 kernel trace of this command, timed-window mean of " + pmc.get("trace_kernel", "?") +
                " (" + os.path.relpath(PMC_FILE, ROOT) + ")")
    return alg_read, alg_write, t, kind


def implementation_bytes(a, prof):
    """Bytes per frame launch that SURVEY 8(d) does not count (a lower bound, by construction): the
    16 B pixel records the ingest writes and the update gathers back (each once), and -- pipelined --
    nothing else by design (the launch reads the next frame's image instead of this frame's; counted
    once in the algorithmic bytes)."""
    W, H = a.width, a.height
    return {"pixel_records_written": PIX_RECORD_BYTES * W * H,
            "pixel_records_read": PIX_RECORD_BYTES * W * H,
            "occupancy_bitmap_read": 512 * 1024}


def raycast_roofline(a, us_call):
    """C5's raycast beside the line: rays/s of the whole call, and -- from the k_raycast SQ counters
    committed under profiles/ for this image size -- its VALU issue rate against the chip's wave64
    VALU issue peak (the kernel is bound by each wave's chain of dependent lookups; the
    VALU fraction shows how much issue bandwidth that chain leaves idle). The rate is taken over the
    whole call (view grid + bitmaps + k_raycast), so it is a lower bound for the kernel's own."""
    rays = a.width * a.height
    out = {"kernel": "k_raycast", "bound": "latency (each wave's ~31 lookup trips: a view-grid cell load, then "
                                           "the voxel read, with ~4.7 waves per SIMD to hide them; DESIGN.md 4)",
           "us_per_call": round(us_call, 3), "rays_per_s": round(rays / (us_call * 1e-6), 1),
           "timing": "events around 50 back-to-back tsdf_raycast calls of the last timed camera, after the loop"}
    try:
        sq = json.load(open(RAYCAST_SQ_FILE))
    except (OSError, ValueError):
        return out
    if sq.get("width") == a.width and sq.get("height") == a.height:
        valu = sq["SQ_INSTS_VALU_per_wave"] * sq["SQ_WAVES"]
        achieved = valu / (us_call * 1e-6)
        out.update({"valu_instr_per_wave": sq["SQ_INSTS_VALU_per_wave"], "salu_instr_per_wave": sq["SQ_INSTS_SALU_per_wave"],
                    "waves": sq["SQ_WAVES"], "achieved": round(achieved / 1e12, 4), "peak": round(VALU_PEAK_WAVE_INSTR / 1e12, 4),
                    "unit": "T wave64 VALU instr/s", "frac": round(achieved / VALU_PEAK_WAVE_INSTR, 4),
                    "counters_source": os.path.relpath(RAYCAST_SQ_FILE, ROOT)})
    return out


def pmc_traffic(a, mode, world, prof):
    """roofline.traffic from a rocprofv3 --pmc pass of this same command (profiles/, written by
    scripts/summarize_prof.py): accepted only when the pass integrated the same frames."""
    key = pmc_key(a, mode, world)
    try:
        runs = json.load(open(PMC_FILE))["runs"]
    except (OSError, ValueError, KeyError):
        return None, "no PMC file (" + os.path.relpath(PMC_FILE, ROOT) + ")"
    for r in runs:
        if r.get("key") != key:
            continue
        if r.get("sum_visible") != prof["sum_visible"] or r.get("sum_updated") != prof["sum_updated"]:
            return None, (f"PMC pass of this command saw N_vis/N_upd sums {r.get('sum_visible')}/"
                          f"{r.get('sum_updated')}, this run {prof['sum_visible']}/{prof['sum_updated']}: rejected")
        return r, "rocprofv3 --pmc FETCH_SIZE (x2, gfx950) + WRITE_SIZE passes of this command, timed-window launches"
    return None, "no PMC pass of this command in " + os.path.relpath(PMC_FILE, ROOT)


def pmc_key(a, mode, world):
    return {"width": a.width, "height": a.height, "voxel": a.voxel, "trunc": a.trunc,
            "max_depth": a.max_depth, "depth_only": bool(a.depth_only), "block_bits": a.block_bits,
            "steps": a.steps, "warmup": a.warmup, "mode": mode, "n_gpus": world, "loop": a.loop,
            "graph": bool(a.graph), "pipelined": os.environ.get("TSDF_PIPELINE", "1") != "0"}


def device_spans(prof, n):
    us = lambda k: round(prof[k] / n * 1e3, 3)
    return {"ingest_dda": us("ms_ingest_device"), "resolve_alloc": us("ms_resolve_alloc_device"),
            "integrate": us("ms_integrate_device"), "resolve_delete": us("ms_resolve_delete_device"),
            "note": "in-kernel 100 MHz clock, mean per timed frame: ingest = k_ingest_dda start -> "
                    "last workgroup arrival; resolve_* = the resolvers (last-arriving workgroups of "
                    "k_ingest_dda / k_integrate, or k_frame's workgroup 0); integrate = the update's "
                    "first workgroup start -> its last workgroup end. Pipelined frames (one k_frame per "
                    "frame): ingest = the previous frame's allocation published -> the frame's last "
                    "tile / sweep workgroup end. C5 eager loop with deferred raycasts: ingest = "
                    "k_render_ingest, the previous frame's raycast beside this frame's ingest"}


def main():
    a = parse()
    import torch

    from tsdf_amd import dist as tdist

    rank, local, world = tdist.env_rank_world()
    if world != a.gpus and world != 1:
        raise SystemExit(f"WORLD_SIZE={world} but --gpus {a.gpus}")
    dist = None
    if world > 1:
        import torch.distributed as dist

        if a.backend == "gloo":  # rehearsal: ranks share the box's GPUs round-robin
            torch.cuda.set_device(local % torch.cuda.device_count())
            dist.init_process_group("gloo")
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    import tsdf_amd
    from tsdf_amd import synth

    cam = synth.camera(a.width, a.height, synth.TUM_FR1 if a.width <= 640 else synth.L515_FULL)
    K = tsdf_amd.CameraIntrinsics(*[float(v) for v in cam.K])
    nframes = a.warmup + a.steps
    if a.shard:
        return rehearsal(a, cam, K, dev)
    if a.broadcast_frames is None:  # one camera feeds the node: its broadcast is part of the frame
        a.broadcast_frames = a.backend == "nccl" and world > 1 and a.mode in ("routed", "sharded")
    if a.broadcast_frames and a.backend == "gloo":
        raise SystemExit("--broadcast-frames broadcasts device frames (RCCL); gloo is host-only")
    mode = a.mode if world > 1 else "single"

    def stream_frames(m):
        off = tdist.stream_offset(m, rank, world)  # streams: each rank's camera a third of an orbit apart
        fr = synth.render_torch(cam, list(range(off, off + nframes)), device=dev)
        return fr, [tsdf_amd.SE3(fr["q"][i], fr["t"][i]) for i in range(nframes)]

    frames, poses = stream_frames(mode)
    torch.cuda.synchronize()
    upload = None
    if a.host_frames:
        if world > 1:
            raise SystemExit("--host-frames is a single-GPU line")
        frames, upload = host_frames(a, frames)
    run = Run(a, mode, rank, world, dev, cam, frames, K, poses, dist)
    elapsed, prof = run.timed()
    st = run.eng.stats()
    if st["status"] != 0:
        raise SystemExit(f"engine status {st['status']:#x} after the timed run")
    value = tdist.units(mode, a.steps, world) / elapsed
    fps_stream = a.steps / elapsed  # frames/s of one stream (sharded: the job's only stream)
    W, H = a.width, a.height
    img_bytes = (12 if a.depth_only else 15) * W * H

    # ---- kernel-level roofline (this rank's frame kernel) ----
    pmc, pmc_src = pmc_traffic(a, mode, world, prof)
    alg_r, alg_w, t_int, ev_kind = kernel_roofline(a, prof, a.steps, pmc)
    alg = alg_r + alg_w
    achieved = alg / t_int / 1e9 if t_int else None
    achieved_r = alg_r / t_int / 1e9 if t_int else None
    # ---- frame-level roofline, SURVEY.md 8d (whole job) ----
    # bytes per frame of the job: sharded -- the ranks' visible blocks sum to the frame's, and every
    # rank reads its frame; streams / single -- every rank its own frame
    vis_sum, upd_sum = tdist.sum_over_ranks([prof["sum_visible"], prof["sum_updated"]], device=dev)
    n_img = world  # every rank reads a frame per step (its own, or the shared one)
    b_read = (vis_sum * BLOCK_READ_BYTES) / a.steps + n_img * img_bytes
    b_write = upd_sum * 12 / a.steps
    steps_per_s = a.steps / elapsed
    frame_frac_read = b_read * steps_per_s / (world * HBM_PEAK_GBS * 1e9)
    frame_frac_rw = (b_read + b_write) * steps_per_s / (world * HBM_PEAK_GBS * 1e9)
    mesh_tris = run.mesh_tris[-1] if run.mesh_tris else None
    ray = None
    if a.loop == "c5" and not run.sharded:
        ray = raycast_roofline(a, run.raycast_timing())
    host_enq = run.host_enqueue_ms
    exch = None
    if run.sharded:  # bytes this rank moved per frame (rank 0's view)
        ks, cs = run.bufs.keys_out.numel(), run.bufs.cands_out.numel()
        exch = {"key_slot_bytes_allgathered": ks * world if mode == "routed" else 0,
                "cand_slot_bytes_allgathered": cs * world,
                "frames_broadcast_in_timed_loop": bool(a.broadcast_frames)}
        exch.update({k: v for k, v in tdist.last_exchange.items()})
    run.close()
    del frames

    secondary = None
    if world > 1 and a.secondary == "streams" and mode != "streams":
        fr2, po2 = stream_frames("streams")
        torch.cuda.synchronize()
        r2 = Run(a, "streams", rank, world, dev, cam, fr2, K, po2, dist)
        el2, _ = r2.timed()
        r2.close()
        secondary = {"mode": "streams", "value": round(tdist.units("streams", a.steps, world) / el2, 2),
                     "unit": "frames/s", "scaling": "weak",
                     "ms_per_step": round(el2 / a.steps * 1e3, 4),
                     "what": "each rank integrates its own camera stream into its own volume (multi-camera "
                             "rig; no data-path collective); value = all ranks' frames / max rank time"}

    bcast = None
    if world > 1 and mode in ("routed", "sharded"):
        bcast = frame_broadcast_ms(a, dist, None, dev)
    cpp = None
    if rank == 0 and world == 1 and a.loop == "c3" and not a.graph and not a.host_frames and not a.no_cpp_loop:
        cpp = cpp_loop(a, cam, nframes)
    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu:
        fr_host = synth.render_torch(cam, list(range(0, min(nframes, 80))), device=dev)
        cpu = cpu_baseline(a, cam, fr_host)

    if rank == 0:
        metric = (f"TSDF integrate frames/s ({W}x{H} depth{'' if a.depth_only else '+label'}, "
                  f"{a.voxel * 1000:g}mm voxel)")
        if a.loop == "c5":
            metric = ("C5 frame loop frames/s (integrate + raycast every frame, marching cubes every 30 "
                      "frames)")
        parallelism = "single" if world == 1 else f"{mode}{world}"
        if world > 1 and a.backend == "gloo":
            parallelism += " (gloo rehearsal, ranks sharing GPUs: not a performance number)"
        if a.graph:
            parallelism += ", one hipGraph launch per frame"
        pf = pipe_fraction(prof)
        roof = {
            "kernel": ("k_integrate_vg (k_integrate + the deferred raycast's view grid)"
                       if a.loop == "c5" and not a.graph and not a.no_defer and world == 1 else "k_integrate")
                      if pf == 0 else
                      "k_frame (one launch per frame: frame b-1's carving then frame b's allocation in "
                      "workgroup 0, frame b's update beside them, frame b+1's pixel records, DDA, key "
                      "dedupe, probe / insert and visibility sweep)",
            "pipelined_fraction": round(pf, 4),
            "bound": "hbm",
            "achieved": None if achieved is None else round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            # frac: the launch's algorithmic read + write bytes (reads and writes share the HBM);
            # frac_read: SURVEY 8(d)'s read bytes alone, over the same duration
            "frac": None if achieved is None else round(achieved / HBM_PEAK_GBS, 4),
            "frac_read_write": None if achieved is None else round(achieved / HBM_PEAK_GBS, 4),
            "frac_read": None if achieved_r is None else round(achieved_r / HBM_PEAK_GBS, 4),
            "traffic": None if pmc is None else int(pmc["hbm_bytes_per_launch"]),
            "traffic_read": None if pmc is None else int(pmc["fetch_bytes_per_launch"]),
            "traffic_write": None if pmc is None else int(pmc["write_bytes_per_launch"]),
            "traffic_source": pmc_src,
            "alg_bytes_per_launch": int(alg),
            "alg_read_bytes_per_launch": int(alg_r),
            "alg_def": ("SURVEY 8(d) per frame launch: N_vis * 6156 + N_upd * 12 + 15 W H (N_vis, N_upd counted on "
                        "device over the timed frames)") if pf > 0 else
                       ("SURVEY 8(d) per k_integrate launch: N_vis * 6156 + N_upd * 12 (the frame image is read "
                        "by k_ingest_dda)"),
            "implementation_bytes_per_launch": implementation_bytes(a, prof),
            "us_per_launch": None if t_int is None else round(t_int * 1e6, 3),
            "event_timed_launches": prof["frames"],
            "event_kind": ev_kind,
            "us_per_launch_device_clock": round(prof["ms_integrate_device"] / a.steps * 1e3, 3),
            "frame": {  # B_read * frames/s / (N x 8 TB/s)
                "bytes_read_per_step": int(b_read),
                "bytes_written_per_step": int(b_write),
                "frac_read": round(frame_frac_read, 4),
                "frac_read_write": round(frame_frac_rw, 4),
                "def": "B_read = 15 W H per frame read + N_vis * 6156 B; write = N_upd * 12 B; "
                       "fraction of N GPUs x 8 TB/s at the measured step rate",
            },
        }
        out = {
            "metric": metric,
            "value": round(value, 2),
            "unit": "frames/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak" if mode == "streams" else ("strong" if world > 1 else "weak"),
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (analytic room scene rendered on GPU, resident in HBM)",
            "config": {
                "workload": workload_name(a),
                "width": W, "height": H, "voxel_m": a.voxel, "truncation_m": a.trunc,
                "pool_blocks": 1 << a.block_bits,
                "parallelism": parallelism,
                "graph_frames_per_launch": a.graph_batch if a.graph else None,
            },
            "roofline": roof,
            "cpu_baseline": cpu,
            "device_us_per_frame": device_spans(prof, a.steps),
            "host_enqueue_ms_per_step": round(host_enq, 4),
            "pmc_key": pmc_key(a, mode, world),  # what scripts/summarize_prof.py files a PMC pass under
            "sum_visible": prof["sum_visible"],
            "sum_updated": prof["sum_updated"],
            "avg_visible_blocks": round(prof["sum_visible"] / a.steps, 1),
            "avg_updated_voxels": round(prof["sum_updated"] / a.steps, 1),
            "active_blocks": st["active_blocks"],
            "mesh_triangles": mesh_tris,
            "status": st["status"],
        }
        if ray is not None:
            out["raycast"] = ray
        if cpp is not None:
            out["cpp_loop"] = cpp
        if upload is not None:
            out["host_frames"] = upload
        if world > 1:
            out["frames_per_s_per_stream"] = round(fps_stream, 2)
        if bcast is not None:
            out["frame_broadcast_ms"] = bcast
        if exch:
            out["exchange_per_rank"] = exch
        if secondary:
            out["secondary"] = secondary
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


def cpp_loop(a, cam, nframes):
    """The same stream and timed window through disinfect-slam_amd/bench_main (C++, the C ABI with
    device frames on the engine's own stream, no Python in the loop): frames/s and the host enqueue per
    frame -- the facade's own overhead, beside the Python line's host_enqueue_ms_per_step. The frames
    are this bench's (synth.render_torch), written to a scratch directory for the child process."""
    import shutil
    import subprocess
    import tempfile

    from tsdf_amd import synth
    exe = os.path.join(os.path.dirname(os.path.abspath(__file__)), "disinfect-slam_amd", "bench_main")
    if not os.path.exists(exe):
        return {"skipped": "bench_main not built"}
    n = a.warmup + a.steps
    fr = synth.render_torch(cam, list(range(0, n)), device="cuda")
    d = tempfile.mkdtemp(prefix="tsdf_cpp_loop_")
    try:
        lines = [f"{a.width} {a.height} {n} " + " ".join(repr(float(v)) for v in cam.K) +
                 f" {a.voxel} {a.trunc} {a.max_depth} {int(not a.depth_only)} {a.block_bits}"]
        for i in range(n):
            for k in ("rgb", "depth", "ht", "lt"):
                fr[k][i].cpu().numpy().tofile(os.path.join(d, f"f{i}_{k}.bin"))
            lines.append(" ".join(repr(float(v)) for v in list(fr["q"][i]) + list(fr["t"][i])))
        with open(os.path.join(d, "meta.txt"), "w") as f:
            f.write("\n".join(lines) + "\n")
        del fr
        r = subprocess.run([exe, d, str(a.warmup), str(a.steps)], capture_output=True, text=True, timeout=120)
        if r.returncode != 0:
            return {"failed": (r.stdout + r.stderr)[-400:]}
        out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
        out["what"] = ("bench_main: this line's stream and window through the C ABI from C++ (tsdf_integrate "
                       "with device frames, tsdf_flush, tsdf_synchronize; no Python) -- the host enqueue floor")
        return out
    finally:
        shutil.rmtree(d, ignore_errors=True)


def host_frames(a, fr, reps=20):
    """--host-frames: the stream's frames copied to host memory (pageable numpy arrays, or pinned torch
    tensors), and the upload alone timed: `reps` uploads of one frame's four arrays (rgb u8, depth /
    ht / lt f32) into device buffers on a side stream, between events -- the PCIe share of a frame."""
    import numpy as np
    import torch
    keys = ("rgb", "depth") + (() if a.depth_only else ("ht", "lt"))
    out = dict(fr)
    for k in keys:
        t = fr[k].cpu()
        out[k] = [t[i].pin_memory() for i in range(t.shape[0])] if a.host_frames == "pinned" else \
                 [np.ascontiguousarray(t[i].numpy()) for i in range(t.shape[0])]
    dst = {k: torch.empty_like(fr[k][0]) for k in keys}
    src = {k: (out[k][0] if a.host_frames == "pinned" else torch.from_numpy(out[k][0])) for k in keys}
    st = torch.cuda.Stream()
    nbytes = sum(v.numel() * v.element_size() for v in dst.values())
    with torch.cuda.stream(st):
        for k in keys:
            dst[k].copy_(src[k], non_blocking=True)
        st.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):
            for k in keys:
                dst[k].copy_(src[k], non_blocking=True)
        e1.record(st)
        st.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    return out, {"kind": a.host_frames, "bytes_per_frame": int(nbytes), "h2d_us_per_frame": round(us, 2),
                 "h2d_gbs": round(nbytes / (us * 1e-6) / 1e9, 2),
                 "note": "upload alone: 4 host-to-device copies of one frame on a side stream, events, "
                         f"{reps} reps; the line's value includes the engine's own "
                         "uploads (copies over two upload streams, overlapped with the previous frames' kernels; "
                         "each call returns once its frame's copies are complete)"}


def frame_broadcast_ms(a, dist, _unused, dev, reps=20):
    """Time of rank 0 broadcasting one frame (rgb u8 + depth / ht / lt f32) to every rank -- what a
    single camera feeding an N-GPU sharded volume adds per frame (reported beside the line unless
    --broadcast-frames puts it in the timed loop)."""
    import torch
    W, H = a.width, a.height
    bufs = [torch.zeros((H, W, 3), dtype=torch.uint8, device=dev)] + \
           [torch.zeros((H, W), dtype=torch.float32, device=dev) for _ in range(1 if a.depth_only else 3)]
    if a.backend == "gloo":
        bufs = [b.cpu() for b in bufs]
    for b in bufs:
        dist.broadcast(b, src=0)
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        for b in bufs:
            dist.broadcast(b, src=0)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    from tsdf_amd import dist as tdist
    return {"ms_per_frame": round(tdist.max_over_ranks(el, device=dev) / reps * 1e3, 4),
            "bytes_per_frame": int(sum(b.numel() * b.element_size() for b in bufs)),
            "backend": a.backend}


def rehearsal(a, cam, K, dev):
    """--shard G: the routed sharded volume's G shards on this one GPU (tsdf_amd.ShardGroup: slots
    exchanged with device copies where a G-GPU job all-gathers them). The group's frame time is the
    sum of the shards' own kernels; reported per shard as that time / G, beside each shard's in-kernel
    device-clock spans (the slowest shard bounds a G-GPU job's frame, plus the two all-gathers)."""
    import torch

    import tsdf_amd
    from tsdf_amd import synth
    G = int(a.shard)
    nframes = a.warmup + a.steps
    fr = synth.render_torch(cam, list(range(nframes)), device=dev)
    poses = [tsdf_amd.SE3(fr["q"][i], fr["t"][i]) for i in range(nframes)]
    pipe = a.mode == "sharded" and not a.graph  # pipelined sharded frames: one exchange per frame
    if a.native_group:  # the library-owned group (tsdf_group_*): the update kernels write every inbox
        grp = tsdf_amd.Group([torch.cuda.current_device()] * G, a.voxel, a.trunc, max_width=a.width,
                             max_height=a.height, num_block_bits=a.block_bits)
        grp.engines = None
    else:
        grp = tsdf_amd.ShardGroup(G, a.voxel, a.trunc, max_width=a.width, max_height=a.height,
                                  num_block_bits=a.block_bits, device=torch.cuda.current_device(),
                                  key_cap=a.key_cap or max(1024, 32768 // G),
                                  cand_cap=a.cand_cap or max(1024, 16384 // G), split=a.mode != "sharded",
                                  graph=(a.width, a.height) if a.graph else None, pipe=pipe)

    def step(i):
        ht = None if a.depth_only else fr["ht"][i]
        lt = None if a.depth_only else fr["lt"][i]
        grp.integrate(fr["rgb"][i], fr["depth"][i], ht, lt, K, poses[i], a.max_depth)

    for i in range(a.warmup):
        step(i)
    grp.flush()
    torch.cuda.synchronize()
    if a.native_group:
        grp.engines = [grp.shard(i) for i in range(G)]
    for e in grp.engines:
        e.profile_begin(integrate_only=True, every=1 << 30)
    t0 = time.perf_counter()
    for i in range(a.warmup, nframes):
        step(i)
    grp.flush()  # (pipelined: the last frames complete inside the timed region)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    profs = [e.profile_end() for e in grp.engines]
    for e in grp.engines:
        if e.stats()["status"]:
            raise SystemExit("a shard engine reported a status")
    n = a.steps
    spans = [device_spans(p, n) for p in profs]
    for s in spans:
        s.pop("note")
    dev_total = [sum(v for v in s.values()) for s in spans]
    out = {
        "metric": "sharded-volume rehearsal: per-shard frame time (one GPU, G shard engines)",
        "value": round(el / n / G * 1e3, 4),
        "unit": "ms/frame/shard",
        "n_gpus": 1,
        "steps": n,
        "warmup": a.warmup,
        "ms_per_step": round(el / n * 1e3, 4),
        "higher_is_better": False,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (analytic room scene rendered on GPU, resident in HBM)",
        "config": {"workload": workload_name(a), "width": a.width, "height": a.height,
                   "parallelism": (f"{G} shards on one GPU, library-owned group (tsdf_group_*: pipelined shard "
                                   "frames, candidates written into every inbox by the update kernels)")
                   if a.native_group else
                   f"{G} {'routed' if a.mode != 'sharded' else 'sharded (pipelined, one exchange per frame)'} shards on one GPU"},
        "shards": G,
        "group_ms_per_frame": round(el / n * 1e3, 4),
        "per_shard_device_us": spans,
        "max_shard_device_us_per_frame": round(max(dev_total), 3),
        "avg_visible_blocks_per_shard": [round(p["sum_visible"] / n, 1) for p in profs],
    }
    grp.close()
    print(json.dumps(out), flush=True)


def cpu_baseline(a, cam, fr):
    """Single-thread oracle on the first frames of the bench's own stream (GPU frames copied to the
    host), from an empty map, ~20 s of CPU work."""
    from _oracle import OracleGrid

    ora = OracleGrid(a.voxel, a.trunc, a.block_bits)
    host = {k: (v.cpu().numpy() if hasattr(v, "cpu") else v) for k, v in fr.items()}
    n_avail = host["depth"].shape[0]
    n = a.cpu_frames
    budget = 20.0
    done, spent = 0, 0.0
    while done < n_avail:
        if n >= 0 and done >= n:
            break
        if n < 0 and spent >= budget:
            break
        ht = None if a.depth_only else host["ht"][done]
        lt = None if a.depth_only else host["lt"][done]
        t0 = time.perf_counter()
        ora.integrate(host["rgb"][done], host["depth"][done], ht, lt, a.max_depth, cam.K,
                      host["q"][done], host["t"][done])
        spent += time.perf_counter() - t0
        done += 1
    ora.close()
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {
        "value": round(done / spent, 4),
        "unit": "frames/s",
        "cores": 1,
        "kind": "port",
        "sample": f"frames 0..{done - 1} of this bench's own {cam.width}x{cam.height} stream (GPU-rendered "
                  f"frames copied to the host) from an empty map, single thread, oracle/tsdf_oracle.c -O2 "
                  f"(host: {model}, nproc={os.cpu_count()}); the GPU line times frames {a.warmup}.."
                  f"{a.warmup + a.steps - 1} of the same stream after {a.warmup} warm-up frames",
    }


if __name__ == "__main__":
    main()
