#!/usr/bin/env python3
"""bench.py -- TSDF integrate frames/s on MI355X (BASELINE.json metric), one JSON line on rank 0.

Workload (N=1): BASELINE.json configs[2] -- synthetic 640x480 depth + per-pixel high/low-touch
probability maps (the segmentation/inference output shape), fused TSDF + RGB + semantic integrate
into a 5 mm voxel-hash volume (3 cm truncation, 4 m max depth, TUM fr1 intrinsics). One step =
one TSDFGrid::Integrate of one frame: DDA block allocation, visibility, fused update, space
carving. All frames are rendered on the GPU and resident in HBM before timing starts.

N>1 (launched by torch.distributed.run, one rank per GPU): default --mode streams runs one camera
stream per GPU into that GPU's own volume (a multi-camera rig; no data-path collective), value =
all frames integrated by all ranks / max rank time, scaling "weak". --mode sharded integrates ONE
stream with the volume spatially sharded by 4^3-block bricks (each rank allocates and integrates
only the blocks it owns), value = frames / max rank time, scaling "strong". --mode routed shards the
same way but splits the block-allocation DDA by pixel-tile rows across ranks and routes each
visible key to its owner with one RCCL all-to-all per frame (SURVEY.md 8e option 2), "strong".

roofline: the fused integrate kernel (k_integrate). Algorithmic bytes per launch:
N_vis * (512 * 12 + 12) voxel state + block metadata read, N_upd * 12 updated voxel state written,
15 * W * H frame bytes read -- N_vis and N_upd are counted on device. Average launch duration from
HIP start/stop events bound to every k_integrate launch of the timed region on the engine stream
(hipExtLaunchKernel: the dispatch's own begin/end timestamps, the interval a rocprofv3 kernel
trace reports); --marker-events times with marker events recorded around the launch instead (each
carries a system-scope release, i.e. an L2 writeback, so it reads a few us longer). The in-kernel
device clock of every launch is reported beside it.
cpu_baseline: the single-threaded CPU oracle (oracle/tsdf_oracle.c, a restatement of the
reference kernels incl. its full-table visibility scan) on a bounded sample of the same stream.
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
    p.add_argument("--mode", choices=("streams", "sharded", "routed"), default="streams")
    p.add_argument("--loop", choices=("c3", "c5"), default="c3",
                   help="c5: BASELINE config C5 -- per frame one hipGraph launch (integrate + raycast of "
                        "the frame's camera), marching cubes of the whole volume every 30 frames")
    p.add_argument("--graph", action="store_true",
                   help="c3 loop through the graph-captured frame (one hipGraph launch per frame)")
    p.add_argument("--shard", default=None, metavar="I/G",
                   help="single-GPU rehearsal of --mode sharded: run shard I of G alone (the G-GPU rate is "
                        "the slowest shard's; every shard sees the whole frame)")
    p.add_argument("--streams-per-gpu", type=int, default=1,
                   help="camera streams per GPU, each its own engine (volume) and HIP stream; their "
                        "frame chains overlap on the device (multi-camera rig; value counts all streams)")
    p.add_argument("--key-cap", type=int, default=16384,
                   help="sharded modes: key records per rank per frame (exchange slot size)")
    p.add_argument("--cand-cap", type=int, default=8192,
                   help="sharded modes: carve-candidate records per rank per frame")
    p.add_argument("--cpu-frames", type=int, default=-1, help="oracle sample size (-1 = auto)")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--block-bits", type=int, default=18)
    p.add_argument("--event-every", type=int, default=8,
                   help="HIP-event-time k_integrate on every n-th timed frame (a profiled dispatch "
                        "runs ~1 us slower, so the loop samples)")
    p.add_argument("--marker-events", action="store_true",
                   help="time k_integrate with marker events recorded around the launch (each is a "
                        "queue marker with a system-scope release: ~3 us of cache writeback each) "
                        "instead of events bound to the kernel's dispatch")
    p.add_argument("--no-events", action="store_true",
                   help="diagnostic: no HIP events in the timed loop (roofline then unmeasured)")
    return p.parse_args()


def main():
    a = parse()
    import numpy as np
    import torch

    from tsdf_amd import dist as tdist

    rank, local, world = tdist.env_rank_world()
    if world != a.gpus and world != 1:
        raise SystemExit(f"WORLD_SIZE={world} but --gpus {a.gpus}")
    dist = None
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    import tsdf_amd
    from tsdf_amd import synth

    cam = synth.camera(a.width, a.height,
                       synth.TUM_FR1 if a.width <= 640 else synth.L515_FULL)
    nphase = min(100, a.steps)  # untimed phase-breakdown pass after the timed region
    nframes = a.warmup + a.steps + nphase
    # streams mode: each rank's camera starts a third of an orbit apart (its own stream)
    offset = tdist.stream_offset(a.mode, rank, world)
    frames = synth.render_torch(cam, list(range(offset, offset + nframes)), device=dev)
    torch.cuda.synchronize()
    shard_index, shard_count = tdist.shard_of(a.mode, rank, world)
    if a.shard:
        if world != 1:
            raise SystemExit("--shard is a single-process rehearsal; use --mode sharded with N ranks")
        shard_index, shard_count = (int(v) for v in a.shard.split("/"))
        if not 0 <= shard_index < shard_count:
            raise SystemExit("--shard I/G needs 0 <= I < G")
    stream = torch.cuda.current_stream()
    eng = tsdf_amd.Engine(a.voxel, a.trunc, max_width=a.width, max_height=a.height,
                          num_block_bits=a.block_bits, device=torch.cuda.current_device(),
                          shard_index=shard_index, shard_count=shard_count,
                          stream=stream.cuda_stream)
    K = tsdf_amd.CameraIntrinsics(*[float(v) for v in cam.K])  # ctypes struct cached once
    poses = [tsdf_amd.SE3(frames["q"][i], frames["t"][i]) for i in range(nframes)]

    routed = a.mode == "routed" and shard_count > 1 and not a.shard
    # --streams-per-gpu: further engines, each on its own HIP stream with its own camera stream
    extra = []
    for k in range(1, a.streams_per_gpu):
        if routed or a.loop == "c5" or a.graph or shard_count > 1:
            raise SystemExit("--streams-per-gpu > 1 takes the eager c3 loop in streams mode")
        off_k = offset + 97 * k  # a different stretch of the orbit per camera
        fr_k = synth.render_torch(cam, list(range(off_k, off_k + nframes)), device=dev)
        s_k = torch.cuda.Stream()
        e_k = tsdf_amd.Engine(a.voxel, a.trunc, max_width=a.width, max_height=a.height,
                              num_block_bits=a.block_bits, device=torch.cuda.current_device(),
                              stream=s_k.cuda_stream)
        extra.append((e_k, fr_k, [tsdf_amd.SE3(fr_k["q"][i], fr_k["t"][i]) for i in range(nframes)], s_k))
    torch.cuda.synchronize()
    if shard_count > 1:  # exchange slots of the sharded frame (RCCL all-gathers on this stream)
        bufs = tdist.ShardBuffers(eng, shard_count, a.key_cap, a.cand_cap, device=dev)

    use_graph = a.loop == "c5" or a.graph
    if use_graph and routed:
        raise SystemExit("--graph / --loop c5 take streams or sharded mode")
    graph = None
    mesh_tris = []
    # C5 over a sharded volume: the graph frame integrates only; every frame's render is the raycast
    # composite (tsdf_amd.dist.render_sharded: view-selected block records all-gathered over RCCL
    # into a replica engine, raycast there), since one shard's own raycast sees only its blocks
    composite = a.loop == "c5" and shard_count > 1
    replica = None
    if use_graph:
        rw, rh = (a.width, a.height) if (a.loop == "c5" and not composite) else (0, 0)
        graph = eng.frame_graph(a.width, a.height, rw, rh)
        rgba = torch.zeros((a.height, a.width, 4), dtype=torch.uint8, device=dev) if rw else None
        normal = torch.zeros_like(rgba) if rw else None
        if composite:
            replica = tsdf_amd.Engine(a.voxel, a.trunc, max_width=a.width, max_height=a.height,
                                      num_block_bits=a.block_bits, device=torch.cuda.current_device(),
                                      stream=stream.cuda_stream)
            c_rgba = torch.zeros((a.height, a.width, 4), dtype=torch.uint8, device=dev)
            c_normal = torch.zeros_like(c_rgba)
        mesh_buf = torch.empty(9 * (8 << 20), dtype=torch.float32, device=dev) if a.loop == "c5" else None

    def step(i):
        ht = None if a.depth_only else frames["ht"][i]
        lt = None if a.depth_only else frames["lt"][i]
        if graph is not None:
            graph.frame(frames["rgb"][i], frames["depth"][i], ht, lt, K, poses[i], a.max_depth,
                        K if rgba is not None else None, poses[i] if rgba is not None else None, rgba, normal)
            if replica is not None:
                tdist.render_sharded(eng, replica, K, a.width, a.height, poses[i], a.max_depth,
                                     rgba=c_rgba, normal=c_normal)
            if a.loop == "c5" and (i + 1) % 30 == 0:  # marching cubes of the whole volume (on device)
                if replica is not None:  # sharded: all blocks gathered into the replica first
                    mesh_tris.append(int(tdist.mesh_sharded(eng, replica, None, 0.99, 0,
                                                            out=mesh_buf).shape[0]))
                else:
                    mesh_tris.append(int(eng.extract_mesh(None, 0.99, 0, out=mesh_buf).shape[0]))
        elif shard_count > 1:
            tdist.integrate_sharded(eng, bufs, frames["rgb"][i], frames["depth"][i], ht, lt, K, poses[i],
                                    a.max_depth, split=a.mode == "routed")
        else:
            eng.integrate(frames["rgb"][i], frames["depth"][i], ht, lt, K, poses[i], a.max_depth)
        for e_k, fr_k, po_k, _ in extra:
            e_k.integrate(fr_k["rgb"][i], fr_k["depth"][i], None if a.depth_only else fr_k["ht"][i],
                          None if a.depth_only else fr_k["lt"][i], K, po_k[i], a.max_depth)

    for i in range(a.warmup):
        step(i)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    if not a.no_events:
        # default: start/stop events bound to every k_integrate dispatch (hipExtLaunchKernel) --
        # the kernel's begin/end timestamps on the engine stream, nothing added to the stream.
        # --marker-events: 2 marker events around the launch on every event_every-th frame
        eng.profile_begin(integrate_only=True, every=a.event_every, kernel_events=not a.marker_events)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.warmup, a.warmup + a.steps):
        step(i)
    t_enq = time.perf_counter()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if dist:
        dist.barrier()
    if a.no_events:  # device-clock and counters still come from a profile window
        eng.profile_begin(integrate_only=True)
    prof = eng.profile_end()
    # phase breakdown (all four phases event-bracketed) on the next frames of the stream, untimed
    eng.profile_begin()
    for i in range(a.warmup + a.steps, nframes):
        if graph is not None:  # graph frames carry no events: the eager calls of the same frame
            eng.integrate(frames["rgb"][i], frames["depth"][i], None if a.depth_only else frames["ht"][i],
                          None if a.depth_only else frames["lt"][i], K, poses[i], a.max_depth)
        else:
            step(i)
    torch.cuda.synchronize()
    phases = eng.profile_end()
    st = eng.stats()
    elapsed = t1 - t0
    elapsed = tdist.max_over_ranks(elapsed, device=dev)
    value = tdist.units(a.mode, a.steps, world) * a.streams_per_gpu / elapsed
    for e_k, _, _, _ in extra:
        if e_k.stats()["status"] != 0:
            raise SystemExit("a further stream's engine reported a status")

    # ---- roofline of the fused integrate kernel (this rank's launches) ----
    W, H = a.width, a.height
    img_bytes = (12 if a.depth_only else 15) * W * H
    alg_bytes = (prof["sum_visible"] * (512 * 12 + 12) + prof["sum_updated"] * 12) / a.steps + img_bytes
    t_int = prof["ms_integrate"] / max(prof["frames"], 1) / 1e3
    event_kind = "marker" if a.marker_events else "kernel-dispatch"
    if graph is not None:  # graph frames carry no events: the in-kernel device clock
        t_int = prof["ms_integrate_device"] / a.steps / 1e3
        event_kind = "none (graph frames): device clock"
    achieved = alg_bytes / t_int / 1e9 if t_int > 0 else 0.0
    traffic = None
    pmc_path = os.path.join(ROOT, "profiles", "pmc_integrate_latest.json")
    if os.path.exists(pmc_path):
        try:
            pmc = json.load(open(pmc_path))
            if pmc.get("width") == W and pmc.get("height") == H:
                traffic = pmc.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu:
        cpu = cpu_baseline(a, cam)

    if rank == 0:
        workload = ("C2: 640x480 depth-only" if a.depth_only else "C3: 640x480 depth + ht/lt semantic")
        if (W, H) != (640, 480):
            workload = f"{W}x{H} depth{'' if a.depth_only else ' + ht/lt semantic'}"
        if a.streams_per_gpu > 1:
            workload += f", {a.streams_per_gpu} camera streams per GPU (one volume each)"
        metric = "TSDF integrate frames/s (640x480 depth+label, 5mm voxel)"
        if a.loop == "c5":
            metric = ("C5 frame loop frames/s (integrate + raycast every frame, marching cubes every 30 "
                      "frames, one hipGraph launch per frame)")
            workload = "C5: " + workload
            if replica is not None:
                workload += (", sharded volume: per-frame raycast composite (view-selected block records "
                             "all-gathered into a replica engine), marching cubes of the gathered volume")
        elif graph is not None:
            workload += " (hipGraph frame)"
        out = {
            "metric": metric,
            "value": round(value, 2),
            "unit": "frames/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak" if a.mode == "streams" else "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (analytic room scene rendered on GPU, resident in HBM)",
            "config": {
                "workload": workload + f", {a.voxel * 1000:g} mm voxel, {a.trunc * 100:g} cm truncation, "
                            f"{a.max_depth:g} m max depth, {'TUM fr1' if W <= 640 else 'L515 full-res'} intrinsics, "
                            "orbit 1 cm + 0.5 deg/frame",
                "width": W, "height": H, "voxel_m": a.voxel, "truncation_m": a.trunc,
                "pool_blocks": 1 << a.block_bits,
                "parallelism": (f"{a.mode}{world}" if world > 1 else
                                f"shard {shard_index} of {shard_count} alone (sharded-mode rehearsal)"
                                if shard_count > 1 else "single"),
            },
            "roofline": {
                "kernel": "k_integrate",
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "alg_bytes_per_launch": int(alg_bytes),
                "us_per_launch": round(t_int * 1e6, 3),
                # cross-check: first-WG start -> last-WG end from the in-kernel 100 MHz clock
                # (what rocprofv3's kernel trace measures; the HIP events above also include the
                # per-launch dispatch / completion overhead)
                "event_timed_launches": prof["frames"],
                "event_kind": event_kind,
                "us_per_launch_device_clock": round(prof["ms_integrate_device"] / a.steps * 1e3, 3),
                "achieved_device_clock": round(alg_bytes / (prof["ms_integrate_device"] / a.steps / 1e3) / 1e9, 1)
                if prof["ms_integrate_device"] > 0 else None,
            },
            "cpu_baseline": cpu,
            "phases_ms_per_frame": {  # separate untimed pass of nphase frames
                "frames": nphase,
                "allocate": round(phases["ms_allocate"] / nphase, 4),
                "visibility": round(phases["ms_visible"] / nphase, 4),
                "integrate": round(phases["ms_integrate"] / nphase, 4),
                "carve": round(phases["ms_carve"] / nphase, 4),
            },
            "host_enqueue_ms_per_step": round((t_enq - t0) / a.steps * 1e3, 4),
            "avg_visible_blocks": round(prof["sum_visible"] / a.steps, 1),
            "mesh_triangles": mesh_tris[-1] if mesh_tris else None,
            "avg_updated_voxels": round(prof["sum_updated"] / a.steps, 1),
            "active_blocks": st["active_blocks"],
            "status": st["status"],
        }
        print(json.dumps(out), flush=True)
    if graph is not None:
        graph.close()
    for e_k, _, _, _ in extra:
        e_k.close()
    if replica is not None:
        replica.close()
    eng.close()
    if dist:
        dist.destroy_process_group()


def cpu_baseline(a, cam):
    """Single-thread oracle on the first frames of the same stream (empty map), host frames."""
    import numpy as np

    from tsdf_amd import synth
    from _oracle import OracleGrid

    ora = OracleGrid(a.voxel, a.trunc, a.block_bits)
    n = a.cpu_frames
    budget = 20.0
    frames_done, spent = 0, 0.0
    i = 0
    while True:
        if n >= 0 and frames_done >= n:
            break
        if n < 0 and (spent >= budget or frames_done >= 60):
            break
        fr = synth.render(cam, i)
        ht = None if a.depth_only else fr["ht"]
        lt = None if a.depth_only else fr["lt"]
        t0 = time.perf_counter()
        ora.integrate(fr["rgb"], fr["depth"], ht, lt, a.max_depth, cam.K, fr["q"], fr["t"])
        spent += time.perf_counter() - t0
        frames_done += 1
        i += 1
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
        "value": round(frames_done / spent, 4),
        "unit": "frames/s",
        "cores": 1,
        "kind": "port",
        "sample": f"first {frames_done} frames of the same {cam.width}x{cam.height} stream from an empty "
                  f"map, single thread, oracle/tsdf_oracle.c -O2 (host: {model}, nproc={os.cpu_count()})",
    }


if __name__ == "__main__":
    main()
