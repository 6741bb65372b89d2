"""Per-workgroup raycast statistics from the DIAG build (TSDF_AMD_LIB=libdisinfect_tsdf_diag.so):
integrate the bench stream, raycast the last frame's view, print the distribution of workgroup
durations and of the lanes' batches / jumps / region steps, slowest tiles first."""
import sys, os, numpy as np
sys.path.insert(0, "disinfect-slam_amd")
import torch, tsdf_amd, ctypes as C
from tsdf_amd import synth, _lib
W, H, N = 640, 480, int(sys.argv[1]) if len(sys.argv) > 1 else 40
cam = synth.camera(W, H, synth.TUM_FR1)
fr = synth.render_torch(cam, list(range(N)), device="cuda")
K = tsdf_amd.CameraIntrinsics(*[float(v) for v in cam.K])
e = tsdf_amd.Engine(0.005, 0.03, max_width=W, max_height=H, num_block_bits=18)
for i in range(N):
    e.integrate(fr["rgb"][i], fr["depth"][i], fr["ht"][i], fr["lt"][i], K, tsdf_amd.SE3(fr["q"][i], fr["t"][i]), 4.0)
rgba = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda"); nrm = torch.zeros_like(rgba)
pose = tsdf_amd.SE3(fr["q"][N - 1], fr["t"][N - 1])
L = _lib.load()
n = 8 * 4096 * 8
buf = np.zeros(n, np.uint64)
for rep in range(3):
    e.raycast(K, W, H, pose, 4.0, rgba=rgba, normal=nrm)
    torch.cuda.synchronize()
    L.tsdf_debug_stamps(e._h, buf.ctypes.data, n, None)
d = buf.reshape(8, 4096, 8)[6]
nwg = ((W + 15) // 16) * ((H + 15) // 16)
d = d[:nwg].astype(np.int64)
t0 = d[:, 0].min()
dur = (d[:, 1] - d[:, 0]) / 100.0  # us
end = (d[:, 1] - t0) / 100.0
print("hit frac", float((rgba[..., 3] == 255).float().mean()))
print("wg duration us: mean %.1f p50 %.1f p90 %.1f max %.1f; last end %.1f; start spread %.1f" % (
    dur.mean(), np.median(dur), np.percentile(dur, 90), dur.max(), end.max(), (d[:, 0].max() - t0) / 100))
for name, col in (("batches", 2), ("jumps", 3), ("region steps", 4)):
    print(f"{name}/lane mean {d[:, col].mean() / 256:.1f}")
print("max batches of a lane (over wgs): mean %.1f max %d; max region steps mean %.1f max %d" % (
    d[:, 5].mean(), d[:, 5].max(), d[:, 6].mean(), d[:, 6].max()))
order = np.argsort(-dur)[:10]
tx = (W + 15) // 16
for w in order:
    print(f"wg {w} tile ({w % tx},{w // tx}) dur {dur[w]:.1f}us batches/lane {d[w,2]/256:.1f} maxb {d[w,5]} jumps/lane {d[w,3]/256:.1f} reg/lane {d[w,4]/256:.1f} maxreg {d[w,6]}")
e.close()
