# host / total time per frame of graph frames vs eager integrate (GPU box): python3 scripts/graph_timing.py
import sys, time, os
sys.path[:0]=['disinfect-slam_amd','tests']
import torch, tsdf_amd
from tsdf_amd import synth
cam=synth.camera(640,480,synth.TUM_FR1)
fr=synth.render_torch(cam,list(range(64)),device='cuda')
K=tsdf_amd.CameraIntrinsics(*[float(v) for v in cam.K])
eng=tsdf_amd.Engine(0.005,0.03,max_width=640,max_height=480,stream=torch.cuda.current_stream().cuda_stream)
g=eng.frame_graph(640,480)
poses=[tsdf_amd.SE3(fr['q'][i],fr['t'][i]) for i in range(64)]
for rep in range(3):
    torch.cuda.synchronize(); t=time.perf_counter()
    for i in range(64): g.frame(fr['rgb'][i],fr['depth'][i],fr['ht'][i],fr['lt'][i],K,poses[i],4.0)
    t1=time.perf_counter(); torch.cuda.synchronize(); t2=time.perf_counter()
    print(f"graph host {1e6*(t1-t)/64:.1f} us/frame, total {1e6*(t2-t)/64:.1f}")
    torch.cuda.synchronize(); t=time.perf_counter()
    for i in range(64): eng.integrate(fr['rgb'][i],fr['depth'][i],fr['ht'][i],fr['lt'][i],K,poses[i],4.0)
    t1=time.perf_counter(); torch.cuda.synchronize(); t2=time.perf_counter()
    print(f"eager host {1e6*(t1-t)/64:.1f} us/frame, total {1e6*(t2-t)/64:.1f}")
g.close(); eng.close()
