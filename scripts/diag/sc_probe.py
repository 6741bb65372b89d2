import ctypes as C, sys, os
sys.path.insert(0, "disinfect-slam_amd")
mode = sys.argv[1]
import torch
torch.zeros(1, device="cuda")
if mode == "engine_first":
    import tsdf_amd
    tsdf_amd._lib.load()
L = C.CDLL("disinfect-slam_amd/libtsdf_selfcheck.so")
L.tsdf_selfcheck_convert.argtypes = [C.c_uint32, C.c_uint32, C.POINTER(C.c_ulonglong), C.POINTER(C.c_uint32)]
b = C.c_ulonglong(); f = C.c_uint32()
print(mode, "rc", L.tsdf_selfcheck_convert(0, 1000, C.byref(b), C.byref(f)), flush=True)
maps = open("/proc/self/maps").read()
print(sorted(set(l.split()[-1] for l in maps.splitlines() if "amdhip" in l or "hsa-runtime" in l)))
