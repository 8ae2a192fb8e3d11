"""Read-pattern ceilings for a fused month-end + scan kernel (dev tool, round 2): one-shot row
sweep vs whole-history walks (1..8 time segments) vs month-block chains.  Interleaves the
variants in one process and prints median GB/s.  Build: hipcc --offload-arch=gfx950 -O3
-fPIC -shared -o libmb2.so mb2.hip"""
import ctypes, json
from pathlib import Path
import numpy as np
import torch

lib = ctypes.CDLL(str(Path(__file__).with_name("libmb2.so")))
lib.mb2_launch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]
N, T_d = 100_000, 10_000
P = torch.rand(T_d, N, dtype=torch.float64, device="cuda")
out = torch.zeros(4, dtype=torch.float64, device="cuda")
lib.mb2_launch_w.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p,
                             ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
names = ["rows", "long_G1", "long_G2", "long_G4", "long_G8", "long_wpb4",
         "chain2_B2", "chain2_B4", "chain2_B8", "chain2_B16", "chain3_B3", "chain3_B6", "chain3_B12",
         "long_wpb4_G2", "long_wpb4_G4", "long_wpb2", "long_wpb2_G2", "long_wpb4_G3"]
T_m = (T_d + 20) // 21
nblk = ((N // 2 + 63) // 64 + 3) // 4
W1 = torch.empty(max(T_m * N, nblk * T_m * 512), dtype=torch.float64, device="cuda")
W2 = torch.empty_like(W1)
W3 = torch.empty(W1.numel() // 2 + 1, dtype=torch.int32, device="cuda")
names += ["long_wpb4_wrows", "long_wpb4_wlog"]
res = {n: [] for n in names}
st = torch.cuda.current_stream()
for rnd in range(8):
    for k, n in enumerate(names):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        if n.startswith("long_wpb4_w"):
            rc = lib.mb2_launch_w(1 if n.endswith("log") else 0, P.data_ptr(), T_d, N, out.data_ptr(),
                                  W1.data_ptr(), W2.data_ptr(), W3.data_ptr(), st.cuda_stream)
        else:
            rc = lib.mb2_launch(k, P.data_ptr(), T_d, N, out.data_ptr(), st.cuda_stream)
        e1.record()
        torch.cuda.synchronize()
        assert rc == 0, (n, rc)
        if rnd:
            res[n].append(8.0 * N * T_d / (e0.elapsed_time(e1) * 1e-3) / 1e9)
summary = {n: round(float(np.median(v)), 1) for n, v in res.items()}
spread = {n: round(float(np.max(v) - np.min(v)), 1) for n, v in res.items()}
print(json.dumps({"N": N, "T_d": T_d, "read_GBps_median": summary, "spread": spread}))
