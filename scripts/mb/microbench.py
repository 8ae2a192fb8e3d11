"""Read-bandwidth ceilings for the engine's access patterns (dev tool).  Interleaves the
variants in one process (MI355X methodology rule 24) and prints median GB/s."""
import ctypes, json, sys
from pathlib import Path
import numpy as np
import torch

lib = ctypes.CDLL(str(Path(__file__).with_name("libmb.so")))
lib.mb_launch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]
N, T_d = 102_400, 10_000  # N % 128 == 0: the tiled kernels address [N/128][T_d][128]
P = torch.rand(T_d, N, dtype=torch.float64, device="cuda")
out = torch.zeros(4, dtype=torch.float64, device="cuda")
names = ["stream_u8", "stream_u16", "rows_d8", "rows_d22", "tiled_d8", "tiled_d22", "long_d22",
         "long_d22_tiled", "long_d32", "long_d12"]
res = {n: [] for n in names}
st = torch.cuda.current_stream()
for rnd in range(6):
    for k, n in enumerate(names):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        rc = lib.mb_launch(k, P.data_ptr(), T_d, N, out.data_ptr(), st.cuda_stream)
        e1.record()
        torch.cuda.synchronize()
        assert rc == 0, (n, rc)
        if rnd:
            res[n].append(8.0 * N * T_d / (e0.elapsed_time(e1) * 1e-3) / 1e9)
summary = {n: round(float(np.median(v)), 1) for n, v in res.items()}
print(json.dumps({"N": N, "T_d": T_d, "read_GBps_median": summary}))
