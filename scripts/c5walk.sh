# C5: general turnover rows walking live ages only (the in-tree build) vs ab/libcsmom_base.so (every age), bench ms/step + the C5 table bit for bit
set -e
mkdir -p gpurun_out/c5w
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --dump gpurun_out/c5w/new.npz > gpurun_out/c5w/new_$i.json 2> gpurun_out/c5w/new_$i.err
  CSMOM_LIB=ab/libcsmom_base.so timeout -k 10 200 python -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --dump gpurun_out/c5w/base.npz > gpurun_out/c5w/base_$i.json 2> gpurun_out/c5w/base_$i.err
done
python -c "
import numpy as np
a=np.load('gpurun_out/c5w/new.npz'); b=np.load('gpurun_out/c5w/base.npz')
for k in a.files:
    x,y=a[k],b[k]
    print(k, x.shape, 'bits equal:', np.array_equal(x.view(np.uint8), y.view(np.uint8)))
"
timeout -k 10 600 python -u -m pytest tests/test_gpu_portfolio.py tests/test_gpu_boot_scan.py -x -q --timeout 300 --timeout-method thread > gpurun_out/c5w/tests.log 2>&1
