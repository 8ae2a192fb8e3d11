set -e
mkdir -p gpurun_out/c5k
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --dump gpurun_out/c5k/new.npz > gpurun_out/c5k/new_$i.json 2> gpurun_out/c5k/new_$i.err
  CSMOM_LIB=ab/libcsmom_base.so timeout -k 10 200 python -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --dump gpurun_out/c5k/base.npz > gpurun_out/c5k/base_$i.json 2> gpurun_out/c5k/base_$i.err
done
python -c "
import numpy as np
a=np.load('gpurun_out/c5k/new.npz'); b=np.load('gpurun_out/c5k/base.npz')
for k in a.files:
    x,y=a[k],b[k]
    print(k, x.shape, 'bits equal:', np.array_equal(x.view(np.uint8), y.view(np.uint8)))
"
