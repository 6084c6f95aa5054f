set -e
mkdir -p gpurun_out/occ
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu > gpurun_out/occ/tests.log 2>&1
for r in 1 2; do
TTMPC_LIB=$PWD/car-trailer-mpc_amd/ttmpc/variants/libttmpc_base.so timeout -k 10 120 python bench.py --config c5 --steps 10 --warmup 2 --cpu-budget 0 --no-latency > gpurun_out/occ/base_c5_$r.json
timeout -k 10 120 python bench.py --config c5 --steps 10 --warmup 2 --cpu-budget 0 --no-latency > gpurun_out/occ/new_c5_$r.json
done
timeout -k 10 120 python bench.py --steps 20 --warmup 3 --cpu-budget 0 --no-latency > gpurun_out/occ/new_c2.json
