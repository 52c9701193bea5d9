set -e
mkdir -p gpurun_out/t3
timeout -k 10 600 python -u -m pytest tests/test_gpu_construction.py tests/test_gpu_mixed.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/t3/gpu_constr.txt 2>&1 || true
timeout -k 10 300 python -u bench.py --task construction --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/t3/bench_construction.json 2> gpurun_out/t3/bench_construction.err
timeout -k 10 300 python -u bench.py --task mixed --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/t3/bench_mixed.json 2> gpurun_out/t3/bench_mixed.err
TASK=construction N=1024 K=3 timeout -k 10 300 python -u tools/stage_profile.py > gpurun_out/t3/stage_construction.txt 2>&1 || true
