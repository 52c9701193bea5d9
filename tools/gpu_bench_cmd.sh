set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_capacity.py tests/test_gpu_staged.py tests/test_gpu_f32_staged.py tests/test_gpu_soccer.py tests/test_gpu_newton.py tests/test_gpu_martial.py tests/test_gpu_assembly.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gpu_t1.txt 2>&1 || true
timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 100 > gpurun_out/bench_t1.json 2> gpurun_out/bench_t1.err
timeout -k 10 300 python -u bench.py --task assembly --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_asm.json 2> gpurun_out/bench_asm.err
TASK=soccer N=4096 K=20 timeout -k 10 300 python -u tools/stage_profile.py > gpurun_out/stage_soccer_f64.txt 2>&1 || true
PREC=f32 TASK=soccer N=4096 K=20 timeout -k 10 300 python -u tools/stage_profile.py > gpurun_out/stage_soccer_f32.txt 2>&1 || true
TASK=assembly N=1024 K=4 timeout -k 10 300 python -u tools/stage_profile.py > gpurun_out/stage_assembly.txt 2>&1 || true
