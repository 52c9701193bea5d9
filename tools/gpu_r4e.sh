# staged RK4 bipedal: tests, then configs[3] bench (fp64 staged, fp32 line), then the soccer
# staged regression tests and the pending solver LDS-rows sweep
set -e
D=gpurun_out/r4e
mkdir -p $D
timeout -k 10 900 python -u -m pytest tests/test_gpu_bipedal.py -v -s --timeout 600 --timeout-method thread -x > $D/bip_tests.txt 2>&1
timeout -k 10 400 python -u bench.py --task bipedal --steps 20 --warmup 3 --no-cpu-baseline > $D/bench_bip.json 2> $D/bench_bip.err
timeout -k 10 600 python -u -m pytest tests/test_gpu_staged.py tests/test_gpu_capacity.py tests/test_gpu_soccer.py -v --timeout 300 --timeout-method thread -x > $D/soccer_tests.txt 2>&1
bash tools/gpu_r4d.sh
