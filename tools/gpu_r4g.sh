set -e
D=gpurun_out/r4g
mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_bipedal.py -v -s --timeout 300 --timeout-method thread -k "distribution or end_to_end" > $D/bip_tests.txt 2>&1
timeout -k 10 400 python -u bench.py --task bipedal --steps 20 --warmup 3 --no-cpu-baseline > $D/bench_bip.json 2> $D/bench_bip.err
timeout -k 10 400 python -u bench.py --task bipedal --steps 10 --warmup 2 --no-cpu-baseline --mono --no-other-line > $D/bench_bip_mono.json 2> $D/bench_bip_mono.err
timeout -k 10 600 python -u -m pytest tests/test_gpu_staged.py tests/test_gpu_capacity.py tests/test_gpu_soccer.py -q --timeout 300 --timeout-method thread -x > $D/soccer_tests.txt 2>&1
bash tools/gpu_r4d.sh
