set -e
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > gpurun_out/gpu_all.txt 2>&1 || true
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/bench_dpp.json 2> gpurun_out/bench_dpp.err
timeout -k 10 300 python -u bench.py --task mixed --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/bench_mixed.json 2> gpurun_out/bench_mixed.err
