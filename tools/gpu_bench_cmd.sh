set -e
timeout -k 10 600 python -u -m pytest tests/test_gpu_capacity.py tests/test_gpu_soccer.py tests/test_gpu_staged.py -v --timeout 300 --timeout-method thread > gpurun_out/t_cap.txt 2>&1
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/bench_cap.json 2> gpurun_out/bench_cap.err
timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-other-line --full-capacity > gpurun_out/bench_fullcap.json 2> gpurun_out/bench_fullcap.err
