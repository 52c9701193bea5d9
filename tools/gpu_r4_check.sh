# Round-4 working check (run through gpurun from the repo root): staged / soccer / capacity /
# single-env / construction GPU tests, then the headline bench.
set -e
D=gpurun_out/${1:-r4b}
mkdir -p $D
timeout -k 10 900 python -u -m pytest tests/test_gpu_staged.py tests/test_gpu_soccer.py tests/test_gpu_capacity.py tests/test_gpu_single_env.py tests/test_gpu_construction.py -v -s --timeout 300 --timeout-method thread > $D/tests.txt 2>&1
timeout -k 10 300 python -u bench.py --steps 100 --no-cpu-baseline > $D/bench.json 2> $D/bench.err
timeout -k 10 300 python -u bench.py --steps 100 --no-cpu-baseline --full-capacity > $D/bench_full.json 2> $D/bench_full.err
