# End-of-round GPU evidence (run through gpurun from the repo root): full GPU suite, smoke,
# headline bench with the CPU baseline, the mixed configs[4] bench.
set -e
mkdir -p gpurun_out/final
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/final/gpu_all.txt 2>&1 || true
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.txt 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err
timeout -k 10 300 python -u bench.py --task mixed --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/final/bench_mixed.json 2> gpurun_out/final/bench_mixed.err
