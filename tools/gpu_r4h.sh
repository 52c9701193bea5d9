set -e
mkdir -p gpurun_out/r4h
STEPS=20 BENCH_ARGS="--task bipedal" bash tools/profile_round.sh r04_bipedal > gpurun_out/r4h/prof_bip.log 2>&1
timeout -k 10 600 python -u bench.py --task mixed --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r4h/bench_mixed.json 2> gpurun_out/r4h/bench_mixed.err
