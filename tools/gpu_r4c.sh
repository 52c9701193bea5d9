set -e
mkdir -p gpurun_out/r4c
BENCH_ARGS="" bash tools/profile_round.sh r04_head > gpurun_out/r4c/prof_head.log 2>&1
BENCH_ARGS="--full-capacity" bash tools/profile_round.sh r04_full > gpurun_out/r4c/prof_full.log 2>&1
TASK=bipedal N=2048 K=3 timeout -k 10 300 python -u tools/stage_profile.py > gpurun_out/r4c/stage_bipedal.txt 2>&1
