set -e
D=gpurun_out/r4i
mkdir -p $D
timeout -k 10 600 python -u bench.py --task mixed --steps 20 --warmup 3 --no-cpu-baseline > $D/mixed_side1.json 2> $D/mixed_side1.err
MGX_SIDE_STREAM=0 timeout -k 10 600 python -u bench.py --task mixed --steps 20 --warmup 3 --no-cpu-baseline > $D/mixed_side0.json 2> $D/mixed_side0.err
MGX_SIDE_STREAM=0 timeout -k 10 400 python -u bench.py --task bipedal --steps 20 --warmup 3 --no-cpu-baseline --no-other-line > $D/bip_side0.json 2> $D/bip_side0.err
timeout -k 10 400 python -u bench.py --task bipedal --steps 20 --warmup 3 --no-cpu-baseline --no-other-line > $D/bip_side1.json 2> $D/bip_side1.err
timeout -k 10 300 python -u bench.py --steps 100 --no-cpu-baseline --no-other-line > $D/soccer.json 2> $D/soccer.err
