# staged row-builder layout by liveness: LDS sizes, staged parity tests, soccer + bipedal bench
set -e
D=gpurun_out/r4l
mkdir -p $D
timeout -k 10 120 python -u tools/lds_info.py soccer f64 > $D/lds.txt 2>&1
timeout -k 10 120 python -u tools/lds_info.py soccer_full f64 >> $D/lds.txt 2>&1
timeout -k 10 120 python -u tools/lds_info.py bipedal f64 >> $D/lds.txt 2>&1
cat $D/lds.txt
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_staged.py tests/test_gpu_soccer.py > $D/tests_soccer.txt 2>&1
tail -3 $D/tests_soccer.txt
timeout -k 10 300 python -u bench.py --steps 100 --no-cpu-baseline --no-other-line > $D/soccer.json 2> $D/soccer.err
cat $D/soccer.json
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bipedal.py > $D/tests_bipedal.txt 2>&1
tail -3 $D/tests_bipedal.txt
timeout -k 10 400 python -u bench.py --task bipedal --steps 20 --warmup 3 --no-cpu-baseline --no-other-line > $D/bip.json 2> $D/bip.err
cat $D/bip.json
[ -n "$SP" ] && TASK=soccer N=4096 K=10 timeout -k 10 300 python -u tools/stage_profile.py > $D/sp_soccer.txt 2>&1
[ -n "$SP" ] && cat $D/sp_soccer.txt || true
