set -e
D=gpurun_out/fullcap
mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_capacity.py > $D/tests.txt 2>&1
tail -1 $D/tests.txt
timeout -k 10 300 python -u bench.py --steps 100 --no-cpu-baseline --no-other-line --full-capacity > $D/full.json 2> $D/full.err
timeout -k 10 300 python -u bench.py --steps 100 --no-cpu-baseline --no-other-line > $D/default.json 2> $D/default.err
timeout -k 10 300 python -u bench.py --task bipedal --steps 20 --warmup 3 --no-cpu-baseline --no-other-line > $D/bip.json 2> $D/bip.err
for f in full default bip; do python -c "import json;d=json.load(open('$D/$f.json'));print('$f',d['value'],d['ms_per_step'])"; done
timeout -k 10 600 python -u bench.py --task mixed --steps 20 --warmup 3 --no-cpu-baseline > $D/mix4.json 2> $D/mix4.err
timeout -k 10 600 python -u bench.py --task mixed --steps 20 --warmup 3 --no-cpu-baseline --mix-priority > $D/mix4p.json 2> $D/mix4p.err
timeout -k 10 600 python -u bench.py --task mixed --steps 20 --warmup 3 --no-cpu-baseline --mix-streams 7 > $D/mix7.json 2> $D/mix7.err
for f in mix4 mix4p mix7; do python -c "import json;d=json.load(open('$D/$f.json'));print('$f',d['value'],d['ms_per_step'],d['config']['task_launch_ms'])"; done
