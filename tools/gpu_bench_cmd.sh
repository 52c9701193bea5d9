set -e
timeout -k 10 300 python -u bench.py --task construction --steps 10 --warmup 2 > gpurun_out/bench_con.json 2> gpurun_out/bench_con.err
TASK=construction N=1024 K=3 timeout -k 10 150 python -u tools/stage_profile.py > gpurun_out/sp_con.txt 2>&1
