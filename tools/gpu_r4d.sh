# solver main-launch LDS rows sweep (MGX_PGS_LDS_ROWS: rows per slot the main launch keeps in LDS;
# slots with more go to the side-stream wide launch)
set -e
D=gpurun_out/r4d
mkdir -p $D
for R in 192 160 128 104 80 64; do
  MGX_PGS_LDS_ROWS=$R timeout -k 10 300 python -u bench.py --steps 100 --no-cpu-baseline --no-other-line > $D/bench_$R.json 2> $D/bench_$R.err
done
for R in 192 104; do
  MGX_PGS_LDS_ROWS=$R timeout -k 10 300 python -u bench.py --steps 100 --no-cpu-baseline --no-other-line --full-capacity > $D/bench_full_$R.json 2> $D/bench_full_$R.err
done
TASK=soccer N=4096 K=10 timeout -k 10 300 python -u tools/stage_profile.py > $D/stage_soccer.txt 2>&1 || true
