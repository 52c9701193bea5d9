# bipedal fp64 8192 envs: the RK4 main solver launch's LDS rows per slot (MGX_RK_LDS_ROWS)
set -e
D=gpurun_out/bipknobs
mkdir -p $D
for r in 160 192 256 320; do
  MGX_RK_LDS_ROWS=$r timeout -k 10 300 python -u bench.py --task bipedal --steps 20 --warmup 3 --no-cpu-baseline --no-other-line > $D/rows_$r.json 2> $D/rows_$r.err
  python -c "import json;d=json.load(open('$D/rows_$r.json'));print('rows $r',d['value'],d['ms_per_step'])"
done
