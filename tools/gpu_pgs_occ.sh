# PGS main-launch occupancy sweep (MGX_PGS_LDS_PAD), soccer fp64 headline config
set -e
D=gpurun_out/pgs_occ
mkdir -p $D
for p in 0 23000 27000 32000 40000 54000; do
  MGX_PGS_LDS_PAD=$p timeout -k 10 200 python -u bench.py --steps 60 --warmup 10 --no-cpu-baseline --no-other-line > $D/occ_$p.json 2> $D/occ_$p.err
  echo "pad=$p $(python -c "import json;d=json.load(open('$D/occ_$p.json'));print(d['value'],d['ms_per_step'])")"
done
