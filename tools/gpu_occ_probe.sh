set -e
for p in 0 40960 53248 81920; do
  MGX_ROWS_LDS=$p timeout -k 10 200 python -u bench.py --steps 40 --warmup 10 > gpurun_out/occ_$p.json 2> gpurun_out/occ_$p.err
  echo "pad=$p $(python -c "import json;d=json.load(open('gpurun_out/occ_$p.json'));print(d['value'],d['ms_per_step'])")"
done
