# soccer fp64 headline knobs at HEAD: reset banks per env, solver lanes per slot
set -e
D=gpurun_out/knobs
mkdir -p $D
for b in 2 3 4 5; do
  timeout -k 10 300 python -u bench.py --steps 100 --no-cpu-baseline --no-other-line --banks $b > $D/banks_$b.json 2> $D/banks_$b.err
  python -c "import json;d=json.load(open('$D/banks_$b.json'));print('banks $b',d['value'],d['ms_per_step'])"
done
MGX_PGS_LPS=64 timeout -k 10 300 python -u bench.py --steps 100 --no-cpu-baseline --no-other-line > $D/lps64.json 2> $D/lps64.err
python -c "import json;d=json.load(open('$D/lps64.json'));print('lps64',d['value'],d['ms_per_step'])"
