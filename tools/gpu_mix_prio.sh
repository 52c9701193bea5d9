set -e
D=gpurun_out/mixprio
mkdir -p $D
for v in 0 0,1 1 0 0,1; do
  MGX_MIX_PRIO_GROUPS=$v timeout -k 10 600 python -u bench.py --task mixed --steps 20 --warmup 3 --no-cpu-baseline > $D/mix_$v.json 2> $D/mix_$v.err
  python -c "import json;d=json.load(open('$D/mix_$v.json'));print('prio $v',d['value'],d['ms_per_step'])"
done
