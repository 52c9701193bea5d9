# End-of-round GPU evidence (run through gpurun from the repo root): full GPU suite, smoke,
# headline bench with the CPU baseline, the full-capacity line and the mixed configs[4] bench.
# Test failures (pytest exit 1) are recorded and the evidence run continues; anything else
# (a fault, an abort, a time limit) ends it.
set -e
D=gpurun_out/${1:-final}
mkdir -p $D
rc=0
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $D/gpu_all.txt 2>&1 || rc=$?
tail -3 $D/gpu_all.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "GPU suite ended with $rc"; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.txt 2>&1
timeout -k 10 300 python -u bench.py > $D/bench.json 2> $D/bench.err
cat $D/bench.json
timeout -k 10 300 python -u bench.py --steps 100 --no-cpu-baseline --no-other-line --full-capacity > $D/bench_full.json 2> $D/bench_full.err
timeout -k 10 600 python -u bench.py --task mixed --steps 20 --warmup 3 --no-cpu-baseline > $D/bench_mixed.json 2> $D/bench_mixed.err
cat $D/bench_mixed.json
