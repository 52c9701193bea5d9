#!/bin/bash
# Profiling evidence for one round (run ON the GPU box from the repo root):
#   1) rocprofv3 --kernel-trace --stats on the bench command itself (its JSON line is kept),
#   2) separate --pmc passes for FETCH_SIZE and WRITE_SIZE (MI355X_MICROARCH.md §HBM:
#      they cannot share a pass; counters only, no trace domains),
#   3) tools/summarize_profile.py -> gpurun_out/prof_<tag>/summary/ (copied into profiles/).
set -eo pipefail
TAG=${1:-r01}
STEPS=${STEPS:-100}
BENCH_ARGS=${BENCH_ARGS:-}   # e.g. "--task bipedal"
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
  python3 "$R/bench.py" --steps "$STEPS" --warmup 10 --no-cpu-baseline --no-f64-line $BENCH_ARGS > "$OUT/bench_under_rocprof.json"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- \
  python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-f64-line $BENCH_ARGS > "$OUT/bench_pmc_fetch.json"
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- \
  python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-f64-line $BENCH_ARGS > "$OUT/bench_pmc_write.json"
python3 "$R/tools/summarize_profile.py" "$OUT" "$TAG"
