#!/bin/bash
# Runs the CPU oracle tests against the ASan + UBSan build of oracle/mjref.c (host
# sanitizers). CPU only. Round 4 log: profiles/r04_oracle_asan.txt.
set -euo pipefail
cd "$(dirname "$0")/.."
make -s -C oracle asan
export MJREF_LIB=$PWD/oracle/_build/libmjref_asan.so
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
LD_PRELOAD="$(gcc -print-file-name=libasan.so):$(gcc -print-file-name=libubsan.so)" \
  python -m pytest tests/test_oracle_physics.py tests/test_oracle_narrowphase.py tests/test_oracle_soccer.py \
  tests/test_oracle_parkour.py tests/test_oracle_bipedal.py tests/test_oracle_dancing.py tests/test_oracle_martial.py \
  tests/test_oracle_assembly.py tests/test_oracle_construction.py tests/test_distributed_cpu.py -q -p no:cacheprovider "$@"
