#!/bin/bash
# SQ stall profile of the bench's step kernels (one --pmc pass, counters only).
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/sq_${1:-x}
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS \
  -d "$OUT" -o run --output-format csv -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-f64-line "${@:2}" > "$OUT/bench.json"
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.defaultdict(set)
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"]
    for key in ("k_soccer_rows", "k_pgs_groups", "k_soccer_finish", "k_soccer_fixup", "k_soccer<float, 0>"):
        if key in k:
            acc[key][r["Counter_Name"]] += float(r["Counter_Value"]); n[key].add(r.get("Dispatch_Id"))
for k, v in acc.items():
    d = len(n[k]); wc = v["SQ_WAVE_CYCLES"]
    print(f"{k:20s} dispatches {d} waves/disp {v['SQ_WAVES']/d:.0f} wave_cycles/disp {wc/d:.3g} "
          f"wait_any {v['SQ_WAIT_ANY']/wc:.2f} wait_inst {v['SQ_WAIT_INST_ANY']/wc:.2f} active {v['SQ_ACTIVE_INST_ANY']/wc:.2f} "
          f"active_valu {v['SQ_ACTIVE_INST_VALU']/wc:.2f} valu_insts/disp {v['SQ_INSTS_VALU']/d:.3g} lds_insts/disp {v['SQ_INSTS_LDS']/d:.3g}")
PY
