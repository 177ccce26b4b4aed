#!/bin/bash
# Round 5: entropy statistics -- GPU tests, batch / per-frame timing, rocprofv3 --stats and two
# PMC passes of the batch bench (k_ent_ac).  Usage: bash tools/gpu_r6am.sh OUT
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT="$ROOT/gpurun_out/$1"; mkdir -p "$OUT"
bash tools/gpu_r6ak.sh "$1" || exit $?
cd /tmp
export EB_MODE=batch
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT --output-format csv -d "$OUT/p1" -o run -- python3 "$ROOT/tools/entropy_bench.py" > "$OUT/p1.log" 2>&1 || { tail -5 "$OUT/p1.log"; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU --output-format csv -d "$OUT/p2" -o run -- python3 "$ROOT/tools/entropy_bench.py" > "$OUT/p2.log" 2>&1 || { tail -5 "$OUT/p2.log"; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/p3" -o run -- python3 "$ROOT/tools/entropy_bench.py" > "$OUT/p3.log" 2>&1 || { tail -5 "$OUT/p3.log"; exit 1; }
cd "$ROOT" && python3 - "$OUT" <<'P'
import collections, csv, glob, sys
d = sys.argv[1]
for k in ("k_ent_ac", "k_ent_dc", "k_ent_hist"):
    per = collections.defaultdict(list)
    for f in sorted(glob.glob(f"{d}/p*/**/*counter_collection.csv", recursive=True)):
        agg = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            if k in r["Kernel_Name"]:
                agg[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (_, c), v in agg.items():
            per[c].append(v)
    print(k, {c: round(sorted(v)[len(v) // 2]) for c, v in sorted(per.items())})
P
