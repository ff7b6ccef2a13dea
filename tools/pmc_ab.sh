#!/bin/bash
# PMC A/B on the GPU box (repo root): SQ counters per kernel for the product library and the given
# variants (libppamd_var_NAME.so): tools/pmc_ab.sh [NAME ...]. One rocprofv3 --pmc pass per library
# (8 SQ counters); the summary per kernel and library goes to gpurun_out/pmcab/summary.txt.
set -e
export TMPDIR=/tmp
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/pmcab
rm -rf $OUT; mkdir -p $OUT
for v in base "$@"; do
  if [ $v = base ]; then export PPAMD_LIB=$ROOT/carnd-path-planning-project_amd/ppamd/libppamd.so
  else export PPAMD_LIB=$ROOT/carnd-path-planning-project_amd/ppamd/libppamd_var_$v.so; fi
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_LDS --output-format csv -d $OUT/$v -o sq -- python3 $ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/$v.log 2>&1
  echo "$v done"
done
python3 - "$OUT" base "$@" > $OUT/summary.txt <<'PY'
import csv, glob, os, sys
from collections import defaultdict
out = sys.argv[1]
for v in sys.argv[2:]:
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(out, v, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            k = row.get("Kernel_Name", "").split("(")[0].replace("void ", "").strip()
            vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k in sorted(vals):
        if not k.startswith(("k_cand", "k_prep", "k_emit")):
            continue
        d = {c: sum(x) / len(x) for c, x in vals[k].items()}
        w = d.get("SQ_WAVES", 1) or 1
        util = d.get("SQ_THREAD_CYCLES_VALU", 0) / max(64 * d.get("SQ_ACTIVE_INST_VALU", 1), 1)
        print(f"{v:10s} {k[:28]:28s} waves {w:10.0f} valu/wave {d.get('SQ_INSTS_VALU', 0) / w:9.1f} "
              f"salu/wave {d.get('SQ_INSTS_SALU', 0) / w:8.1f} lds/wave {d.get('SQ_INSTS_LDS', 0) / w:7.1f} "
              f"valu_total {d.get('SQ_INSTS_VALU', 0):.4g} lane_util {util:.3f}")
PY
cat $OUT/summary.txt
