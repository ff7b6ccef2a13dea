#!/bin/bash
# FETCH_SIZE / WRITE_SIZE per kernel for the product library and variants (GPU box, repo root):
#   tools/fetch_ab.sh OUTDIR [NAME ...]   (NAME: libppamd_var_NAME.so; "base": the product library)
# One rocprofv3 --pmc pass per counter and library; per-kernel averages -> OUTDIR/summary.txt.
set -e
export TMPDIR=/tmp
ROOT=$(pwd)
OUT=$ROOT/$1; shift
mkdir -p $OUT
for v in "$@"; do
  if [ $v = base ]; then export PPAMD_LIB=$ROOT/carnd-path-planning-project_amd/ppamd/libppamd.so
  else export PPAMD_LIB=$ROOT/carnd-path-planning-project_amd/ppamd/libppamd_var_$v.so; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $OUT/$v/$c -o pmc -- python3 $ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > $OUT/$v.$c.log 2>&1
  done
  echo "$v done"
done
python3 - "$OUT" "$@" > $OUT/summary.txt <<'PY'
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
        if not k.startswith(("k_cand", "k_prep", "k_emit", "k_winner")):
            continue
        d = {c: sum(x) / len(x) for c, x in vals[k].items()}
        print(f"{v:10s} {k[:28]:28s} FETCH_KiB_raw {d.get('FETCH_SIZE', 0):14.1f} WRITE_KiB {d.get('WRITE_SIZE', 0):14.1f}")
PY
cat $OUT/summary.txt
