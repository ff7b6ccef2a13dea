#!/bin/bash
# On the GPU box: times every libppamd_var_*.so (and the product library) with bench.py, one
# process after another; one summary line per library into gpurun_out/variants.txt.
cd "$(dirname "$0")/.." || exit 1
shopt -s nullglob
mkdir -p gpurun_out
out=gpurun_out/variants.txt
: > $out
for lib in carnd-path-planning-project_amd/ppamd/libppamd.so carnd-path-planning-project_amd/ppamd/libppamd_var_*.so; do
  PPAMD_LIB=$PWD/$lib timeout -k 10 240 python bench.py --no-cpu-baseline "$@" > gpurun_out/vb.log 2>&1 || { echo "$lib FAILED" >> $out; tail -5 gpurun_out/vb.log >> $out; exit 1; }
  python - "$lib" >> $out <<'PY'
import json, sys
line = [l for l in open("gpurun_out/vb.log") if l.startswith("{")][-1]
j = json.loads(line)
print(sys.argv[1].split("/")[-1], "%.4g" % j["value"], j["ms_per_step"], {k: (round(v, 3) if v is not None else None) for k, v in j["kernels_ms_avg"].items()})
PY
done
cat $out
