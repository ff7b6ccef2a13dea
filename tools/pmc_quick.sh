#!/bin/bash
# One SQ counter pass of a bench configuration per library (GPU box, repo root):
#   ARGS="<bench args>" tools/pmc_quick.sh TAG [VARIANT ...]  -> per-kernel counters per wave
set -e -o pipefail
export TMPDIR=/tmp
T=$1; shift
for lib in default "$@"; do
  if [ $lib = default ]; then unset PPAMD_LIB; else export PPAMD_LIB=$PWD/carnd-path-planning-project_amd/ppamd/libppamd_var_$lib.so; fi
  timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmcq_${T}_$lib -o q -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-pcie ${ARGS:-} > gpurun_out/pmcq_${T}_$lib.log 2>&1
  f=$(find gpurun_out/pmcq_${T}_$lib -name "*counter_collection.csv" | head -1)
  python3 - "$f" "$lib" <<'PY'
import csv, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float)); d = collections.defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    k = r['Kernel_Name'].split('(')[0][:26]
    if not k.startswith(('void k_', 'k_')): continue
    agg[k][r['Counter_Name']] += float(r['Counter_Value']); d[k].add(r['Dispatch_Id'])
for k, v in agg.items():
    w = v['SQ_WAVES'] or 1
    util = v['SQ_THREAD_CYCLES_VALU'] / max(v['SQ_ACTIVE_INST_VALU'] * 64, 1)
    print(f"{sys.argv[2]:8s} {k:26s} waves/launch {w/len(d[k]):9.0f} VALU/wave {v['SQ_INSTS_VALU']/w:8.0f} LDS/wave {v['SQ_INSTS_LDS']/w:6.0f} SALU/wave {v['SQ_INSTS_SALU']/w:6.0f} util {util:.3f}")
PY
done
