#!/bin/bash
# A/B of library debug switches (include/pp.h PP_DBG_*) on one box (GPU box, repo root):
#   ARGS="<bench args>" tools/dbg_ab.sh RUNS "KEY=VALUE[,KEY=VALUE]" ["..." ...]
# alternating runs of the default and each switch set; "-" is the default. Prints step and
# per-kernel ms of each bench line.
set -e -o pipefail
R=$1; shift
A=${ARGS:-}
for i in $(seq $R); do
  for set in - "$@"; do
    D=""
    if [ "$set" != - ]; then for kv in ${set//,/ }; do D="$D --debug $kv"; done; fi
    timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-pcie --steps 10 --warmup 3 $A $D > gpurun_out/dbg_ab.json 2>/dev/null
    python3 -c "
import json;d=json.loads(open('gpurun_out/dbg_ab.json').read().strip().splitlines()[-1])
print('%-16s'%'$set', 'step %.3f ms'%d['ms_per_step'], ' '.join('%s %.3f'%(k,v) for k,v in d['kernels_ms_avg'].items() if v))"
  done
done
