#!/bin/bash
# A/B of bench lines between the default library and variants (GPU box, repo root):
#   ARGS="<bench args>" tools/ab.sh RUNS VARIANT [VARIANT ...]
# alternating runs; prints step and per-kernel ms (variants: libppamd_var_<name>.so)
set -e -o pipefail
R=$1; shift
A=${ARGS:-}
for i in $(seq $R); do
  for lib in default "$@"; do
    if [ $lib = default ]; then unset PPAMD_LIB; else export PPAMD_LIB=$PWD/carnd-path-planning-project_amd/ppamd/libppamd_var_$lib.so; fi
    timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-pcie --steps 10 --warmup 3 $A > gpurun_out/ab_$lib.json 2>/dev/null
    python3 -c "
import json;d=json.loads(open('gpurun_out/ab_$lib.json').read().strip().splitlines()[-1])
print('%-8s'%'$lib', 'step %.3f ms'%d['ms_per_step'], ' '.join('%s %.3f'%(k,v) for k,v in d['kernels_ms_avg'].items() if v), 'frac %.4f'%d['roofline']['frac'])"
  done
done
