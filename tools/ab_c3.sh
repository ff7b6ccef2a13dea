#!/bin/bash
# A/B of config 3 (all paths) between the default library and a variant (GPU box, repo root):
#   tools/ab_c3.sh <variant> [runs]   -> alternating bench lines, k_cand ms from the roofline
set -e -o pipefail
V=$1; R=${2:-2}; V2=${3:-}; V3=${4:-}
C3="--emit-paths --n-speeds 8 --n-points 100 --scenes 262144 --no-cpu-baseline --no-pcie --steps 10 --warmup 3"
for i in $(seq $R); do
  for lib in default $V $V2 $V3; do
    if [ $lib = default ]; then unset PPAMD_LIB; else export PPAMD_LIB=$PWD/carnd-path-planning-project_amd/ppamd/libppamd_var_$lib.so; fi
    timeout -k 10 120 python3 bench.py $C3 > gpurun_out/ab_$lib.json 2>/dev/null
    python3 -c "
import json;d=json.loads(open('gpurun_out/ab_$lib.json').read().strip().splitlines()[-1])
r=d['roofline'];print('$lib', 'step %.3f ms'%d['ms_per_step'], 'kcand %.3f ms'%d['kernels_ms_avg']['k_cand'], 'frac %.4f'%r['frac'])"
  done
done
