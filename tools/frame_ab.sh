#!/bin/bash
# A/B of pp_plan_frame latency (tools/bench_frame.py) between the default library and variants
# (GPU box, repo root): tools/frame_ab.sh RUNS VARIANT [VARIANT ...]; alternating runs.
set -e -o pipefail
R=$1; shift
for i in $(seq $R); do
  for lib in default "$@"; do
    if [ $lib = default ]; then unset PPAMD_LIB; else export PPAMD_LIB=$PWD/carnd-path-planning-project_amd/ppamd/libppamd_var_$lib.so; fi
    timeout -k 10 120 python3 tools/bench_frame.py --frames 1000 > gpurun_out/frame_ab_$lib.json 2>/dev/null
    python3 -c "
import json;d=json.loads(open('gpurun_out/frame_ab_$lib.json').read().strip().splitlines()[-1])
print('%-8s'%'$lib', 'frame median %.1f us p10 %.1f p90 %.1f'%(d['gpu_median_us'],d['gpu_p10_us'],d['gpu_p90_us']), 'same_plan', d.get('same_plan'))"
  done
done
