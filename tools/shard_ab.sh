#!/bin/bash
# K1 launch-shape A/B at the 8-GPU shard size (262,144 scenes per GPU): lanes per scene
# (PP_PREP_G) and waves per SIMD (PP_PREP_W4); one bench line each, two passes.
mkdir -p gpurun_out/shard
run() { name=$1; shift
  env "$@" timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-pcie --steps 20 --scenes 262144 > gpurun_out/shard/$name.json 2>/dev/null || exit 1
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);print(sys.argv[2],'%.4g'%d['value'],round(d['ms_per_step'],3),{k:round(v,3) for k,v in d['kernels_ms_avg'].items() if v})" gpurun_out/shard/$name.json $name
}
for rep in 1 2; do
  run base
  run w4_off PP_PREP_W4=0
  run g2 PP_PREP_G=2
  run g2_w4off PP_PREP_G=2 PP_PREP_W4=0
  run g4 PP_PREP_G=4
done
