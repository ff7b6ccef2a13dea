#!/bin/bash
# K1 launch-shape A/B at the 8-GPU shard size (262,144 scenes per GPU): lanes per scene
# (bench.py --debug prep_group=G) and waves per SIMD (--debug prep_waves=3|4); one bench line each, two passes.
mkdir -p gpurun_out/shard
run() { name=$1; shift
  timeout -k 10 200 python3 bench.py "$@" --no-cpu-baseline --no-pcie --steps 20 --scenes 262144 > gpurun_out/shard/$name.json 2>/dev/null || exit 1
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);print(sys.argv[2],'%.4g'%d['value'],round(d['ms_per_step'],3),{k:round(v,3) for k,v in d['kernels_ms_avg'].items() if v})" gpurun_out/shard/$name.json $name
}
for rep in 1 2; do
  run base
  run w3 --debug prep_waves=3
  run g2 --debug prep_group=2
  run g2_w3 --debug prep_group=2 --debug prep_waves=3
  run g4 --debug prep_group=4
done
