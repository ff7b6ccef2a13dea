#!/bin/bash
# A/B of pp_eval's split pipeline (PP_SPLIT=n chunks alternating over two streams, PP_SPLIT_STAGGER)
# on the GPU box: parity suite under the split, then bench lines (config 5 and a 262,144-scene shard).
mkdir -p gpurun_out/r02m
PP_SPLIT=2 PP_SPLIT_STAGGER=1 timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r02m/gpu_tests_split2s1.log 2>&1 || { tail -5 gpurun_out/r02m/gpu_tests_split2s1.log; exit 1; }
tail -1 gpurun_out/r02m/gpu_tests_split2s1.log
run() { # name scenes env...
  name=$1; sc=$2; shift 2
  env "$@" timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-pcie --steps 20 --scenes $sc > gpurun_out/r02m/$name.json 2>/dev/null || exit 1
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);print(sys.argv[2],'%.4g'%d['value'],round(d['ms_per_step'],3))" gpurun_out/r02m/$name.json "$name $sc"
}
for rep in 1 2; do
  run base 2097152 PP_SPLIT=0
  run split2 2097152 PP_SPLIT=2
  run split2_s1 2097152 PP_SPLIT=2 PP_SPLIT_STAGGER=1
  run split2_s2 2097152 PP_SPLIT=2 PP_SPLIT_STAGGER=2
  run split3_s1 2097152 PP_SPLIT=3 PP_SPLIT_STAGGER=1
  run base 262144 PP_SPLIT=0
  run split2 262144 PP_SPLIT=2
  run split2_s1 262144 PP_SPLIT=2 PP_SPLIT_STAGGER=1
done
