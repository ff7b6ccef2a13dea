#!/bin/bash
# Every bench line under profiles/ for one round (GPU box, repo root): tools/bench_configs.sh TAG
# -> gpurun_out/TAG/*.json. Each run under its own time limit; stops at the first failure.
set -e
T=${1:-r01}
O=gpurun_out/$T
mkdir -p $O
run() { name=$1; shift; timeout -k 10 300 python3 bench.py "$@" > $O/$name.json 2> $O/$name.err; echo "$name: $(tail -1 $O/$name.json | cut -c1-160)"; }
run bench
run bench_config2 --scenes 4096 --no-cpu-baseline
run bench_config3_allpaths --emit-paths --n-speeds 8 --n-points 100 --scenes 262144 --no-cpu-baseline
run bench_config4_montecarlo --draws 64 --n-speeds 1 --scenes 16384 --no-cpu-baseline
run bench_config4_montecarlo_comfort --draws 64 --n-speeds 1 --scenes 16384 --comfort --no-cpu-baseline
run bench_rollout_2M_x10 --rollout 10 --no-cpu-baseline
run bench_rollout_64k_x100 --rollout 100 --scenes 65536 --no-cpu-baseline
run bench_rollout_1_x100 --rollout 100 --scenes 1 --no-cpu-baseline
