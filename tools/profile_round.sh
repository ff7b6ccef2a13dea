#!/bin/bash
# Round measurement on the GPU box: bench (with CPU baseline), rocprofv3 kernel-trace stats of the
# same command, and the PMC counter passes. Outputs under gpurun_out/<tag>/.
set -e
TAG=${1:-r01}
OUT=gpurun_out/$TAG
ROOT=$(pwd)
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err
echo "bench rc=$?"; tail -1 $OUT/bench.json | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/stats -o run -- python3 $ROOT/bench.py --no-cpu-baseline > $OUT/bench_under_rocprof.json 2> $OUT/rocprof.err
echo "rocprof rc=$?"
bash tools/pmc.sh $OUT/pmc
