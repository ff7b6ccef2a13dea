#!/bin/bash
# Full round measurement on the GPU box (repo root): GPU parity tests, PMC passes summarised into
# profiles/pmc_summary.json, then the default bench line (reads that summary for roofline.traffic)
# and the rocprofv3 kernel-trace stats of the same command. Outputs under gpurun_out/<tag>/.
set -e
TAG=${1:-r01}
OUT=gpurun_out/$TAG
ROOT=$(pwd)
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
tail -2 $OUT/gpu_tests.log
bash tools/pmc.sh $OUT/pmc
python3 tools/pmc_summarize.py $OUT/pmc k_cand_S2097152_C15_N50 > $OUT/pmc_summary.txt
cp profiles/pmc_summary.json $OUT/pmc_summary.json
timeout -k 10 400 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err
tail -1 $OUT/bench.json | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/stats -o run -- python3 $ROOT/bench.py --no-cpu-baseline > $OUT/bench_under_rocprof.json 2> $OUT/rocprof.err
echo "rocprof done"
