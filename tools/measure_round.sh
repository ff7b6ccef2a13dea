#!/bin/bash
# Full round measurement on the GPU box (repo root): GPU parity tests and smoke, PMC passes
# summarised into profiles/pmc_summary.json (configs 5, 3, 4 and 2), the default bench line (reads
# that summary for roofline.traffic / traffic_pipeline), the rocprofv3 kernel-trace stats of the
# same command, and the other BASELINE configurations. Outputs under gpurun_out/<tag>/.
# Every GPU step has its own time limit; the script stops at the first failure.
set -eo pipefail
TAG=${1:-r04}
OUT=gpurun_out/$TAG
ROOT=$(pwd)
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
bash tools/pmc.sh $OUT/pmc
python3 tools/pmc_summarize.py $OUT/pmc k_cand_S2097152_C15_N50 > $OUT/pmc_summary.txt
bash tools/pmc.sh $OUT/pmc3 --steps 2 --warmup 1 --no-cpu-baseline --no-pcie --emit-paths --n-speeds 8 --n-points 100 --scenes 262144
python3 tools/pmc_summarize.py $OUT/pmc3 k_cand_S262144_C24_N100_paths > $OUT/pmc3_summary.txt
bash tools/pmc.sh $OUT/pmc4 --steps 2 --warmup 1 --no-cpu-baseline --no-pcie --draws 64 --n-speeds 1 --scenes 16384
python3 tools/pmc_summarize.py $OUT/pmc4 k_cand_S16384_C192_N50_D64 > $OUT/pmc4_summary.txt
bash tools/pmc.sh $OUT/pmc2 --steps 20 --warmup 5 --no-cpu-baseline --no-pcie --scenes 4096
python3 tools/pmc_summarize.py $OUT/pmc2 k_cand_S4096_C15_N50 > $OUT/pmc2_summary.txt
cp profiles/pmc_summary.json $OUT/pmc_summary.json
timeout -k 10 400 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err
tail -1 $OUT/bench.json | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/stats -o run -- python3 $ROOT/bench.py --no-cpu-baseline --no-pcie > $OUT/bench_under_rocprof.json 2> $OUT/rocprof.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/stats3 -o run -- python3 $ROOT/bench.py --no-cpu-baseline --no-pcie --emit-paths --n-speeds 8 --n-points 100 --scenes 262144 > $OUT/bench3_under_rocprof.json 2> $OUT/rocprof3.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/stats_shard -o run -- python3 $ROOT/bench.py --no-cpu-baseline --no-pcie --scenes 262144 > $OUT/bench_shard_under_rocprof.json 2> $OUT/rocprof_shard.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/stats4 -o run -- python3 $ROOT/bench.py --no-cpu-baseline --draws 64 --n-speeds 1 --scenes 16384 > $OUT/bench4_under_rocprof.json 2> $OUT/rocprof4.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/stats2 -o run -- python3 $ROOT/bench.py --no-cpu-baseline --scenes 4096 --steps 300 --warmup 30 > $OUT/bench2_under_rocprof.json 2> $OUT/rocprof2.err
# the profiler's average K2 durations per launch shape (bench.py: roofline.frac_rocprof)
(python3 tools/rocprof_summarize.py $OUT/stats k_cand_S2097152_C15_N50 1 &&
 python3 tools/rocprof_summarize.py $OUT/stats3 k_cand_S262144_C24_N100_paths 1 &&
 python3 tools/rocprof_summarize.py $OUT/stats_shard k_cand_S262144_C15_N50 2 &&
 python3 tools/rocprof_summarize.py $OUT/stats4 k_cand_S16384_C192_N50_D64 1 &&
 python3 tools/rocprof_summarize.py $OUT/stats2 k_cand_S4096_C15_N50 1)
cp profiles/rocprof_summary.json $OUT/rocprof_summary.json
echo "rocprof done"
run() { name=$1; shift; timeout -k 10 300 python3 bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err; echo "$name: $(tail -1 $OUT/$name.json | cut -c1-200)"; }
run bench_config2 --scenes 4096 --steps 300 --warmup 30 --no-cpu-baseline
run bench_config3_allpaths --emit-paths --n-speeds 8 --n-points 100 --scenes 262144 --no-cpu-baseline
run bench_config4_montecarlo --draws 64 --n-speeds 1 --scenes 16384 --no-cpu-baseline
run bench_shard_262144 --scenes 262144 --no-cpu-baseline --no-pcie
run bench_rollout_2M_x10 --rollout 10 --no-cpu-baseline --no-pcie
run bench_rollout_64k_x100 --rollout 100 --scenes 65536 --no-cpu-baseline --no-pcie
