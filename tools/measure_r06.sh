#!/bin/bash
# Round-6 measurement on the GPU box (repo root), in two calls on the final library build:
#   tools/measure_r06.sh A TAG   GPU suite on the product and -DPP_CHECK builds + smoke (gpu_suite.sh),
#                                rocprofv3 kernel-trace stats of the bench per launch shape, summarised
#                                into profiles/rocprof_summary.json (copied to gpurun_out/TAG/)
#   tools/measure_r06.sh B TAG   PMC passes (FETCH_SIZE, WRITE_SIZE, SQ, F64) per launch shape into
#                                profiles/pmc_summary.json, the SQ stall pass, then every bench line
#                                (they read both summaries; copy A's summary into profiles/ before B)
# Round 6: the split shards' counters are per-call (pmc_summarize's parts: 2 or 3 dispatches of each
# kernel per call); the comfort cost mode has its own tags (_comfort).
set -eo pipefail
PART=$1
TAG=${2:-r06}
OUT=gpurun_out/$TAG
ROOT=$(pwd)
mkdir -p $OUT
export TMPDIR=/tmp
NP="--no-cpu-baseline --no-pcie --no-shard-projection --no-comfort"
if [ "$PART" = A ]; then
  bash tools/gpu_suite.sh $TAG/suite
  rp() { name=$1; shift; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/$name -o run -- python3 $ROOT/bench.py $NP "$@" > $OUT/$name.json 2> $OUT/$name.err; echo "rocprof $name done"; }
  echo '{}' > profiles/rocprof_summary.json       # only this build's kernel traces
  rp stats5
  rp stats5_comfort --comfort
  rp stats3 --emit-paths --n-speeds 8 --n-points 100 --scenes 262144
  rp stats_shard --scenes 262144
  rp stats_524288 --scenes 524288
  rp stats_1048576 --scenes 1048576
  rp stats4 --draws 64 --n-speeds 1 --scenes 16384
  rp stats2 --scenes 4096 --steps 300 --warmup 30
  python3 tools/rocprof_summarize.py $OUT/stats5 k_cand_S2097152_C15_N50 1
  python3 tools/rocprof_summarize.py $OUT/stats5_comfort k_cand_S2097152_C15_N50_comfort 1
  python3 tools/rocprof_summarize.py $OUT/stats3 k_cand_S262144_C24_N100_paths 1
  python3 tools/rocprof_summarize.py $OUT/stats_shard k_cand_S262144_C15_N50 2
  python3 tools/rocprof_summarize.py $OUT/stats_524288 k_cand_S524288_C15_N50 3
  python3 tools/rocprof_summarize.py $OUT/stats_1048576 k_cand_S1048576_C15_N50 3
  python3 tools/rocprof_summarize.py $OUT/stats4 k_cand_S16384_C192_N50_D64 1
  python3 tools/rocprof_summarize.py $OUT/stats2 k_cand_S4096_C15_N50 1
  cp profiles/rocprof_summary.json $OUT/rocprof_summary.json
  for f in stats5 stats5_comfort stats3 stats_shard stats_524288 stats_1048576 stats4 stats2; do
    cp $(find $OUT/$f -name "*kernel_stats.csv" | head -1) $OUT/kernel_stats_$f.csv
  done
  exit 0
fi
# part B
echo '{}' > profiles/pmc_summary.json             # only this build's counters
pm() { name=$1; tag=$2; parts=$3; shift 3; bash tools/pmc.sh $OUT/$name --steps 2 --warmup 1 $NP "$@" > $OUT/$name.log 2>&1; python3 tools/pmc_summarize.py $OUT/$name $tag $parts > $OUT/${name}_summary.txt; echo "pmc $name done"; }
pm pmc5 k_cand_S2097152_C15_N50 1
pm pmc5_comfort k_cand_S2097152_C15_N50_comfort 1 --comfort
pm pmc3 k_cand_S262144_C24_N100_paths 1 --emit-paths --n-speeds 8 --n-points 100 --scenes 262144
pm pmc_shard k_cand_S262144_C15_N50 2 --scenes 262144
pm pmc4 k_cand_S16384_C192_N50_D64 1 --draws 64 --n-speeds 1 --scenes 16384
bash tools/pmc.sh $OUT/pmc2 --steps 20 --warmup 5 $NP --scenes 4096 > $OUT/pmc2.log 2>&1
python3 tools/pmc_summarize.py $OUT/pmc2 k_cand_S4096_C15_N50 > $OUT/pmc2_summary.txt
cp profiles/pmc_summary.json $OUT/pmc_summary.json
bash tools/pmc_stalls.sh $TAG
python3 tools/pmc_stalls_summary.py $TAG profiles/r06_pmc_stalls.json > $OUT/stalls_summary.txt
cp profiles/r06_pmc_stalls.json $OUT/
run() { name=$1; shift; timeout -k 10 400 python3 bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err; echo "$name: $(tail -1 $OUT/$name.json | cut -c1-220)"; }
run bench
run bench_config2 --scenes 4096 --steps 300 --warmup 30 --no-cpu-baseline
run bench_config3_allpaths --emit-paths --n-speeds 8 --n-points 100 --scenes 262144 --no-cpu-baseline
run bench_config4_montecarlo --draws 64 --n-speeds 1 --scenes 16384 --no-cpu-baseline
run bench_config5_comfort --comfort --no-cpu-baseline --no-pcie
run bench_shard_262144 --scenes 262144 --no-cpu-baseline --no-pcie
run bench_shard_524288 --scenes 524288 --no-cpu-baseline --no-pcie
run bench_shard_1048576 --scenes 1048576 --no-cpu-baseline --no-pcie
run bench_rollout_2M_x10 --rollout 10 --no-cpu-baseline --no-pcie
