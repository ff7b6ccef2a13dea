#!/bin/bash
# Round-4 measurement on the GPU box (repo root), without the PMC passes (tools/pmc.sh): the GPU
# suite on the product and -DPP_CHECK builds with smoke (tools/gpu_suite.sh), the default bench
# line, rocprofv3 kernel-trace stats of the bench per BASELINE config (summarised into
# profiles/rocprof_summary.json for roofline.frac_rocprof, copied back with the outputs), every
# config's bench line, the shard step with the split on and off, and config 1's latency.
set -eo pipefail
TAG=${1:-r04}
OUT=gpurun_out/$TAG
ROOT=$(pwd)
mkdir -p $OUT
export TMPDIR=/tmp
[ "${2:-}" = "--no-suite" ] || bash tools/gpu_suite.sh $TAG/suite
rp() { name=$1; shift; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/$name -o run -- python3 $ROOT/bench.py --no-cpu-baseline --no-pcie "$@" > $OUT/$name.json 2> $OUT/$name.err; echo "rocprof $name done"; }
rp stats5
rp stats3 --emit-paths --n-speeds 8 --n-points 100 --scenes 262144
rp stats_shard --scenes 262144
rp stats_524288 --scenes 524288
rp stats_1048576 --scenes 1048576
rp stats4 --draws 64 --n-speeds 1 --scenes 16384
rp stats2 --scenes 4096 --steps 300 --warmup 30
python3 tools/rocprof_summarize.py $OUT/stats5 k_cand_S2097152_C15_N50 1
python3 tools/rocprof_summarize.py $OUT/stats3 k_cand_S262144_C24_N100_paths 1
python3 tools/rocprof_summarize.py $OUT/stats_shard k_cand_S262144_C15_N50 2
python3 tools/rocprof_summarize.py $OUT/stats_524288 k_cand_S524288_C15_N50 3
python3 tools/rocprof_summarize.py $OUT/stats_1048576 k_cand_S1048576_C15_N50 3
python3 tools/rocprof_summarize.py $OUT/stats4 k_cand_S16384_C192_N50_D64 1
python3 tools/rocprof_summarize.py $OUT/stats2 k_cand_S4096_C15_N50 1
cp profiles/rocprof_summary.json $OUT/rocprof_summary.json
run() { name=$1; shift; timeout -k 10 300 python3 bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err; echo "$name: $(tail -1 $OUT/$name.json | cut -c1-160)"; }
run bench
run bench_config2 --scenes 4096 --steps 300 --warmup 30 --no-cpu-baseline
run bench_config3_allpaths --emit-paths --n-speeds 8 --n-points 100 --scenes 262144 --no-cpu-baseline
run bench_config4_montecarlo --draws 64 --n-speeds 1 --scenes 16384 --no-cpu-baseline
run bench_shard_262144 --scenes 262144 --no-cpu-baseline --no-pcie
run bench_rollout_2M_x10 --rollout 10 --no-cpu-baseline --no-pcie
timeout -k 10 300 python3 tools/split_probe.py 262144 2 > $OUT/split_probe.txt 2>&1; tail -4 $OUT/split_probe.txt
timeout -k 10 300 python3 tools/split_probe.py 524288 2 > $OUT/split_probe_524288.txt 2>&1; tail -4 $OUT/split_probe_524288.txt
timeout -k 10 200 python3 tools/bench_frame.py --frames 2000 > $OUT/frame.json 2> $OUT/frame.err; cat $OUT/frame.json
L=$PWD/carnd-path-planning-project_amd/ppamd
PPAMD_LIB=$L/libppamd_var_fprof.so timeout -k 10 120 python3 tools/frame_prof.py > $OUT/frame_prof.json 2>&1; tail -1 $OUT/frame_prof.json
PPAMD_LIB=$L/libppamd_var_trace.so timeout -k 10 120 python3 tools/trace_frame.py > $OUT/trace_frame.json 2>&1; tail -1 $OUT/trace_frame.json
