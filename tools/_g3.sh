set -o pipefail
O=gpurun_out/r04_s3; mkdir -p $O
PPAMD_LIB=$PWD/carnd-path-planning-project_amd/ppamd/libppamd_var_trace.so timeout -k 10 120 python3 tools/trace_frame.py > $O/trace_frame.txt 2>&1 || { tail -20 $O/trace_frame.txt; exit 1; }
tail -1 $O/trace_frame.txt
bash tools/gpu_suite.sh r04_s3 || exit 1
timeout -k 10 200 python3 bench.py --scenes 262144 --no-cpu-baseline --no-pcie > $O/bench_shard.json 2>$O/shard.err || exit 1
python3 -c "import json;d=json.loads(open('$O/bench_shard.json').read().splitlines()[-1]);print('shard', round(d['ms_per_step'],4), d['kernels_ms_avg'], d['roofline']['launches_per_step'], round(d['roofline']['frac'],4))"
