set -o pipefail
O=gpurun_out/r04_s6; mkdir -p $O
PPAMD_LIB=$PWD/carnd-path-planning-project_amd/ppamd/libppamd_var_fprof.so timeout -k 10 120 python3 tools/frame_prof.py 2>&1 | tail -1
run() { name=$1; shift; timeout -k 10 300 python3 bench.py "$@" > $O/$name.json 2> $O/$name.err; python3 -c "import json;d=json.loads(open('$O/$name.json').read().splitlines()[-1]);print('$name', round(d['ms_per_step'],4), {k:(round(v,4) if v else v) for k,v in d['kernels_ms_avg'].items()})"; }
for i in 1 2; do run bench5_$i --no-cpu-baseline --no-pcie; run shard_$i --scenes 262144 --no-cpu-baseline --no-pcie; done
