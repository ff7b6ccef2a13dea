set -o pipefail
O=gpurun_out/r02ac; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 > $O/c5.json 2> $O/c5.err || exit 1
python -c "import json;j=json.loads(open('$O/c5.json').read().strip().splitlines()[-1]);print('c5',j['ms_per_step'],j['value']/1e9,j['kernels_ms_avg'])"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$O/stats -o run -- python3 bench.py --no-cpu-baseline > $O/c5_prof.json 2> $O/c5_prof.err || exit 1
cut -c1-120 $O/stats/run_kernel_stats.csv | head -8
