set -o pipefail
O=gpurun_out/r02r; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 120 python bench.py --no-cpu-baseline > $O/c5.json 2> $O/c5.err || exit 1
python -c "import json;j=json.loads(open('$O/c5.json').read().strip().splitlines()[-1]);print('c5',j['ms_per_step'],j['kernels_ms_avg'])"
timeout -k 10 120 python bench.py --scenes 4096 --steps 300 --warmup 30 --no-cpu-baseline > $O/c2.json 2> $O/c2.err || exit 1
python -c "import json;j=json.loads(open('$O/c2.json').read().strip().splitlines()[-1]);print('c2',j['ms_per_step'],j['kernels_ms_avg'])"
