set -o pipefail
O=gpurun_out/r02v; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
PPAMD_LIB=$PWD/carnd-path-planning-project_amd/ppamd/libppamd_var_check.so PP_CHECK_OUT=$PWD/$O/check.json timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/check_tests.log 2>&1 || { tail -30 $O/check_tests.log; cat $O/check.json; exit 1; }
tail -1 $O/check_tests.log; cat $O/check.json
timeout -k 10 120 python bench.py --no-cpu-baseline > $O/c5.json 2> $O/c5.err || exit 1
python -c "import json;j=json.loads(open('$O/c5.json').read().strip().splitlines()[-1]);print('c5',j['ms_per_step'],j['kernels_ms_avg'])"
