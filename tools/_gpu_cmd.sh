set -o pipefail
O=gpurun_out/r02ab; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for S in 262144 524288 2097152; do
timeout -k 10 120 python bench.py --scenes $S --steps 30 --warmup 5 --no-cpu-baseline > $O/s$S.json 2> $O/s$S.err || exit 1
python -c "import json;j=json.loads(open('$O/s$S.json').read().strip().splitlines()[-1]);print('S=$S',j['ms_per_step'],j['value']/1e9,j['kernels_ms_avg'])"
done
PP_PREP_W4=1 timeout -k 10 120 python bench.py --scenes 524288 --steps 30 --warmup 5 --no-cpu-baseline > $O/w4.json 2> $O/w4.err || exit 1
python -c "import json;j=json.loads(open('$O/w4.json').read().strip().splitlines()[-1]);print('S=524288 W4',j['ms_per_step'],j['value']/1e9,j['kernels_ms_avg'])"
