set -o pipefail
O=gpurun_out/r02w; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for F in 1 0 1 0; do
PP_STEP_FUSED=$F timeout -k 10 120 python bench.py --scenes 4096 --steps 300 --warmup 30 --no-cpu-baseline > $O/c2_s$F.json 2> $O/c2_s$F.err || exit 1
python -c "import json;j=json.loads(open('$O/c2_s$F.json').read().strip().splitlines()[-1]);print('c2 step_fused=$F',j['ms_per_step'],j['kernels_ms_avg'])"
done
