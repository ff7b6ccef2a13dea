set -o pipefail
mkdir -p gpurun_out/r02j
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r02j/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r02j/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r02j/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02j/smoke.log 2>&1 || { cat gpurun_out/r02j/smoke.log; exit 1; }
cat gpurun_out/r02j/smoke.log
for G in 0 1 4 8; do
  PP_PREP_G=$G timeout -k 10 120 python bench.py --scenes 4096 --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/r02j/c2_G$G.json 2> gpurun_out/r02j/c2_G$G.err || exit 1
  python -c "import json;j=json.loads(open('gpurun_out/r02j/c2_G$G.json').read().strip().splitlines()[-1]);print('c2 G=$G',j['ms_per_step'],j['kernels_ms_avg'])"
done
bash tools/variants_bench.sh > gpurun_out/r02j/vb.txt 2>&1 && cat gpurun_out/variants.txt
