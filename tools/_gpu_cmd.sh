set -o pipefail
O=gpurun_out/${1:-var}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
PPAMD_LIB=$PWD/carnd-path-planning-project_amd/ppamd/libppamd_var_carry.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_baseline_configs.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/carry_tests.log 2>&1 || { tail -30 $O/carry_tests.log; exit 1; }
tail -1 $O/carry_tests.log
bash tools/variants_bench.sh --steps 20 || exit 1
cp gpurun_out/variants.txt $O/
