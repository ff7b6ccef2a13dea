set -o pipefail
O=gpurun_out/${1:-var}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_baseline_configs.py tests/test_pipeline.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/variants_bench.sh --steps 20 || exit 1
cp gpurun_out/variants.txt $O/
