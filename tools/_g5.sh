set -o pipefail
O=gpurun_out/r04_s5; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_cartable.py tests/test_abi_caller.py tests/test_baseline_configs.py tests/test_shape_sequence.py tests/test_rollout.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
bash tools/frame_ab.sh 2 fw0 rep serpass 2>&1 | tee $O/frame_ab.txt
ARGS="--scenes 4096 --steps 300 --warmup 30" bash tools/ab.sh 2 rep serpass 2>&1 | tee $O/ab2.txt
PPAMD_LIB=$PWD/carnd-path-planning-project_amd/ppamd/libppamd_var_trace.so timeout -k 10 120 python3 tools/trace_frame.py 2>&1 | tail -1
