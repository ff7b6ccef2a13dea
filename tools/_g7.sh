set -o pipefail
O=gpurun_out/r04_s7; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_cartable.py tests/test_abi_caller.py tests/test_rollout.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
PPAMD_LIB=$PWD/carnd-path-planning-project_amd/ppamd/libppamd_var_fprof.so timeout -k 10 120 python3 tools/frame_prof.py 2>&1 | tail -1
timeout -k 10 200 python3 tools/bench_frame.py --frames 2000 2>/dev/null | tail -1 | cut -c1-200
