#!/bin/bash
# Config-1 check on the GPU box (repo root): pp_plan_frame's parity tests, its latency next to the
# reference's planning code (tools/bench_frame.py), and the single-frame kernel's phase timeline
# (tools/trace_frame.py on the -DPP_TRACE build). tools/gpu_frame_check.sh [TAG]
set -o pipefail
O=gpurun_out/${1:-frame}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_cartable.py tests/test_abi_caller.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 200 python3 tools/bench_frame.py --frames 2000 > $O/frame.json 2> $O/frame.err || { tail -20 $O/frame.err; exit 1; }
cat $O/frame.json
PPAMD_LIB=$PWD/carnd-path-planning-project_amd/ppamd/libppamd_var_trace.so timeout -k 10 120 python3 tools/trace_frame.py > $O/trace_frame.txt 2>&1 || { tail -20 $O/trace_frame.txt; exit 1; }
tail -1 $O/trace_frame.txt
