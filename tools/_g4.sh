set -o pipefail
timeout -k 10 300 python3 tools/split_probe.py 262144 3 > gpurun_out/split_probe.txt 2>&1; cat gpurun_out/split_probe.txt
for v in trace trace2; do PPAMD_LIB=$PWD/carnd-path-planning-project_amd/ppamd/libppamd_var_$v.so timeout -k 10 120 python3 tools/trace_frame.py 2>&1 | tail -1; done
