set -o pipefail
O=gpurun_out/r04_s10; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
bash tools/frame_ab.sh 2 sw0 2>&1 | tee $O/frame_ab.txt
for S in 4096 3000; do echo "S=$S"; ARGS="--scenes $S --steps 300 --warmup 30" bash tools/ab.sh 2 sw0 2>&1; done | tee $O/ab2.txt
PPAMD_LIB=$PWD/carnd-path-planning-project_amd/ppamd/libppamd_var_fprof.so timeout -k 10 120 python3 tools/frame_prof.py 2>&1 | tail -1
