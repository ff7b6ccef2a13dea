set -o pipefail
O=gpurun_out/r02n; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
bash tools/variants_bench.sh --scenes 4096 --steps 200 --warmup 20 > $O/vb.txt 2>&1 || { tail -20 $O/vb.txt; exit 1; }
cp gpurun_out/variants.txt $O/variants_c2.txt; cat $O/variants_c2.txt
timeout -k 10 120 python bench.py --no-cpu-baseline > $O/c5.json 2> $O/c5.err || exit 1
python -c "import json;j=json.loads(open('$O/c5.json').read().strip().splitlines()[-1]);print('c5',j['ms_per_step'],j['kernels_ms_avg'])"
timeout -k 10 200 python bench.py --scenes 262144 --n-speeds 8 --n-points 100 --emit-paths --no-cpu-baseline > $O/c3.json 2> $O/c3.err || exit 1
python -c "import json;j=json.loads(open('$O/c3.json').read().strip().splitlines()[-1]);print('c3',j['ms_per_step'],j['kernels_ms_avg'],j['roofline']['frac'])"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$O/c2prof -o run -- python3 bench.py --scenes 4096 --steps 200 --warmup 20 --no-cpu-baseline > $O/c2_prof.json 2> $O/c2_prof.err || exit 1
ls -R $O/c2prof | head
