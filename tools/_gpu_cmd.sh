set -o pipefail
O=gpurun_out/r02t; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for F in 1 0 1 0; do
PP_PREP_ST=$F timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 > $O/c5_st$F.json 2> $O/c5_st$F.err || exit 1
python -c "import json;j=json.loads(open('$O/c5_st$F.json').read().strip().splitlines()[-1]);print('c5 st=$F',j['ms_per_step'],j['kernels_ms_avg'])"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for F in 1 0; do
PP_PREP_ST=$F timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $PWD/$O/fetch$F -o f -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/fetch$F.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv,glob
for F in "10":
    for f in glob.glob(f"gpurun_out/r02t/fetch{F}/**/*counter_collection.csv", recursive=True):
        v={}
        for r in csv.DictReader(open(f)):
            k=r["Kernel_Name"].split("(")[0]
            if "k_prep" in k: v.setdefault(k,[]).append(float(r["Counter_Value"]))
        print(F, {k:sum(x)/len(x) for k,x in v.items()})
PY
