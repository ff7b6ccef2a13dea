#!/bin/bash
# GPU box (repo root): the round's parity evidence. tools/gpu_suite.sh TAG [BENCH ARGS...]
#   1. pytest -m gpu on the product library (every call under PP_DBG_POISON, tests/conftest.py)
#   2. the same suite on the -DPP_CHECK build (tools/variants.sh check "-DPP_CHECK"): bounds of
#      every kernel store, LDS poison per k_cand group, flagged-group list bounds; the violation
#      record goes to gpurun_out/TAG/check.json and any violation fails the step
#   3. smoke(), then one short default bench line (no CPU baseline) for a timing sanity check
# Each GPU step has its own time limit; the script stops at the first failure.
set -eo pipefail
TAG=${1:-suite}; shift || true
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
T="python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread"
timeout -k 10 420 $T > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
CHK=carnd-path-planning-project_amd/ppamd/libppamd_var_check.so
if [ -f $CHK ]; then
  PPAMD_LIB=$PWD/$CHK PP_CHECK_OUT=$OUT/check.json timeout -k 10 600 $T > $OUT/gpu_tests_check.log 2>&1 || { tail -40 $OUT/gpu_tests_check.log; cat $OUT/check.json 2>/dev/null; exit 1; }
  tail -1 $OUT/gpu_tests_check.log; cat $OUT/check.json
fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-pcie "$@" > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);print('%.4g'%d['value'],round(d['ms_per_step'],3),{k:round(v,3) for k,v in d['kernels_ms_avg'].items() if v})" $OUT/bench.json
