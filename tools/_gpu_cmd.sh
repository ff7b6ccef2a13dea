set -o pipefail
O=gpurun_out/${1:-var}; mkdir -p $O
export TMPDIR=/tmp
ROOT=$PWD
for v in base nocars nomatch; do
  if [ $v = base ]; then L=$ROOT/carnd-path-planning-project_amd/ppamd/libppamd.so; else L=$ROOT/carnd-path-planning-project_amd/ppamd/libppamd_var_$v.so; fi
  PPAMD_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_BUSY_CYCLES --output-format csv -d $ROOT/$O/$v -o $v -- python3 $ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/$v.log 2>&1 || { tail $O/$v.log; exit 1; }
  echo "$v done"
done
