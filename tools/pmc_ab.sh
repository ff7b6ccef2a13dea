#!/bin/bash
# PMC A/B: SQ counters for the product lib and a variant (k_prep focus)
set -e
export TMPDIR=/tmp
ROOT=$(pwd)
for v in base cs0; do
  if [ $v = base ]; then export PPAMD_LIB=$ROOT/carnd-path-planning-project_amd/ppamd/libppamd.so; else export PPAMD_LIB=$ROOT/carnd-path-planning-project_amd/ppamd/libppamd_var_$v.so; fi
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_LDS --output-format csv -d $ROOT/gpurun_out/pmcab/$v/sq -o sq -- python3 $ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $ROOT/gpurun_out/pmcab/$v.sq.log 2>&1
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_RD --output-format csv -d $ROOT/gpurun_out/pmcab/$v/w -o w -- python3 $ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $ROOT/gpurun_out/pmcab/$v.w.log 2>&1
  echo "$v done"
done
