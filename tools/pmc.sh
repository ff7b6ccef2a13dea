#!/bin/bash
# PMC passes for the roofline/traffic figures (run on the GPU box from the repo root).
# One rocprofv3 invocation per counter group (FETCH_SIZE and WRITE_SIZE cannot share a pass);
# --pmc is never combined with sys/runtime/hip traces.
set -e
OUT=${1:-gpurun_out/pmc}
shift || true
ARGS=${@:---steps 2 --warmup 1 --no-cpu-baseline --no-pcie}
ROOT=$(pwd)
mkdir -p $OUT
export TMPDIR=/tmp
run() {
  name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d $ROOT/$OUT/$name -o $name -- python3 $ROOT/bench.py $ARGS > $ROOT/$OUT/$name.log 2>&1
  echo "pass $name rc=$?"
}
run fetch FETCH_SIZE
run write WRITE_SIZE
run sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE
run f64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP64_TRANS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_INT32
