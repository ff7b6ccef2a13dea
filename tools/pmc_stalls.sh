#!/bin/bash
# SQ stall counters of the benched library per launch shape (GPU box, repo root):
#   tools/pmc_stalls.sh TAG  ->  gpurun_out/TAG/stall_{c5,c3,c4}/  (one --pmc pass each, 8 SQ counters)
# Summarise with tools/pmc_stalls_summary.py TAG.
set -eo pipefail
TAG=${1:-stalls}
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
B="--steps 2 --warmup 1 --no-cpu-baseline --no-pcie --no-shard-projection --no-comfort"
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU"
for c in c5 c3 c4; do
  case $c in c5) X="";; c3) X="--emit-paths --n-speeds 8 --n-points 100 --scenes 262144";; c4) X="--draws 64 --n-speeds 1 --scenes 16384";; esac
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $PWD/$O/stall_$c -o run -- python3 bench.py $B $X > $O/stall_$c.log 2>&1
  echo "stall $c done"
done
