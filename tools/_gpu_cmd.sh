set -o pipefail
O=gpurun_out/r02s; mkdir -p $O
bash tools/variants_bench.sh --steps 30 > $O/vb.txt 2>&1 || { tail -20 $O/vb.txt; exit 1; }
cp gpurun_out/variants.txt $O/variants_a.txt
bash tools/variants_bench.sh --steps 30 > $O/vb.txt 2>&1 || { tail -20 $O/vb.txt; exit 1; }
cp gpurun_out/variants.txt $O/variants_b.txt; cat $O/variants_a.txt $O/variants_b.txt
