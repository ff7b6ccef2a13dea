set -o pipefail
bash tools/gpu_frame_check.sh r04_f2 || exit 1
bash tools/frame_ab.sh 2 ec8 ec16 > gpurun_out/r04_f2/frame_ab.txt 2>&1; cat gpurun_out/r04_f2/frame_ab.txt
ARGS="--scenes 4096 --steps 300 --warmup 30" bash tools/ab.sh 2 ec8 ec16 > gpurun_out/r04_f2/ab2.txt 2>&1; cat gpurun_out/r04_f2/ab2.txt
