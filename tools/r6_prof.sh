set -o pipefail
bash tools/gpu.sh prof || exit 1
python tools/step_gantt.py gpurun_out/prof_cnn_b1/run_kernel_trace.csv > gpurun_out/r6_b256_gantt.txt 2>&1
python tools/roofline_r4.py gpurun_out/prof_cnn_b1/run_kernel_trace.csv --batch 256 > gpurun_out/r6_b256_roofline.txt 2>&1
cp gpurun_out/prof_cnn_b1_summary.txt gpurun_out/r6_b256_kernel_stats.txt
rm -rf gpurun_out/prof_cnn_b1
BENCH_ARGS="--batch-size 32" bash tools/gpu.sh prof || exit 1
python tools/step_gantt.py gpurun_out/prof_cnn_b1/run_kernel_trace.csv > gpurun_out/r6_b32_gantt.txt 2>&1
python tools/roofline_r4.py gpurun_out/prof_cnn_b1/run_kernel_trace.csv --batch 32 > gpurun_out/r6_b32_roofline.txt 2>&1
cp gpurun_out/prof_cnn_b1_summary.txt gpurun_out/r6_b32_kernel_stats.txt
rm -rf gpurun_out/prof_cnn_b1
bash tools/gpu.sh abvar:adamv4 abvar:adamv4p4
BENCH_ARGS="--batch-size 32" bash tools/gpu.sh abvar:adamv4
