#!/bin/bash
# Round-6 evidence: CNN-B1 only profiles (no MLP / groupBy extras in the traced process), overlapped
# and serialized, b256 and b32, a PMC report, the groupBy cardinality sweep and a ResNet-50 line.
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/r6ev
mkdir -p $O
bash tools/gpu.sh prof || exit 1
python tools/step_gantt.py gpurun_out/prof_cnn_b1/run_kernel_trace.csv > $O/cnn_b1_b256_gantt.txt 2>&1
python tools/roofline_r4.py gpurun_out/prof_cnn_b1/run_kernel_trace.csv --batch 256 > $O/cnn_b1_b256_roofline_overlapped.txt 2>&1
cp gpurun_out/prof_cnn_b1_summary.txt $O/cnn_b1_b256_kernel_stats.txt
rm -rf gpurun_out/prof_cnn_b1
PTG_SIDE_STREAM=0 bash tools/gpu.sh prof || exit 1
python tools/roofline_r4.py gpurun_out/prof_cnn_b1/run_kernel_trace.csv --batch 256 --serial > $O/cnn_b1_b256_roofline_serialized.txt 2>&1
python tools/step_gantt.py gpurun_out/prof_cnn_b1/run_kernel_trace.csv > $O/cnn_b1_b256_gantt_serialized.txt 2>&1
rm -rf gpurun_out/prof_cnn_b1
BENCH_ARGS="--batch-size 32" bash tools/gpu.sh prof || exit 1
python tools/step_gantt.py gpurun_out/prof_cnn_b1/run_kernel_trace.csv > $O/cnn_b1_b32_gantt.txt 2>&1
python tools/roofline_r4.py gpurun_out/prof_cnn_b1/run_kernel_trace.csv --batch 32 > $O/cnn_b1_b32_roofline.txt 2>&1
cp gpurun_out/prof_cnn_b1_summary.txt $O/cnn_b1_b32_kernel_stats.txt
rm -rf gpurun_out/prof_cnn_b1
bash tools/gpu.sh pmc || exit 1
cp gpurun_out/pmc_cnn_b1_report.txt $O/cnn_b1_pmc_report.txt
rm -rf gpurun_out/pmc_cnn_b1_a gpurun_out/pmc_cnn_b1_b
timeout -k 10 400 python -u tools/groupby_sweep.py > $O/groupby_cardinality_sweep.txt 2>&1 || exit 1
bash tools/gpu.sh bench:resnet50 || exit 1
cp gpurun_out/bench_resnet50.json $O/bench_resnet50_b128.json
