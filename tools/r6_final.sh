#!/bin/bash
# Round-6 end evidence: GPU suite, smoke, default bench line, CNN-B1 profiles (overlapped / serialized
# b256, b32, b64), PMC report, ResNet-50 and MNIST lines.  Outputs: gpurun_out/r6end/
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/r6end
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1 \
  || { tail -40 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
timeout -k 10 600 python bench.py > $O/bench_cnn_b1.json 2> $O/bench_cnn_b1.err || { tail -20 $O/bench_cnn_b1.err; exit 1; }
cut -c1-200 $O/bench_cnn_b1.json
bash tools/gpu.sh prof > /dev/null || exit 1
python tools/step_gantt.py gpurun_out/prof_cnn_b1/run_kernel_trace.csv > $O/cnn_b1_b256_gantt.txt 2>&1
python tools/roofline_r4.py gpurun_out/prof_cnn_b1/run_kernel_trace.csv --batch 256 > $O/cnn_b1_b256_roofline_overlapped.txt 2>&1
cp gpurun_out/prof_cnn_b1_summary.txt $O/cnn_b1_b256_kernel_stats.txt
rm -rf gpurun_out/prof_cnn_b1
PTG_SIDE_STREAM=0 bash tools/gpu.sh prof > /dev/null || exit 1
python tools/roofline_r4.py gpurun_out/prof_cnn_b1/run_kernel_trace.csv --batch 256 --serial > $O/cnn_b1_b256_roofline_serialized.txt 2>&1
python tools/step_gantt.py gpurun_out/prof_cnn_b1/run_kernel_trace.csv > $O/cnn_b1_b256_gantt_serialized.txt 2>&1
rm -rf gpurun_out/prof_cnn_b1
for B in 32 64; do
  BENCH_ARGS="--batch-size $B" bash tools/gpu.sh prof > /dev/null || exit 1
  python tools/step_gantt.py gpurun_out/prof_cnn_b1/run_kernel_trace.csv > $O/cnn_b1_b${B}_gantt.txt 2>&1
  python tools/roofline_r4.py gpurun_out/prof_cnn_b1/run_kernel_trace.csv --batch $B > $O/cnn_b1_b${B}_roofline.txt 2>&1
  rm -rf gpurun_out/prof_cnn_b1
done
bash tools/gpu.sh pmc > /dev/null || exit 1
cp gpurun_out/pmc_cnn_b1_report.txt $O/cnn_b1_pmc_report.txt
rm -rf gpurun_out/pmc_cnn_b1_a gpurun_out/pmc_cnn_b1_b
timeout -k 10 300 python bench.py --workload resnet50 > $O/bench_resnet50_b128.json 2>/dev/null || exit 1
timeout -k 10 300 python bench.py --workload mnist > $O/bench_mnist.json 2>/dev/null || exit 1
cut -c1-160 $O/bench_resnet50_b128.json $O/bench_mnist.json
echo done
