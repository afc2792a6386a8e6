#!/bin/bash
# quick gantts of the current step at b256 / b32 / b64 (CNN only)
set -o pipefail
export PYTHONPATH=$PWD
for B in 256 32 64; do
  BENCH_ARGS="--batch-size $B" bash tools/gpu.sh prof > /dev/null || exit 1
  python tools/step_gantt.py gpurun_out/prof_cnn_b1/run_kernel_trace.csv > gpurun_out/gantt_b$B.txt 2>&1
  rm -rf gpurun_out/prof_cnn_b1
done
