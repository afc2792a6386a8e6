#!/usr/bin/env bash
# Round-5 end-of-round evidence on one MI355X (through gpurun from the repo root), in parts:
#   bash tools/r5_final.sh cnn      driver-style bench + b256 traces (overlapped, serialized) + b32 trace + PMC
#   bash tools/r5_final.sh rn50     ResNet-50 bench + trace + PMC
#   bash tools/r5_final.sh df       groupBy cardinality sweep, 1B orderBy, DataFrame operator profile
# Every step is a tools/gpu.sh task with its own time limit; a part stops at its first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R" && mkdir -p gpurun_out
case "$1" in
  cnn)
    bash tools/gpu.sh bench && cp gpurun_out/bench_cnn_b1.json gpurun_out/r5_bench_final.json &&
      bash tools/gpu.sh prof && cp gpurun_out/prof_cnn_b1_summary.txt gpurun_out/r5_b256_kernel_stats.txt &&
      python tools/roofline_r4.py gpurun_out/prof_cnn_b1/run_kernel_trace.csv > gpurun_out/r5_roofline_overlapped.txt &&
      python tools/step_gantt.py gpurun_out/prof_cnn_b1/run_kernel_trace.csv > gpurun_out/r5_gantt_b256.txt &&
      PTG_SIDE_STREAM=0 bash tools/gpu.sh prof &&
      python tools/roofline_r4.py gpurun_out/prof_cnn_b1/run_kernel_trace.csv --serial > gpurun_out/r5_roofline_serial.txt &&
      PROF_STEPS=20 BENCH_ARGS="--batch-size 32" bash tools/gpu.sh prof && cp gpurun_out/prof_cnn_b1_summary.txt gpurun_out/r5_b32_kernel_stats.txt &&
      python tools/step_gantt.py gpurun_out/prof_cnn_b1/run_kernel_trace.csv > gpurun_out/r5_gantt_b32.txt &&
      python tools/roofline_r4.py gpurun_out/prof_cnn_b1/run_kernel_trace.csv --batch 32 > gpurun_out/r5_roofline_b32.txt &&
      bash tools/gpu.sh pmc && cp gpurun_out/pmc_cnn_b1_report.txt gpurun_out/r5_pmc_report.txt ;;
  rn50)
    BENCH_ARGS="--steps 20 --warmup 5" bash tools/gpu.sh bench:resnet50 && cp gpurun_out/bench_resnet50.json gpurun_out/r5_rn50_bench.json &&
      PROF_STEPS=5 bash tools/gpu.sh prof:resnet50 && cp gpurun_out/prof_resnet50_summary.txt gpurun_out/r5_rn50_kernel_stats.txt &&
      bash tools/gpu.sh pmc:resnet50 && cp gpurun_out/pmc_resnet50_report.txt gpurun_out/r5_rn50_pmc_report.txt ;;
  df)
    PY_ARGS="--keys 1000,65536,1000000,16000000,128000000" bash tools/gpu.sh py:tools/groupby_sweep.py &&
      cp gpurun_out/groupby_sweep.log gpurun_out/r5_groupby_sweep.log &&
      BENCH_ARGS="--steps 3 --warmup 1" bash tools/gpu.sh bench:sort && cp gpurun_out/bench_sort.json gpurun_out/r5_sort.json &&
      PY_ARGS="--sparse --steps 5" bash tools/gpu.sh py:tools/groupby_case.py && cp gpurun_out/groupby_case.log gpurun_out/r5_groupby_sparse1m.log ;;
  *) echo "usage: $0 cnn|rn50|df"; exit 2 ;;
esac
