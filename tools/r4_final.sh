#!/usr/bin/env bash
# Round-4 end-of-round evidence on one MI355X (run through gpurun from the repo root).  Every step
# is a tools/gpu.sh task with its own time limit; the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R" && mkdir -p gpurun_out
bash tools/gpu.sh bench && cp gpurun_out/bench_cnn_b1.json gpurun_out/r4_bench_final.json &&
  bash tools/gpu.sh prof && python tools/roofline_r4.py gpurun_out/prof_cnn_b1/run_kernel_trace.csv > gpurun_out/r4_roofline_overlapped.txt &&
  PTG_SIDE_STREAM=0 bash tools/gpu.sh prof && python tools/roofline_r4.py gpurun_out/prof_cnn_b1/run_kernel_trace.csv --serial > gpurun_out/r4_roofline_serial.txt 2>&1 ;
rc=$?
[ $rc -eq 0 ] || { echo "final chain stopped ($rc)"; exit $rc; }
bash tools/gpu.sh pmc && cp gpurun_out/pmc_cnn_b1_report.txt gpurun_out/r4_pmc_report.txt &&
  PY_ARGS="--keys 1000,65536,1000000,16000000,128000000" bash tools/gpu.sh py:tools/groupby_sweep.py && cp gpurun_out/groupby_sweep.log gpurun_out/r4_groupby_sweep.log &&
  PY_ARGS="--rows 200000000" PROF_TAG=dfops bash tools/gpu.sh profpy:tools/df_ops_profile.py &&
  PY_ARGS="--batch 64 --steps 40" bash tools/gpu.sh psmodes
