#!/bin/bash
# step gantts (b256 unless B is set) under the default library and each variant named in $@
# (PTG_HIP_LIB=libptg_hip_<name>.so): gpurun_out/gantt_<name>.txt
set -o pipefail
export PYTHONPATH=$PWD
for v in default "$@"; do
  lib=""; [ "$v" != default ] && lib="libptg_hip_$v.so"
  PTG_HIP_LIB=$lib BENCH_ARGS="--batch-size ${B:-256}" bash tools/gpu.sh prof > /dev/null || exit 1
  python tools/step_gantt.py gpurun_out/prof_cnn_b1/run_kernel_trace.csv > gpurun_out/gantt_$v.txt 2>&1
  rm -rf gpurun_out/prof_cnn_b1
done
