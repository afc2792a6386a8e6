#!/bin/bash
# conv1 forward prefetch depth: per-kernel time in the step (rocprof) and end-to-end A/B
set -o pipefail
export PYTHONPATH=$PWD
for pd in 1 2 3 4; do
  PTG_CONV1_PD=$pd BENCH_ARGS="--batch-size ${B:-256}" bash tools/gpu.sh prof > /dev/null || exit 1
  python tools/step_gantt.py gpurun_out/prof_cnn_b1/run_kernel_trace.csv > gpurun_out/gantt_pd$pd.txt 2>&1
  rm -rf gpurun_out/prof_cnn_b1
  echo "pd=$pd $(grep -h 'conv1_fwd\|^step' gpurun_out/gantt_pd$pd.txt | tr '\n' ' ' | cut -c1-200)"
done
ABM_ENVS="PTG_CONV1_PD=1;PTG_CONV1_PD=2;PTG_CONV1_PD=4" bash tools/gpu.sh abm
