#!/bin/bash
set -o pipefail
export PYTHONPATH=$PWD
bash tools/gpu.sh tests:"models or dist or graph" || exit 1
for B in 256 32 64; do
  echo "# batch $B"
  ABM_ENVS="PTG_ADAM_STREAM=0" BENCH_ARGS="--batch-size $B" bash tools/gpu.sh abm || exit 1
done
