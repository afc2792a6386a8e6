#!/bin/bash
set -o pipefail
export PYTHONPATH=$PWD
for B in 256 32; do
  echo "# batch $B"
  ABM_ENVS="PTG_SPARSE_POOL_LAYERS=2;PTG_SPARSE_POOL_LAYERS=3;PTG_SPARSE_POOL_LAYERS=2,3" BENCH_ARGS="--batch-size $B" bash tools/gpu.sh abm || exit 1
done
