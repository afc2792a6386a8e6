#!/bin/bash
set -o pipefail
export PYTHONPATH=$PWD
timeout -k 10 120 python tools/wgrad_check.py 2>&1 | grep shape || exit 1
bash tools/gpu.sh tests:"wgrad" || exit 1
for B in 32 64; do
  echo "# batch $B"
  ABM_ENVS="PTG_WG_SMALL_N=0" BENCH_ARGS="--batch-size $B" bash tools/gpu.sh abm || exit 1
done
