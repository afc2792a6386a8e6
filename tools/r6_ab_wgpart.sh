#!/bin/bash
set -o pipefail
export PYTHONPATH=$PWD
for m in 0 1; do
  echo "== PTG_WG_PARTIAL=$m"
  PTG_WG_PARTIAL=$m timeout -k 10 120 python tools/wgrad_check.py 2>&1 | grep shape || exit 1
  PTG_WG_PARTIAL=$m timeout -k 10 120 python tools/cnn_layer_bench.py --only wgrad2,wgrad3,wgrad4,wgrad5 2>&1 | grep op || exit 1
  PTG_WG_PARTIAL=$m timeout -k 10 120 python tools/cnn_layer_bench.py --batch 32 --only wgrad2,wgrad3,wgrad4,wgrad5 2>&1 | grep op || exit 1
done
PTG_WG_PARTIAL=1 bash tools/gpu.sh tests:"wgrad or models" || exit 1
for B in 256 32 64; do
  echo "# batch $B"
  ABM_ENVS="PTG_WG_PARTIAL=1" BENCH_ARGS="--batch-size $B" bash tools/gpu.sh abm || exit 1
done
