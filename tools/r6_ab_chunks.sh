#!/bin/bash
# A/B: big Dense dW+Adam as 1 (default) / 2 / 4 / 8 row-chunk launches forked along the backward chain
set -o pipefail
export PYTHONPATH=$PWD
bash tools/gpu.sh tests:"chunked_dense_adam or flip_in_adam" || exit 1
for B in 32 64 256; do
  echo "# batch $B"
  ABM_ENVS="PTG_DENSE_ADAM_CHUNKS=2;PTG_DENSE_ADAM_CHUNKS=4;PTG_DENSE_ADAM_CHUNKS=8" BENCH_ARGS="--batch-size $B" bash tools/gpu.sh abm || exit 1
done
