#!/bin/bash
set -o pipefail
export PYTHONPATH=$PWD
for lib in "" libptg_hip_wg64a.so libptg_hip_wg64b.so libptg_hip_wg32a.so; do
  echo "== ${lib:-default}"
  PTG_HIP_LIB=$lib timeout -k 10 120 python tools/wgrad_check.py 2>&1 | grep shape || exit 1
  PTG_HIP_LIB=$lib timeout -k 10 120 python tools/cnn_layer_bench.py --only wgrad3,wgrad4,wgrad5 2>&1 | grep op || exit 1
  PTG_HIP_LIB=$lib timeout -k 10 120 python tools/cnn_layer_bench.py --batch 32 --only wgrad4,wgrad5 2>&1 | grep op || exit 1
done
