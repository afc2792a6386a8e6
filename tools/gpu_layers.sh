#!/bin/bash
# Per-op CNN-B1 layer timings (+ the conv/prelu kernel tests) on one MI355X; A/B of PTG_CONV_WLDS.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_nn_kernels_gpu.py -q -x -k "prelu_pool or halo" > gpurun_out/layers_pytest.log 2>&1 || { tail -30 gpurun_out/layers_pytest.log; exit 1; }
tail -2 gpurun_out/layers_pytest.log
echo "== WLDS on"
PYTHONPATH=. timeout -k 10 300 python tools/cnn_layer_bench.py ${LAYER_ARGS:-} 2>&1 | tee gpurun_out/layers.log
echo "== WLDS off"
PTG_CONV_WLDS=0 PYTHONPATH=. timeout -k 10 300 python tools/cnn_layer_bench.py --only fwd3,fwd4,fwd5,dgrad2,dgrad3,dgrad4,dgrad5 2>&1 | tee gpurun_out/layers_off.log
