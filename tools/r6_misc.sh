#!/bin/bash
# Round-6 evidence run: MNIST bf16 bench line + kernel stats (BASELINE config 3), the full default
# bench line (CNN-B1 + extras incl. the fit-amortised MLP), and the multi-rank DataFrame path's
# torch-op census (1-rank RCCL group with PTG_COLLECTIVES_WORLD1).
set -o pipefail
export PYTHONPATH=$PWD
bash tools/gpu.sh bench:mnist || exit 1
bash tools/gpu.sh prof:mnist || exit 1
timeout -k 10 300 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || { tail -20 gpurun_out/bench_full.err; exit 1; }
cat gpurun_out/bench_full.json
timeout -k 10 300 python tools/df_torch_ops.py --multirank --rows 4000000 > gpurun_out/df_torch_ops_multirank.txt 2>&1 || { tail -20 gpurun_out/df_torch_ops_multirank.txt; exit 1; }
cat gpurun_out/df_torch_ops_multirank.txt
