#!/bin/bash
# after the fill / multi-rank DataFrame fixes: MNIST line + stats, the census again, and the GPU tests
# that cover those paths
set -o pipefail
export PYTHONPATH=$PWD
bash tools/gpu.sh tests:"dist or df or models or mnist or workloads" || exit 1
bash tools/gpu.sh bench:mnist || exit 1
bash tools/gpu.sh prof:mnist || exit 1
timeout -k 10 300 python tools/df_torch_ops.py --multirank --rows 4000000 > gpurun_out/df_torch_ops_multirank.txt 2>&1 || { tail -20 gpurun_out/df_torch_ops_multirank.txt; exit 1; }
grep -v "^\[W\|RCCL\|HIP version\|ROCm version\|Hostname\|Librccl\|amdgpu.ids" gpurun_out/df_torch_ops_multirank.txt
