#!/bin/bash
# A/B of the low-LDS dW+Adam GEMM (libptg_hip_lowlds.so, -DPTG_ADAM_LOWLDS=1) vs the default, with
# and without an LDS pad, at b256 and b32 (bench.py, CNN only, interleaved x2)
set -o pipefail
export PYTHONPATH=$PWD
for B in 256 32; do
  for i in 1 2; do
    for cfg in "default" "lowlds:0" "lowlds:24000"; do
      lib=""; pad=""
      if [ "$cfg" != "default" ]; then lib=libptg_hip_lowlds.so; pad=${cfg#*:}; fi
      PTG_HIP_LIB=$lib PTG_ADAM_LDS_PAD=$pad timeout -k 10 200 python bench.py --batch-size $B --groupby-extra 0 \
        --extra-batches "" --mlp-batches "" --sim-world 0 > gpurun_out/ablow.json 2> gpurun_out/ablow.err || { tail -20 gpurun_out/ablow.err; exit 1; }
      echo "b$B $cfg $(python -c "import json; d = json.load(open('gpurun_out/ablow.json')); print(d['ms_per_step'])")"
    done
  done
done
