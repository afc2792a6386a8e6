#!/bin/bash
# A/B on one box: eager vs HIP-graph replay of the training step (CNN-B1 b256, ResNet-50 b128)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for g in 0 1 0 1; do
  timeout -k 10 300 python bench.py --groupby-extra 0 --graph $g --steps 30 --warmup 5 > gpurun_out/ab_cnn_g$g.json 2> gpurun_out/ab_cnn_g$g.err || { tail -30 gpurun_out/ab_cnn_g$g.err; exit 1; }
  echo "cnn graph=$g $(cut -c1-200 gpurun_out/ab_cnn_g$g.json)"
done
for g in 0 1; do
  timeout -k 10 300 python bench.py --workload resnet50 --batch-size 128 --steps 10 --warmup 3 --graph $g > gpurun_out/ab_rn_g$g.json 2> gpurun_out/ab_rn_g$g.err || { tail -30 gpurun_out/ab_rn_g$g.err; exit 1; }
  echo "rn50 graph=$g $(cut -c1-200 gpurun_out/ab_rn_g$g.json)"
done
echo done
