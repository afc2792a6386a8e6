#!/bin/bash
# A/B of the persistent-grid oversubscription on CNN-B1 / CNN-A1 (1 GPU).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for k in 1 2 4; do
  for wl in cnn_b1 cnn_a1; do
    PTG_PERSIST_OVERSUB=$k timeout -k 10 200 python bench.py --workload $wl --groupby-extra 0 > gpurun_out/os_$k_$wl.json 2>/dev/null || exit 1
    echo "oversub=$k $wl $(python -c "import json;d=json.load(open('gpurun_out/os_$k_$wl.json'));print(d['value'], d['ms_per_step'])")"
  done
done
