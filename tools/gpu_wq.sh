#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_nn_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "work_queue or halo or sparse or sel" > gpurun_out/wq_pytest.log 2>&1 || { tail -30 gpurun_out/wq_pytest.log; exit 1; }
tail -1 gpurun_out/wq_pytest.log
for d in 0 1; do for wl in cnn_b1 cnn_a1; do
  PTG_PERSIST_DYNAMIC=$d timeout -k 10 200 python bench.py --workload $wl --groupby-extra 0 > gpurun_out/wq.json 2>/dev/null || exit 1
  echo "dynamic=$d $wl $(python -c "import json;d=json.load(open('gpurun_out/wq.json'));print(d['value'], d['ms_per_step'])")"
done; done
