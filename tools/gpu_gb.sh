#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python workloads/joint/etl_to_train.py --rows 20000000 --out /tmp/joint --epochs 2 --batch-size 8192 > gpurun_out/joint.log 2>&1 || { tail -30 gpurun_out/joint.log; exit 1; }
tail -1 gpurun_out/joint.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_gb -o run -- python bench.py --workload groupby --steps 3 --warmup 1 > gpurun_out/prof_gb.log 2>&1 || exit 1
tail -1 gpurun_out/prof_gb.log
echo done
