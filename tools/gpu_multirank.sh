#!/bin/bash
# 2 ranks sharing the one GPU of a gpurun box (gloo collectives): sharded vs all-reduce update with the
# HIP kernels, then the bench contract at --gpus 2.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PTG_DIST_BACKEND=gloo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 tools/rehearse_multirank.py > gpurun_out/rehearse.log 2>&1 || { tail -40 gpurun_out/rehearse.log; exit 1; }
grep REHEARSAL gpurun_out/rehearse.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 2 --steps 4 --warmup 2 --groupby-extra 0 --batch-size 64 > gpurun_out/bench2.log 2>&1 || { tail -40 gpurun_out/bench2.log; exit 1; }
grep metric gpurun_out/bench2.log
echo done
