#!/bin/bash
# End-to-end workloads on the GPU: joint ETL->Parquet->train, MNIST CNN, ResNet-50 trainer, groupBy.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python workloads/joint/etl_to_train.py --rows 20000000 --out /tmp/joint --epochs 2 --batch-size 8192 > gpurun_out/joint.log 2>&1 || { tail -30 gpurun_out/joint.log; exit 1; }
tail -1 gpurun_out/joint.log
timeout -k 10 300 python workloads/raw-tf/train_mnist.py --epochs 3 --steps-per-epoch 50 --batch-size 256 --output-dir /tmp/mnist > gpurun_out/mnist.log 2>&1 || { tail -30 gpurun_out/mnist.log; exit 1; }
tail -1 gpurun_out/mnist.log
timeout -k 10 300 python workloads/raw-tf/train_resnet50.py --epochs 2 --steps-per-epoch 10 --batch-size 128 --output-dir /tmp/rn50 > gpurun_out/rn50_train.log 2>&1 || { tail -30 gpurun_out/rn50_train.log; exit 1; }
tail -1 gpurun_out/rn50_train.log
timeout -k 10 300 python bench.py --workload groupby --steps 3 --warmup 1 > gpurun_out/bench_groupby.json 2> gpurun_out/bench_groupby.err || { tail -30 gpurun_out/bench_groupby.err; exit 1; }
cat gpurun_out/bench_groupby.json
timeout -k 10 300 python bench.py > gpurun_out/bench_cnn.json 2> gpurun_out/bench_cnn.err && cat gpurun_out/bench_cnn.json
timeout -k 10 400 python bench.py --workload resnet50 --batch-size 128 --steps 10 --warmup 3 > gpurun_out/bench_rn50.json 2> gpurun_out/bench_rn50.err && cat gpurun_out/bench_rn50.json
echo done
