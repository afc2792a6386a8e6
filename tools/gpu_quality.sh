#!/bin/bash
# Model-quality run of the reference's CNN-B1 on synthetic laser-spot frames:
# train_tf_ps.py --data-is-images for 150 epochs (the reference's schedule) at batch 32 and 256,
# history.json + mae.png + log copied under gpurun_out/quality/.  Each step under its own timeout.
set -o pipefail
OUT=gpurun_out/quality
mkdir -p $OUT/b32 $OUT/b256
EPOCHS=${EPOCHS:-150}
N=${N:-3000}
timeout -k 10 560 python -u workloads/raw-tf/train_tf_ps.py --data-is-images --synthetic $N --data-path /tmp/laser \
    --epochs $EPOCHS --batch-size 32 --output-dir /tmp/q32 --plot --cache-decoded --strategy none \
    > $OUT/b32/train.log 2>&1 || exit $?
cp /tmp/q32/history.json /tmp/q32/mae.png $OUT/b32/ || exit $?
timeout -k 10 400 python -u workloads/raw-tf/train_tf_ps.py --data-is-images --data-path /tmp/laser \
    --epochs $EPOCHS --batch-size 256 --output-dir /tmp/q256 --plot --cache-decoded --strategy none \
    > $OUT/b256/train.log 2>&1 || exit $?
cp /tmp/q256/history.json /tmp/q256/mae.png $OUT/b256/
