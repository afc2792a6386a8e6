#!/bin/bash
# A/B of one environment switch on the CNN-B1 bench: AB_ENV="VAR=value" (B side), alternating runs.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 200 python bench.py --groupby-extra 0 > gpurun_out/ab_a$i.json 2> gpurun_out/ab_a.err || { tail -20 gpurun_out/ab_a.err; exit 1; }
  echo "A $(cut -c1-140 gpurun_out/ab_a$i.json)"
  timeout -k 10 200 env $AB_ENV python bench.py --groupby-extra 0 > gpurun_out/ab_b$i.json 2> gpurun_out/ab_b.err || { tail -20 gpurun_out/ab_b.err; exit 1; }
  echo "B $(cut -c1-140 gpurun_out/ab_b$i.json)"
done
if [ "${PROF:-0}" = "1" ]; then
  export $AB_ENV
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ab -o run -- python bench.py --steps 10 --warmup 3 --groupby-extra 0 > gpurun_out/prof_ab.log 2>&1 || exit 1
fi
echo done
