#!/usr/bin/env bash
# One parameterised driver for GPU-box work (run through gpurun from the repo root):
#   gpurun --timeout 900 -- 'bash tools/gpu.sh tests bench prof'
# Tasks run in the order given; every GPU step has its own time limit and the first failure
# ends the script (no GPU step runs after a fault, abort or timeout).  Outputs go to gpurun_out/.
#   tests            pytest -m gpu (one process, per-test timeout)
#   tests:<expr>     pytest -m gpu -k <expr>
#   smoke            __graft_entry__.smoke()
#   bench            bench.py (defaults; BENCH_ARGS adds flags)
#   bench:<wl>       bench.py --workload <wl> (BENCH_ARGS adds flags)
#   prof[:<wl>]      rocprofv3 --kernel-trace --stats over a short bench run -> gpurun_out/prof_<wl>
#   pmc[:<wl>]       two PMC passes (MFMA/LDS/VALU/wait counters; FETCH_SIZE) -> gpurun_out/pmc_<wl>_{a,b}
#   ab               A/B: bench.py twice plain, twice with AB_ENV set (interleaved)
#   abm[:<wl>]       multi-way A/B: bench.py under each env set of ABM_ENVS ("X=1;Y=0"), plus defaults, x2
#   abvar:<name>     A/B: bench.py with the default library vs PTG_HIP_LIB=libptg_hip_<name>.so (built here by
#                    python -m pyspark_tf_gke_amd._native.build --variant <name> -D MACRO=..), interleaved x2
#   py:<script>      timeout 300 python <script> (e.g. py:tools/gemm_bench.py)
#   e2e              joint ETL->Parquet->train + MNIST + synthetic image train_tf_ps.py
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd /tmp && export TMPDIR=/tmp && cd "$R" && mkdir -p gpurun_out
export PYTHONPATH=$R
STEP_T=${STEP_T:-300}

fail() { echo "FAILED: $1"; [ -f "$2" ] && tail -40 "$2"; exit 1; }

for task in "$@"; do
  name=${task%%:*}; arg=""; [ "$name" != "$task" ] && arg=${task#*:}
  echo "== $task ($(date +%T))"
  case $name in
    tests)
      log=gpurun_out/pytest_gpu${arg:+_$arg}.log
      timeout -k 10 ${TESTS_T:-1100} python -u -m pytest tests -m gpu ${TESTS_X--x} -q --timeout 240 --timeout-method thread \
        ${arg:+-k "$arg"} > "$log" 2>&1 || fail tests "$log"
      tail -2 "$log" ;;
    smoke)
      timeout -k 10 $STEP_T python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
        || fail smoke gpurun_out/smoke.log
      tail -2 gpurun_out/smoke.log ;;
    bench)
      wl=${arg:-cnn_b1}
      timeout -k 10 $STEP_T python bench.py --workload "$wl" $BENCH_ARGS > "gpurun_out/bench_$wl.json" \
        2> "gpurun_out/bench_$wl.err" || fail bench "gpurun_out/bench_$wl.err"
      cat "gpurun_out/bench_$wl.json" ;;
    prof)
      wl=${arg:-cnn_b1}
      timeout -k 10 $STEP_T rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/prof_$wl" -o run -- \
        python bench.py --workload "$wl" --steps ${PROF_STEPS:-10} --warmup 3 --groupby-extra 0 --extra-batches "" --mlp-batches "" --sim-world 0 \
        $BENCH_ARGS > "gpurun_out/prof_$wl.log" 2>&1 || fail prof "gpurun_out/prof_$wl.log"
      grep metric "gpurun_out/prof_$wl.log" | cut -c1-200
      python tools/prof_summary.py "gpurun_out/prof_$wl/run_kernel_stats.csv" $(( ${PROF_STEPS:-10} + 3 )) > "gpurun_out/prof_${wl}_summary.txt" 2>&1 || true
      head -40 "gpurun_out/prof_${wl}_summary.txt" ;;
    pmc)
      wl=${arg:-cnn_b1}
      timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS \
        SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE --output-format csv \
        -d "gpurun_out/pmc_${wl}_a" -o run -- python bench.py --workload "$wl" --steps 2 --warmup 1 --groupby-extra 0 --mlp-batches "" --sim-world 0 \
        --extra-batches "" $BENCH_ARGS > "gpurun_out/pmc_${wl}_a.log" 2>&1 || fail pmc_a "gpurun_out/pmc_${wl}_a.log"
      timeout -s KILL 150 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "gpurun_out/pmc_${wl}_b" \
        -o run -- python bench.py --workload "$wl" --steps 2 --warmup 1 --groupby-extra 0 --extra-batches "" --mlp-batches "" --sim-world 0 \
        $BENCH_ARGS > "gpurun_out/pmc_${wl}_b.log" 2>&1 || fail pmc_b "gpurun_out/pmc_${wl}_b.log"
      python tools/pmc_report.py "gpurun_out/pmc_${wl}_a" "gpurun_out/pmc_${wl}_b" > "gpurun_out/pmc_${wl}_report.txt" \
        2>&1 || true
      head -30 "gpurun_out/pmc_${wl}_report.txt" ;;
    ab)
      for i in 1 2; do
        timeout -k 10 $STEP_T python bench.py --groupby-extra 0 --extra-batches "" --mlp-batches "" --sim-world 0 $BENCH_ARGS > gpurun_out/ab_a$i.json \
          2> gpurun_out/ab_a.err || fail ab_a gpurun_out/ab_a.err
        echo "A $(cut -c1-160 gpurun_out/ab_a$i.json)"
        timeout -k 10 $STEP_T env $AB_ENV python bench.py --groupby-extra 0 --extra-batches "" --mlp-batches "" --sim-world 0 $BENCH_ARGS \
          > gpurun_out/ab_b$i.json 2> gpurun_out/ab_b.err || fail ab_b gpurun_out/ab_b.err
        echo "B $(cut -c1-160 gpurun_out/ab_b$i.json)"
      done ;;
    abm)
      # multi-way interleaved A/B: ABM_ENVS="A=1 B=2;C=0;" (';'-separated env sets, empty = defaults)
      wl=${arg:-cnn_b1}
      IFS=';' read -ra sets <<< "${ABM_ENVS:-}"
      for i in 1 2; do
        for e in "${sets[@]}" ""; do
          timeout -k 10 $STEP_T env $e python bench.py --workload "$wl" --groupby-extra 0 --extra-batches "" --mlp-batches "" --sim-world 0 \
            $BENCH_ARGS > gpurun_out/abm.json 2> gpurun_out/abm.err || fail abm gpurun_out/abm.err
          echo "[${e:-default}] $(python -c "import json; d = json.load(open('gpurun_out/abm.json')); print(d['value'], d['ms_per_step'], 'final_loss', d['config'].get('final_loss'))")"
        done
      done ;;
    abvar)
      for i in 1 2; do
        for lib in "" "libptg_hip_$arg.so"; do
          PTG_HIP_LIB=$lib timeout -k 10 $STEP_T python bench.py --groupby-extra 0 --extra-batches "" --mlp-batches "" --sim-world 0 $BENCH_ARGS \
            > gpurun_out/abvar.json 2> gpurun_out/abvar.err || fail abvar gpurun_out/abvar.err
          echo "${lib:-default} $(cut -c1-160 gpurun_out/abvar.json)"
        done
      done ;;
    profpy)
      # profpy:<script>: rocprofv3 kernel stats of one python script (PY_ARGS, PROF_TAG, PROF_DIV = divisor)
      tag=$(basename "$arg" .py)${PROF_TAG:+_$PROF_TAG}
      timeout -k 10 $STEP_T rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/prof_$tag" -o run -- \
        python $arg $PY_ARGS > "gpurun_out/prof_$tag.log" 2>&1 || fail "profpy $arg" "gpurun_out/prof_$tag.log"
      grep -v "^\[" "gpurun_out/prof_$tag.log" | tail -3 | cut -c1-250
      python tools/prof_summary.py "gpurun_out/prof_$tag/run_kernel_stats.csv" ${PROF_DIV:-1} \
        > "gpurun_out/prof_${tag}_summary.txt" 2>&1 || true
      head -${PROF_HEAD:-16} "gpurun_out/prof_${tag}_summary.txt" | cut -c1-200 ;;
    joint2)
      # Spark ETL -> Parquet -> train with 2 executors/workers sharing the GPU (gloo: RCCL refuses two
      # ranks on one device)
      PTG_DIST_BACKEND=gloo timeout -k 10 $STEP_T python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port 29641 workloads/joint/etl_to_train.py --rows ${JOINT_ROWS:-5000000} \
        --out /tmp/joint2 --epochs 2 --batch-size 8192 > gpurun_out/joint2.log 2>&1 || fail joint2 gpurun_out/joint2.log
      tail -4 gpurun_out/joint2.log | cut -c1-300 ;;
    psmodes)
      # psmodes[:<nproc>]: the reference's PS loop, sync vs async, N ranks sharing the GPU (gloo control)
      PTG_DIST_BACKEND=gloo timeout -k 10 $STEP_T python -m pyspark_tf_gke_amd.runtime.launcher --nproc ${arg:-2} -- \
        python tools/ps_modes_bench.py $PY_ARGS > gpurun_out/psmodes_${arg:-2}.log 2>&1 || fail psmodes gpurun_out/psmodes_${arg:-2}.log
      grep '"mode"' gpurun_out/psmodes_${arg:-2}.log | cut -c1-400 ;;
    py)
      out=gpurun_out/$(basename "$arg" .py).log
      timeout -k 10 $STEP_T python $arg $PY_ARGS > "$out" 2>&1 || fail "py $arg" "$out"
      tail -${PY_TAIL:-30} "$out" ;;
    e2e)
      timeout -k 10 $STEP_T python workloads/joint/etl_to_train.py --rows 20000000 --out /tmp/joint --epochs 2 \
        --batch-size 8192 > gpurun_out/joint.log 2>&1 || fail joint gpurun_out/joint.log
      tail -3 gpurun_out/joint.log
      timeout -k 10 $STEP_T python workloads/raw-tf/train_mnist.py --epochs 3 --steps-per-epoch 50 --batch-size 256 \
        --output-dir /tmp/mnist > gpurun_out/mnist.log 2>&1 || fail mnist gpurun_out/mnist.log
      tail -3 gpurun_out/mnist.log
      timeout -k 10 $STEP_T python workloads/raw-tf/train_tf_ps.py --data-is-images --synthetic ${E2E_IMAGES:-4096} \
        --data-path /tmp/imgs --epochs ${E2E_EPOCHS:-6} --batch-size 256 --cache-decoded --output-dir /tmp/cnn \
        > gpurun_out/train_images.log 2>&1 || fail images gpurun_out/train_images.log
      grep -E "Epoch|samples/s" gpurun_out/train_images.log | tail -6 ;;
    *) echo "unknown task $task"; exit 2 ;;
  esac
done
echo "== done ($(date +%T))"
