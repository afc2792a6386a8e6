#!/usr/bin/env bash
# Launch distributed PS training on one 8xMI355X node
# (reference: workloads/raw-tf/run_tf_training_from_bastion.sh:10-135).
#
# The reference detects the chief's routable IPv4, looks up the worker/PS LoadBalancer IPs with
# kubectl and runs train_tf_ps.py --use-ps against the remote tf.distribute servers.  Here the
# workers and parameter-server shards are GPU ranks of one node: the launcher spawns one process
# per rank (RANK/LOCAL_RANK/WORLD_SIZE, MASTER_ADDR=127.0.0.1), the chief is rank 0, and the
# address flags are kept as an address book (validated, not dialled).
set -euo pipefail
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
ROOT="$(cd "$HERE/../.." && pwd)"

WORKERS="${WORKERS:-tf-trainer-0 tf-trainer-1}"
PS="${PS:-tf-trainer-ps-0}"
EPOCHS="${EPOCHS:-10}"
BATCH_SIZE="${BATCH_SIZE:-64}"
NPROC="${NPROC:-$(python3 -c 'import torch; print(max(1, torch.cuda.device_count()))' 2>/dev/null || echo 1)}"
GRPC_PORT="${TF_GRPC_PORT:-2222}"
CHIEF_PORT="${CHIEF_PORT:-2223}"

# chief address: single node -> loopback (the reference probes `ip route get 8.8.8.8` / hostname -I)
CHIEF_ADDR="${CHIEF_ADDR:-127.0.0.1}"
n_workers=$(wc -w <<<"$WORKERS")
n_ps=$(wc -w <<<"$PS")
worker_addrs=""
for i in $(seq 0 $((n_workers - 1))); do worker_addrs+="${worker_addrs:+,}127.0.0.1:$((GRPC_PORT + i))"; done
ps_addrs=""
for i in $(seq 0 $((n_ps - 1))); do ps_addrs+="${ps_addrs:+,}127.0.0.1:$((GRPC_PORT + 100 + i))"; done
export no_proxy="${no_proxy:-}${no_proxy:+,}127.0.0.1,localhost"
export HSA_ENABLE_IPC_MODE_LEGACY=0

echo "[bastion] chief=${CHIEF_ADDR}:${CHIEF_PORT} workers=${worker_addrs} ps=${ps_addrs} ranks=${NPROC}"
exec python3 -m pyspark_tf_gke_amd.runtime.launcher --nproc "$NPROC" --master-addr 127.0.0.1 -- \
  python3 "$ROOT/workloads/raw-tf/train_tf_ps.py" --use-ps \
  --worker-replicas "$n_workers" --ps-replicas "$n_ps" \
  --worker-addrs "$worker_addrs" --ps-addrs "$ps_addrs" \
  --chief-addr "$CHIEF_ADDR" --chief-port "$CHIEF_PORT" \
  --epochs "$EPOCHS" --batch-size "$BATCH_SIZE" "$@"
