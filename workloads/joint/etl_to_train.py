"""Joint pipeline (BASELINE.json): Spark ETL -> Parquet -> TF train with every GPU acting as one
executor and one worker.  Launch on N GPUs with
``python -m pyspark_tf_gke_amd.cli.spark_submit --num-executors N workloads/joint/etl_to_train.py``
(or torchrun).  Implementation: pyspark_tf_gke_amd/pipeline/joint.py."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))

from pyspark_tf_gke_amd.parallel import comm  # noqa: E402
from pyspark_tf_gke_amd.pipeline import run_joint  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=int(os.environ.get("JOINT_ROWS", "10000000")), help="rows per executor")
    ap.add_argument("--out", default=os.environ.get("OUTPUT_DIR", "./joint-out"))
    ap.add_argument("--epochs", type=int, default=int(os.environ.get("EPOCHS", "2")))
    ap.add_argument("--batch-size", type=int, default=int(os.environ.get("BATCH_SIZE", "8192")))
    ap.add_argument("--handoff", choices=["parquet", "device"], default="parquet")
    ap.add_argument("--master", default=os.environ.get("SPARK_MASTER", "mi355x"))
    a = ap.parse_args(argv)
    rep = run_joint(a.rows, a.out, a.epochs, a.batch_size, a.handoff, a.master)
    if comm.rank() == 0:
        print(json.dumps(rep))


if __name__ == "__main__":
    main()
