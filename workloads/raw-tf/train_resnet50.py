"""BASELINE.json workload: resnet50 training on synthetic data (see pyspark_tf_gke_amd/cli/train_baseline.py).
Launch N workers with `python -m pyspark_tf_gke_amd.runtime.launcher --nproc N -- python workloads/raw-tf/train_resnet50.py`."""
import sys

import _path  # noqa: F401

from pyspark_tf_gke_amd.cli.train_baseline import main

if __name__ == "__main__":
    sys.exit(main(["--model", "resnet50"] + sys.argv[1:]))
