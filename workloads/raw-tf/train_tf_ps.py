"""TF trainer entry point with the reference's exact flag surface (workloads/raw-tf/train_tf_ps.py:822-899).

CSV mode trains the MLP on health.csv (label_map.json, model.keras, history.json); ``--data-is-images``
trains the laser-spot CNN (``--synthetic N`` generates N random images of the reference shape when
the dataset is absent).  ``--use-ps`` runs ParameterServerStrategy + ClusterCoordinator over the
launched ranks (RCCL), otherwise a single-process ``model.fit``.  Implementation:
pyspark_tf_gke_amd/cli/train.py.
"""
import sys

import _path  # noqa: F401

from pyspark_tf_gke_amd.cli.train import main

if __name__ == "__main__":
    sys.exit(main())
