"""Make the in-tree package importable when a check is run as a script."""
import os
import sys

_ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), *([".."] * 4)))
if os.path.isdir(os.path.join(_ROOT, "pyspark_tf_gke_amd")) and _ROOT not in sys.path:
    sys.path.insert(0, _ROOT)
