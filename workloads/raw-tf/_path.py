"""Make the in-tree package importable when a workload is run as a script from any directory."""
import os
import sys

_ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
if os.path.isdir(os.path.join(_ROOT, "pyspark_tf_gke_amd")) and _ROOT not in sys.path:
    sys.path.insert(0, _ROOT)
