"""Device ops. ``ops.nn``: training kernels (GEMM/conv/PReLU/pool/loss/Adam); ``ops.df``: DataFrame and
ML kernels (expression VM, compaction, hash aggregation, partitioning, k-means, silhouette)."""
from . import nn  # noqa: F401
