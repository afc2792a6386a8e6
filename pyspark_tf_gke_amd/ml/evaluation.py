"""ClusteringEvaluator (spark_workload_to_cloud_k8s.py:141-144): silhouette with squared Euclidean
distance, Spark's closed form — per-cluster (count, sum vector, sum of squared norms) are
accumulated on the device and all-reduced, then each point's a/b terms are dot products against
the k cluster sums (one kernel), and the mean is reduced across ranks."""
from __future__ import annotations

import torch

import numpy as np

from ..ops import df as D
from ..parallel import comm
from .base import Params


class ClusteringEvaluator(Params):
    _defaults = {"predictionCol": "prediction", "featuresCol": "features", "metricName": "silhouette",
                 "distanceMeasure": "squaredEuclidean", "weightCol": None}

    def __init__(self, predictionCol="prediction", featuresCol="features", metricName="silhouette",  # noqa: N803
                 distanceMeasure="squaredEuclidean", weightCol=None):  # noqa: N803
        super().__init__(predictionCol=predictionCol, featuresCol=featuresCol, metricName=metricName,
                         distanceMeasure=distanceMeasure, weightCol=weightCol)

    def evaluate(self, df, params=None) -> float:
        if self.getOrDefault("distanceMeasure") != "squaredEuclidean":
            raise NotImplementedError("only squaredEuclidean silhouette")
        t = df._t
        X = t.column(self.getOrDefault("featuresCol")).data.float().contiguous()
        a = t.column(self.getOrDefault("predictionCol")).data.int().contiguous()
        k_loc = int(a.max().item()) + 1 if a.numel() else 0
        k = comm.all_reduce_int([k_loc], op=torch.distributed.ReduceOp.MAX)[0]
        S, Q, cnt = D.silhouette_sum(X, a, k)
        if comm.distributed():
            buf = torch.cat([S.view(-1), Q, cnt]).contiguous()
            comm.all_reduce_(buf)
            kd = S.numel()
            S.copy_(buf[:kd].view_as(S)); Q.copy_(buf[kd:kd + k]); cnt.copy_(buf[kd + k:])
        total = D.silhouette_points(X, a, S, Q, cnt)
        n = X.shape[0]
        total, n = comm.all_reduce_float([total, n])
        return float(total / n) if n else float("nan")

    def isLargerBetter(self) -> bool:  # noqa: N802
        return True


_ = np
