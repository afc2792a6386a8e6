"""KMeans / KMeansModel (k_means.py:83-87, :138-162; spark_workload_to_cloud_k8s.py:117-133).

The feature matrix stays resident on the GPU for the whole fit (the reference re-runs its JDBC
scan + pipeline every Lloyd iteration because nothing is cached).  Each iteration is
ONE fused assign+accumulate kernel (centers in LDS, per-workgroup partial sums in LDS) plus a
k x D center update; across ranks the (k*D + k) partial sums and the cost are all-reduced (the
role of Spark's treeAggregate + broadcast, M6/M7).  Convergence follows Spark: stop when every
center moved less than ``tol`` (squared distance <= tol^2) or after ``maxIter``.

Initialisation: ``k-means||`` (Spark's default, initSteps=2): uniform first center, then
``initSteps`` rounds sampling each point with probability min(1, 2k d^2(x)/cost), candidates
weighted by the points they attract, reduced to k centers by weighted k-means++ on the driver —
seeded, deterministic for a given seed and world size.  ``random`` init is also supported.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ..ops import df as D
from ..parallel import comm
from ..sql import types as T
from ..sql.dataframe import DataFrame
from ..sql.table import ColumnVector
from .base import Estimator, MLReadable, MLWritable, Model, read_data, write_data, write_metadata
from .linalg import DenseVector


def _allreduce_np(a: np.ndarray) -> np.ndarray:
    if comm.world_size() == 1:
        return a
    return np.sum(comm.all_gather_object(a), axis=0)


class KMeans(Estimator, MLWritable, MLReadable):
    _defaults = {"featuresCol": "features", "predictionCol": "prediction", "k": 2, "initMode": "k-means||",
                 "initSteps": 2, "tol": 1e-4, "maxIter": 20, "seed": None, "distanceMeasure": "euclidean",
                 "weightCol": None}

    def __init__(self, featuresCol="features", predictionCol="prediction", k=2, initMode="k-means||",  # noqa: N803
                 initSteps=2, tol=1e-4, maxIter=20, seed=None, distanceMeasure="euclidean", weightCol=None):  # noqa: N803
        super().__init__(featuresCol=featuresCol, predictionCol=predictionCol, k=k, initMode=initMode,
                         initSteps=initSteps, tol=tol, maxIter=maxIter, seed=seed, distanceMeasure=distanceMeasure,
                         weightCol=weightCol)

    def _features(self, df: DataFrame):
        cv = df._t.column(self.getOrDefault("featuresCol"))
        if not isinstance(cv.dtype, T.VectorUDT):
            raise TypeError("features column must be a vector column (use VectorAssembler)")
        return cv.data.float().contiguous()

    def _init_centers(self, X: torch.Tensor, k: int, rng: np.random.Generator) -> torch.Tensor:
        n, Dm = X.shape
        dev = X.device
        if self.getOrDefault("initMode") == "random":
            loc = X[torch.from_numpy(rng.choice(n, size=min(k, n), replace=False)).to(dev)].cpu().numpy() if n else np.zeros((0, Dm))
            allc = np.concatenate(comm.all_gather_object(loc)) if comm.world_size() > 1 else loc
            return torch.from_numpy(allc[rng.choice(len(allc), size=k, replace=len(allc) < k)]).float().to(dev)
        # ---- k-means|| (distributed)
        counts = comm.all_gather_object(n) if comm.world_size() > 1 else [n]
        total = sum(counts)
        first = int(rng.integers(total))
        owner = int(np.searchsorted(np.cumsum(counts), first, side="right"))
        local_first = first - int(sum(counts[:owner]))
        c0 = X[local_first].cpu().numpy() if comm.rank() == owner else None
        if comm.world_size() > 1:
            c0 = next(c for c in comm.all_gather_object(c0) if c is not None)
        cands = [np.asarray(c0, dtype=np.float32)]
        mind = torch.empty(n, dtype=torch.float32, device=dev)
        for step in range(int(self.getOrDefault("initSteps"))):
            C = torch.from_numpy(np.stack(cands)).float().to(dev)
            if C.shape[0] * Dm > 8192:
                C = C[: max(1, 8192 // Dm)]
            D.kmeans_assign_accum(X, C, mind=mind)
            cost = float(_allreduce_np(np.array([float(mind.double().sum())]))[0])
            if cost <= 0:
                break
            g = torch.Generator(device="cpu")
            g.manual_seed(int(rng.integers(1 << 31)) + comm.rank())
            u = torch.rand(n, generator=g).to(dev)
            pick = (u < (2.0 * k * mind / cost)).to(torch.uint8)
            idx = D.compact(pick)
            new = X[idx].cpu().numpy() if idx.numel() else np.zeros((0, Dm), np.float32)
            if comm.world_size() > 1:
                new = np.concatenate(comm.all_gather_object(new))
            cands += list(new)
        C = np.stack(cands).astype(np.float32)
        # weights: number of points closest to each candidate
        w = np.zeros(len(C))
        for s0 in range(0, len(C), max(1, 8192 // Dm)):
            pass
        Ct = torch.from_numpy(C).to(dev)
        assign = torch.empty(n, dtype=torch.int32, device=dev)
        chunk = max(1, min(256, 8192 // Dm))
        best = torch.full((n,), math.inf, dtype=torch.float32, device=dev)
        barg = torch.zeros(n, dtype=torch.int64, device=dev)
        for s0 in range(0, len(C), chunk):
            D.kmeans_assign_accum(X, Ct[s0:s0 + chunk].contiguous(), assign=assign, mind=mind)
            better = mind < best
            best = torch.where(better, mind, best)
            barg = torch.where(better, assign.long() + s0, barg)
        w = np.bincount(barg.cpu().numpy(), minlength=len(C)).astype(np.float64)
        w = _allreduce_np(w)
        return torch.from_numpy(_weighted_kmeanspp(C.astype(np.float64), w, k, rng)).float().to(dev)

    def _fit(self, df: DataFrame):
        X = self._features(df)
        n, Dm = X.shape
        k = int(self.getOrDefault("k"))
        seed = self.getOrDefault("seed")
        rng = np.random.default_rng(0 if seed is None else int(seed))
        C = self._init_centers(X, k, rng)
        if C.shape[0] < k:
            raise ValueError("fewer distinct points than k")
        dev = X.device
        sums = torch.zeros((k, Dm), dtype=torch.float32, device=dev)
        counts = torch.zeros(k, dtype=torch.float32, device=dev)
        cost = torch.zeros(1, dtype=torch.float64, device=dev)
        moved = torch.zeros(1, dtype=torch.float32, device=dev)
        tol = float(self.getOrDefault("tol"))
        max_iter = int(self.getOrDefault("maxIter"))
        it = 0
        for it in range(1, max_iter + 1):
            sums.zero_(); counts.zero_(); cost.zero_(); moved.zero_()
            D.kmeans_assign_accum(X, C, sums=sums, counts=counts, cost=cost)
            if comm.world_size() > 1:
                buf = torch.cat([sums.view(-1), counts]).contiguous()
                comm.all_reduce_(buf)
                sums.copy_(buf[: k * Dm].view(k, Dm)); counts.copy_(buf[k * Dm:])
            D.kmeans_update(sums, counts, C, moved)
            if float(moved.item()) <= tol * tol:
                break
        assign = torch.empty(n, dtype=torch.int32, device=dev)
        cost.zero_()
        counts.zero_()
        sums.zero_()
        D.kmeans_assign_accum(X, C, assign=assign, sums=sums, counts=counts, cost=cost)
        sizes = _allreduce_np(counts.cpu().numpy().astype(np.float64))
        tcost = float(_allreduce_np(cost.cpu().numpy())[0])
        model = KMeansModel(C.cpu().numpy().astype(np.float64))
        model._params.update(self._params)
        model.summary = KMeansSummary(k, it, tcost, [int(s) for s in sizes])
        return model

    def _save_impl(self, path):
        write_metadata(self, path)

    @classmethod
    def _load_impl(cls, path, meta):
        o = cls()
        o._params.update(meta["paramMap"])
        o.uid = meta["uid"]
        return o


def _weighted_kmeanspp(C: np.ndarray, w: np.ndarray, k: int, rng) -> np.ndarray:
    """Weighted k-means++ on the candidate set, then a few local Lloyd iterations (Spark's
    LocalKMeans with 30 iterations)."""
    m = len(C)
    if m <= k:
        reps = np.concatenate([C, C[rng.integers(m, size=k - m)]]) if m < k else C
        return reps
    centers = [C[rng.choice(m, p=w / w.sum())]]
    d2 = ((C - centers[0]) ** 2).sum(1)
    for _ in range(1, k):
        p = w * d2
        if p.sum() <= 0:
            j = int(rng.integers(m))
        else:
            j = int(rng.choice(m, p=p / p.sum()))
        centers.append(C[j])
        d2 = np.minimum(d2, ((C - C[j]) ** 2).sum(1))
    cen = np.stack(centers)
    for _ in range(30):
        dist = ((C[:, None, :] - cen[None, :, :]) ** 2).sum(2)
        a = dist.argmin(1)
        moved = False
        for j in range(k):
            sel = a == j
            if w[sel].sum() > 0:
                nc = (C[sel] * w[sel, None]).sum(0) / w[sel].sum()
                moved |= not np.allclose(nc, cen[j])
                cen[j] = nc
        if not moved:
            break
    return cen


class KMeansSummary:
    def __init__(self, k, num_iter, cost, sizes):
        self.k = k
        self.numIter = num_iter
        self.trainingCost = cost
        self.clusterSizes = sizes


class KMeansModel(Model, MLWritable, MLReadable):
    _defaults = KMeans._defaults

    def __init__(self, centers=None, **kw):
        super().__init__(**kw)
        self._centers = np.asarray(centers if centers is not None else np.zeros((0, 0)), dtype=np.float64)
        self.summary = None

    @property
    def hasSummary(self):  # noqa: N802
        return self.summary is not None

    def clusterCenters(self):  # noqa: N802
        return [c.copy() for c in self._centers]

    def _transform(self, df: DataFrame) -> DataFrame:
        t = df._t
        X = t.column(self.getOrDefault("featuresCol")).data.float().contiguous()
        C = torch.from_numpy(self._centers).float().to(X.device)
        assign = torch.empty(X.shape[0], dtype=torch.int32, device=X.device)
        if X.shape[0]:
            D.kmeans_assign_accum(X, C, assign=assign)
        return df._new(t.with_column(self.getOrDefault("predictionCol"), ColumnVector(assign, T.IntegerType())))

    def predict(self, value) -> int:
        v = np.asarray(getattr(value, "toArray", lambda: value)(), dtype=np.float64)
        return int(((self._centers - v) ** 2).sum(1).argmin())

    def computeCost(self, df: DataFrame) -> float:  # noqa: N802 (removed in Spark 3; kept for convenience)
        t = df._t
        X = t.column(self.getOrDefault("featuresCol")).data.float().contiguous()
        C = torch.from_numpy(self._centers).float().to(X.device)
        cost = torch.zeros(1, dtype=torch.float64, device=X.device)
        D.kmeans_assign_accum(X, C, cost=cost)
        return float(_allreduce_np(cost.cpu().numpy())[0])

    def _save_impl(self, path):
        write_metadata(self, path)
        import pyarrow as pa

        write_data(path, {"clusterIdx": pa.array(list(range(len(self._centers))), pa.int32()),
                          "clusterCenter": pa.array([list(map(float, c)) for c in self._centers],
                                                    pa.list_(pa.float64()))})

    @classmethod
    def _load_impl(cls, path, meta):
        data = read_data(path)
        order = np.argsort(data["clusterIdx"])
        o = cls(np.asarray([data["clusterCenter"][i] for i in order]))
        o._params.update(meta["paramMap"])
        o.uid = meta["uid"]
        return o


_ = DenseVector
