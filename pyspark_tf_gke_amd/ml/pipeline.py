"""Pipeline / PipelineModel (k_means.py:71-74, :151-152; spark_workload_to_cloud_k8s.py:104-107)
with Spark-ML-style persistence of the fitted stages."""
from __future__ import annotations

import json
import os

from .base import Estimator, MLReadable, MLWritable, Model, load_any, write_metadata


class Pipeline(Estimator, MLWritable, MLReadable):
    _defaults = {"stages": None}

    def __init__(self, stages=None):
        super().__init__()
        self.stages = list(stages or [])

    def setStages(self, stages):  # noqa: N802
        self.stages = list(stages)
        return self

    def getStages(self):  # noqa: N802
        return list(self.stages)

    def _fit(self, df):
        fitted = []
        cur = df
        for i, st in enumerate(self.stages):
            if isinstance(st, Estimator):
                m = st.fit(cur)
            else:
                m = st
            fitted.append(m)
            if i + 1 < len(self.stages):
                cur = m.transform(cur)
        return PipelineModel(fitted)

    def _save_impl(self, path):
        _save_stages(self, self.stages, path)

    @classmethod
    def _load_impl(cls, path, meta):
        return cls(_load_stages(path, meta))


class PipelineModel(Model, MLWritable, MLReadable):
    _defaults = {"stages": None}

    def __init__(self, stages=None):
        super().__init__()
        self.stages = list(stages or [])

    def _transform(self, df):
        for st in self.stages:
            df = st.transform(df)
        return df

    def _save_impl(self, path):
        _save_stages(self, self.stages, path)

    @classmethod
    def _load_impl(cls, path, meta):
        return cls(_load_stages(path, meta))


def _save_stages(obj, stages, path):
    uids = [s.uid for s in stages]
    write_metadata(obj, path, {"paramMap": {"stageUids": uids}})
    for i, st in enumerate(stages):
        st._save_impl(os.path.join(path, "stages", f"{i}_{st.uid}"))


def _load_stages(path, meta):
    out = []
    for i, uid in enumerate(meta["paramMap"]["stageUids"]):
        out.append(load_any(os.path.join(path, "stages", f"{i}_{uid}")))
    return out


_ = json
