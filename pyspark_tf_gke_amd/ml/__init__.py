"""``pyspark.ml``-shaped API: Pipeline, feature transformers, KMeans, ClusteringEvaluator."""
from . import clustering, evaluation, feature, linalg  # noqa: F401
from .clustering import KMeans, KMeansModel  # noqa: F401
from .evaluation import ClusteringEvaluator  # noqa: F401
from .feature import (OneHotEncoder, OneHotEncoderModel, StringIndexer, StringIndexerModel,  # noqa: F401
                      VectorAssembler)
from .pipeline import Pipeline, PipelineModel  # noqa: F401
