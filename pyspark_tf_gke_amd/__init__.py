"""pyspark_tf_gke_amd — an MI355X-native distributed DataFrame + training runtime.

Capability parity target: greg-ogs/PySpark-TF-GKE (Spark DataFrame/ML workloads + TF/Keras
training with ParameterServerStrategy).  Compute runs in hand-written gfx950 HIP kernels
(csrc/kernels), tensors move over RCCL/xGMI, one process per GPU.

Subpackages: ``sql`` (SparkSession/DataFrame), ``ml`` (Pipeline, StringIndexer, OneHotEncoder,
VectorAssembler, KMeans, ClusteringEvaluator), ``nn`` (Keras-shaped layers/models/optimizers),
``data`` (tf.data-shaped Dataset), ``distribute`` (strategies, ClusterCoordinator),
``parallel`` (RCCL process groups, shuffles), ``models`` (model families), ``ops`` (kernels),
``runtime`` (launcher, config), ``utils`` (logging, profiling, checkpoints), ``cli``.
"""
__version__ = "0.1.0"
