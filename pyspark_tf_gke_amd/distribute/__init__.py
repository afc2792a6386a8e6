"""``tf.distribute``-shaped API over RCCL: strategies, cluster resolution, coordinator."""
from .cluster import (ClusterSpec, InputContext, MinSizePartitioner, Server, SimpleClusterResolver,  # noqa: F401
                      TFConfigClusterResolver, build_cluster_def, make_tf_config, validate_chief_addr)
from .coordinator import ClusterCoordinator, RemoteValue  # noqa: F401
from .strategy import (MirroredStrategy, MultiWorkerMirroredStrategy, OneDeviceStrategy,  # noqa: F401
                       Strategy, current_strategy)
from .ps import ParameterServerStrategy  # noqa: F401


class cluster_resolver:  # noqa: N801 - namespace like tf.distribute.cluster_resolver
    SimpleClusterResolver = SimpleClusterResolver
    TFConfigClusterResolver = TFConfigClusterResolver


class coordinator:  # noqa: N801
    ClusterCoordinator = ClusterCoordinator


class experimental:  # noqa: N801
    class partitioners:  # noqa: N801
        MinSizePartitioner = MinSizePartitioner
