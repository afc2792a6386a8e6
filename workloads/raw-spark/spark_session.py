"""Session factory for the raw-spark workloads (reference: workloads/raw-spark/spark_session.py:6-91).

Same contract: ``CreateSparkSession().new_spark_session() -> (spark, logger, DB_CONFIG)`` with the
reference's logging format and DB defaults.  The master defaults to the MI355X executors
(``mi355x``: one executor per GPU rank, launched by ``cli.spark_submit``); ``SPARK_MASTER`` overrides
it (``local[2]`` runs on the host).  The driver host/port and block-manager port confs are kept and
validated, though executors exchange data over RCCL instead of Netty.
"""
import os
import socket

import _path  # noqa: F401

from pyspark_tf_gke_amd.sql import SparkSession
from pyspark_tf_gke_amd.utils.logging import get_logger


class CreateSparkSession:
    def __init__(self):
        self.logger = get_logger(__name__)
        self.DB_CONFIG = {
            "host": "host.docker.internal",
            "port": "3306",
            "user": "root",
            "password": "",
            "database": "health_data",
            "table": "health_disparities",
        }

    def new_spark_session(self):
        self.logger.info("Creating Spark session for external (outside K8s) driver...")
        master_url = os.environ.get("SPARK_MASTER", "mi355x")
        driver_host = os.environ.get("SPARK_DRIVER_HOST", "127.0.0.1")
        driver_port = os.environ.get("SPARK_DRIVER_PORT", "7078")
        blockmanager_port = os.environ.get("SPARK_BLOCKMGR_PORT", "7079")
        for what, host in (("database host", self.DB_CONFIG["host"]), ("driver host", driver_host)):
            try:
                self.logger.info(f"Resolved {what} {host} to {socket.gethostbyname(host)}")
            except OSError as e:
                self.logger.warning(f"Could not resolve {what} {host}: {e}")
        self.logger.info(f"Using master={master_url}, driver_host={driver_host}, "
                         f"driver_port={driver_port}, blockManagerPort={blockmanager_port}")
        spark = (SparkSession.builder.appName("ReadMySQLDataOutsideK8s").master(master_url)
                 .config("spark.driver.host", driver_host)
                 .config("spark.driver.bindAddress", "0.0.0.0")
                 .config("spark.driver.port", driver_port)
                 .config("spark.blockManager.port", blockmanager_port)
                 .getOrCreate())
        self.logger.info("Spark session created successfully.")
        spark.sparkContext.setLogLevel("ERROR")
        self.logger.info("Set Spark log level to ERROR to suppress Spark INFO/WARN logs.")
        return spark, self.logger, self.DB_CONFIG
