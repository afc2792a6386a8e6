"""Cluster connectivity check with a partitioned JDBC read
(reference: spark_checks/python_checks/spark_workload_to_local_k8s.py:26-146)."""
import os
import sys

import _path  # noqa: F401

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))
from google_health_SQL import RetrieveDataFromMySQLOutside  # noqa: E402
from spark_session import CreateSparkSession  # noqa: E402


def main():
    spark, logger, db = CreateSparkSession().new_spark_session()
    try:
        df = RetrieveDataFromMySQLOutside(logger, db, spark).read_data_from_mysql(partitioned=True, show=50)
        logger.info(f"Rows read: {df.count()} in {df.rdd.getNumPartitions()} JDBC partitions")
    finally:
        spark.stop()
        logger.info("Spark session stopped.")


if __name__ == "__main__":
    main()
