"""In-cluster (driver-on-a-rank) non-partitioned JDBC read with show(50)
(reference: workloads/raw-spark/pod_google_health_SQL.py:7-140)."""
import os

import _path  # noqa: F401

from google_health_SQL import RetrieveDataFromMySQLOutside
from spark_session import CreateSparkSession


def main():
    os.environ.setdefault("SPARK_DRIVER_HOST", "127.0.0.1")
    spark, logger, db = CreateSparkSession().new_spark_session()
    try:
        df = RetrieveDataFromMySQLOutside(logger, db, spark).read_data_from_mysql(partitioned=False, show=50)
        logger.info(f"Rows read: {df.count()}")
    finally:
        spark.stop()
        logger.info("Spark session stopped.")


if __name__ == "__main__":
    main()
