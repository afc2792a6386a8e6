"""Partitioned JDBC read of the health table (reference: workloads/raw-spark/google_health_SQL.py:9-49).

The ``jdbc:mysql://host:port/<db>`` URL resolves to ``$PTG_JDBC_ROOT/<db>.sqlite`` (written by
``load_csv.py``); the partitioned read keeps Spark's column-partitioning predicates
(partitionColumn=id, lowerBound=1, upperBound=1000000, numPartitions=16) and spreads the 16
partitions over the executor ranks.
"""
import os

import _path  # noqa: F401


class RetrieveDataFromMySQLOutside:
    def __init__(self, logger, DB, spark):  # noqa: N803
        self.DB_CONFIG = DB
        self.spark = spark
        self.logger = logger

    def read_data_from_mysql(self, partitioned=True, show=5):
        host = os.environ.get("DB_HOST", self.DB_CONFIG["host"])
        port = os.environ.get("DB_PORT", self.DB_CONFIG["port"])
        user = os.environ.get("DB_USER", self.DB_CONFIG["user"])
        password = os.environ.get("DB_PASSWORD", self.DB_CONFIG["password"])
        database = os.environ.get("DB_NAME", self.DB_CONFIG["database"])
        table = os.environ.get("DB_TABLE", self.DB_CONFIG["table"])
        self.logger.info(f"Connecting to MySQL database '{database}' on '{host}:{port}'...")
        jdbc_url = f"jdbc:mysql://{host}:{port}/{database}"
        reader = (self.spark.read.format("jdbc").option("url", jdbc_url).option("dbtable", table)
                  .option("user", user).option("password", password).option("driver", "com.mysql.cj.jdbc.Driver"))
        if partitioned:
            reader = (reader.option("partitionColumn", "id").option("lowerBound", "1")
                      .option("upperBound", "1000000").option("numPartitions", "16"))
        df = reader.load()
        self.logger.info("Data loaded successfully.")
        df.printSchema()
        df.show(show)
        return df
