"""Engine smoke check (reference: spark_checks/python_checks/spark_installation_check.py:12-46):
``local[2]`` session with 2 shuffle partitions, a 3-row DataFrame, show, filter Age > 30."""
import _path  # noqa: F401

from pyspark_tf_gke_amd.sql import SparkSession

spark = None
try:
    spark = (SparkSession.builder.appName("Spark Workloads")
             .config("spark.sql.shuffle.partitions", "2")
             .config("spark.default.parallelism", "2")
             .config("spark.sql.streaming.forceDeleteTempCheckpointDir", "True")
             .master("local[2]")
             .getOrCreate())
    print(f"Spark version: {spark.version}")
    print(f"Application ID: {spark.sparkContext.applicationId}")
    df = spark.createDataFrame([("Alice", 34), ("Bob", 45), ("Charlie", 29)], ["Name", "Age"])
    print("Sample DataFrame:")
    df.show()
    print("DataFrame with age > 30:")
    df.filter(df.Age > 30).show()
finally:
    if spark is not None:
        print("Stopping Spark session...")
        spark.stop()
