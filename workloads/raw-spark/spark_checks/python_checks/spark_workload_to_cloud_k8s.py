"""CSV -> KMeans(k=5) -> silhouette -> model save (reference:
spark_checks/python_checks/spark_workload_to_cloud_k8s.py:25-169).

The reference reads ``gs://<GCP_PROJECT_ID>-datasets/health.csv``.  Object storage is replaced by a
dataset directory: ``$PTG_DATASETS_DIR/health.csv`` (or ``$HEALTH_CSV``); models are written under
``$MODEL_OUTPUT_DIR`` (default: current directory) in Spark-ML layout (metadata JSON + Parquet data).
"""
import os

import _path  # noqa: F401

from pyspark_tf_gke_amd.ml import Pipeline
from pyspark_tf_gke_amd.ml.clustering import KMeans
from pyspark_tf_gke_amd.ml.evaluation import ClusteringEvaluator
from pyspark_tf_gke_amd.ml.feature import OneHotEncoder, StringIndexer, VectorAssembler
from pyspark_tf_gke_amd.sql import SparkSession
from pyspark_tf_gke_amd.sql.functions import col, isnan, when


def dataset_path():
    if os.environ.get("HEALTH_CSV"):
        return os.environ["HEALTH_CSV"]
    root = os.environ.get("PTG_DATASETS_DIR")
    if not root and os.environ.get("GCP_PROJECT_ID"):
        root = f"{os.environ['GCP_PROJECT_ID']}-datasets"
    if not root:
        raise ValueError("set PTG_DATASETS_DIR (or HEALTH_CSV) to the directory holding health.csv")
    return os.path.join(root, "health.csv")


def main():
    spark = (SparkSession.builder.appName("HealthKMeansClassification")
             .config("spark.kubernetes.container.image", "spark:latest")
             .config("spark.kubernetes.namespace", "default")
             .getOrCreate())
    bar = "=" * 107
    try:
        print("Loading health dataset...")
        health_df = spark.read.csv(dataset_path(), header=True, inferSchema=True)
        print("Dataset Schema:")
        health_df.printSchema()
        print("Sample Data:")
        health_df.show(5)
        print(f"Total number of rows: {health_df.count()}")
        print("Checking for missing values in 'measure_name'...")
        print(f"Column 'measure_name' has {health_df.filter(col('measure_name').isNull()).count()} missing values")
        health_df = health_df.filter(col("measure_name").isNotNull())
        print(f"Rows after filtering out missing 'measure_name' values: {health_df.count()}")
        stages = [StringIndexer(inputCol="measure_name", outputCol="measure_name_index", handleInvalid="keep"),
                  OneHotEncoder(inputCol="measure_name_index", outputCol="measure_name_vec")]
        numeric_cols = ["value", "lower_ci", "upper_ci"]
        for c in numeric_cols:
            if c in health_df.columns:
                mean_val = (health_df.select(c).filter(~isnan(col(c)) & col(c).isNotNull())
                            .agg({c: "avg"}).collect()[0][0])
                health_df = health_df.withColumn(c, when(col(c).isNull() | isnan(col(c)), mean_val).otherwise(col(c)))
        stages.append(VectorAssembler(inputCols=["measure_name_vec"] + numeric_cols, outputCol="features",
                                      handleInvalid="keep"))
        print("Applying feature engineering pipeline...")
        pipeline_model = Pipeline(stages=stages).fit(health_df)
        dataset = pipeline_model.transform(health_df).select("features")
        print("Training K-Means model...")
        model = KMeans().setK(5).setSeed(1).fit(dataset)
        predictions = model.transform(dataset)
        print("Sample Predictions (Cluster Assignments):")
        predictions.select("features", "prediction").show(5)
        print("Cluster Centers:")
        for center in model.clusterCenters():
            print(center)
        silhouette = ClusteringEvaluator().evaluate(predictions)
        print(f"Silhouette with squared Euclidean distance = {silhouette}")
        out = os.environ.get("MODEL_OUTPUT_DIR", ".")
        model_path = os.path.join(out, "health_kmeans_model")
        pipeline_path = os.path.join(out, "health_kmeans_pipeline")
        print(f"Saving K-Means model to {model_path}")
        model.write().overwrite().save(model_path)
        print(f"Saving K-Means pipeline to {pipeline_path}")
        pipeline_model.write().overwrite().save(pipeline_path)
    finally:
        for line in (bar, bar, bar, "Stopping Spark session...", bar, bar, bar):
            print(line)
        spark.stop()


if __name__ == "__main__":
    main()
