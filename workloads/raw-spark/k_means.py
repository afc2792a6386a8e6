"""KMeans clustering of the health table (reference: workloads/raw-spark/k_means.py:9-212).

Pipeline: null filter on measure_name -> StringIndexer(keep) -> OneHotEncoder -> mean imputation of
value/lower_ci/upper_ci -> measure_name one-hot repeated MEASURE_NAME_WEIGHT times (default 5) ->
VectorAssembler(keep) -> KMeans(k=25, seed=1, maxIter=1000); then single-row inference on the
reference's 7 labels (RUN_INFERENCE, default true).  Feature assembly, k-means|| init, Lloyd
iterations and assignment run as HIP kernels on the executor GPUs with RCCL all-reduces.
"""
import os

import _path  # noqa: F401

from pyspark_tf_gke_amd.ml import Pipeline, PipelineModel
from pyspark_tf_gke_amd.ml.clustering import KMeans, KMeansModel
from pyspark_tf_gke_amd.ml.feature import OneHotEncoder, StringIndexer, VectorAssembler
from pyspark_tf_gke_amd.sql.functions import col, isnan, when

INFERENCE_LABELS = ["Able-Bodied", "Asthma", "Avoided Care Due to Cost", "Cancer", "Cardiovascular Diseases",
                    "Child Poverty", "Premature Death"]
INFERENCE_VALUES = [0, 10, 20, 30, 40, 50, 60]


class KMeansWorkload:
    DB_CONFIG = None
    pipeline_model = None
    kmeans_model = None

    def __init__(self):
        self.logger = None

    def k_means(self, input_df, k=25, max_iter=1000):
        self.logger.info("Checking for missing values in 'measure_name'...")
        nulls = input_df.filter(col("measure_name").isNull()).count()
        self.logger.info(f"Column 'measure_name' has {nulls} missing values")
        input_df = input_df.filter(col("measure_name").isNotNull())
        self.logger.info(f"Rows after filtering out missing 'measure_name' values: {input_df.count()}")
        stages = [StringIndexer(inputCol="measure_name", outputCol="measure_name_index", handleInvalid="keep"),
                  OneHotEncoder(inputCol="measure_name_index", outputCol="measure_name_vec")]
        numeric_cols = ["value", "lower_ci", "upper_ci"]
        for c in numeric_cols:
            if c in input_df.columns:
                mean_val = (input_df.select(c).filter(~isnan(col(c)) & col(c).isNotNull())
                            .agg({c: "avg"}).collect()[0][0])
                input_df = input_df.withColumn(c, when(col(c).isNull() | isnan(col(c)), mean_val).otherwise(col(c)))
        try:
            repeats = int(os.environ.get("MEASURE_NAME_WEIGHT", "5"))
        except ValueError:
            repeats = 5
        repeats = max(1, repeats)
        self.logger.info(f"Applying measure_name weight by repeating measure_name_vec {repeats} time(s)")
        stages.append(VectorAssembler(inputCols=["measure_name_vec"] * repeats + numeric_cols, outputCol="features",
                                      handleInvalid="keep"))
        self.logger.info("Applying feature engineering pipeline...")
        pipeline_model = Pipeline(stages=stages).fit(input_df)
        dataset = pipeline_model.transform(input_df).select("features")
        self.logger.info("Training K-Means model...")
        model = KMeans().setK(k).setSeed(1).setMaxIter(max_iter).fit(dataset)
        self.logger.info(f"K-Means trained: {model.summary.numIter} iterations, "
                         f"training cost {model.summary.trainingCost:.6g}")
        save_dir = os.environ.get("MODEL_OUTPUT_DIR")
        if save_dir and os.environ.get("SAVE_MODELS", "false").lower() in ("1", "true", "yes", "y"):
            model.write().overwrite().save(os.path.join(save_dir, "health_kmeans_model"))
            pipeline_model.write().overwrite().save(os.path.join(save_dir, "health_kmeans_pipeline"))
        return pipeline_model, model

    def _get_model_paths(self):
        base_dir = os.environ.get("MODEL_OUTPUT_DIR", "/opt/spark/work-dir/models")
        return os.path.join(base_dir, "health_kmeans_model"), os.path.join(base_dir, "health_kmeans_pipeline")

    def load_models(self):
        model_path, pipeline_path = self._get_model_paths()
        self.logger.info(f"Loading K-Means model from {model_path}")
        self.logger.info(f"Loading Pipeline model from {pipeline_path}")
        return PipelineModel.load(pipeline_path), KMeansModel.load(model_path)

    def infer_single_row(self, spark, entry_str="Able-Bodied", entry_num=0):
        data = [(entry_str, entry_num, entry_num + 7, entry_num + 5)]
        input_df = spark.createDataFrame(data, ["measure_name", "value", "lower_ci", "upper_ci"], _local=True)
        if not KMeansWorkload.pipeline_model or not KMeansWorkload.kmeans_model:
            raise RuntimeError("In-memory models not available. Ensure k_means() has been executed before inference.")
        features_df = KMeansWorkload.pipeline_model.transform(input_df)
        predictions_df = KMeansWorkload.kmeans_model.transform(features_df)
        row = predictions_df.select("prediction").first()
        prediction = int(row["prediction"]) if row is not None else None
        self.logger.info(f"Inference prediction: {prediction}")
        return prediction, predictions_df

    @classmethod
    def main(cls):
        from google_health_SQL import RetrieveDataFromMySQLOutside
        from spark_session import CreateSparkSession

        spark, instance = None, cls()
        try:
            spark, logger, db_conf = CreateSparkSession().new_spark_session()
            cls.DB_CONFIG = db_conf
            instance.logger = logger
            df = RetrieveDataFromMySQLOutside(logger, db_conf, spark).read_data_from_mysql()
            k = int(os.environ.get("KMEANS_K", "25"))
            cls.pipeline_model, cls.kmeans_model = instance.k_means(df, k=k)
            logger.info("Running inference on a single row to verify the model is working correctly...")
            if os.environ.get("RUN_INFERENCE", "true").lower() in ("1", "true", "yes", "y"):
                try:
                    for label, num in zip(INFERENCE_LABELS, INFERENCE_VALUES):
                        instance.infer_single_row(spark, entry_str=label, entry_num=num)
                except Exception as ie:  # noqa: BLE001 - the reference logs and continues (k_means.py:195-196)
                    instance.logger.warning(f"Single-row inference skipped due to error: {ie}")
        except Exception as e:  # noqa: BLE001 - the reference logs the failure (k_means.py:197-198)
            if instance.logger is not None:
                instance.logger.error(f"An error occurred: {e}")
            raise
        finally:
            if spark:
                spark.stop()
                bar = "=" * 80
                for line in (bar, bar, bar, "Spark session stopped.", bar, bar, bar):
                    instance.logger.info(line)


if __name__ == "__main__":
    KMeansWorkload.main()
