"""PySpark-shaped SQL/DataFrame API on the MI355X executors (``pyspark.sql`` surface used by the
reference's raw-spark workloads)."""
from . import functions, types  # noqa: F401
from .column import Column  # noqa: F401
from .dataframe import DataFrame, GroupedData, Row  # noqa: F401
from .session import SparkContext, SparkSession  # noqa: F401
