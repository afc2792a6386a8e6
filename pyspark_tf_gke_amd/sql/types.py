"""Spark SQL data types (the subset the reference's DataFrames carry: health.csv columns are
strings, integers/longs and doubles; ML adds vectors)."""
from __future__ import annotations

import datetime

import torch


class DataType:
    simple = "unknown"
    torch_dtype = None

    def simpleString(self):  # noqa: N802 (pyspark naming)
        return self.simple

    def typeName(self):  # noqa: N802
        return self.simple

    def __repr__(self):
        return type(self).__name__ + "()"

    def __eq__(self, other):
        return type(self) is type(other)

    def __hash__(self):
        return hash(type(self).__name__)


class StringType(DataType):
    simple = "string"
    torch_dtype = torch.int32  # dictionary codes


class IntegerType(DataType):
    simple = "int"
    torch_dtype = torch.int32


class LongType(DataType):
    simple = "bigint"
    torch_dtype = torch.int64


class DoubleType(DataType):
    simple = "double"
    torch_dtype = torch.float64


class FloatType(DataType):
    simple = "float"
    torch_dtype = torch.float32


class BooleanType(DataType):
    simple = "boolean"
    torch_dtype = torch.bool


class TimestampType(DataType):
    """Microseconds since the Unix epoch (UTC), int64 on device (Spark's internal representation)."""
    simple = "timestamp"
    torch_dtype = torch.int64


_EPOCH = datetime.datetime(1970, 1, 1)


def to_micros(v):
    """datetime / ISO string ('YYYY-MM-DD HH:MM:SS[.ffffff]') / number -> epoch microseconds."""
    if v is None:
        return None
    if isinstance(v, (int, float)):
        return int(v)
    if isinstance(v, str):
        v = datetime.datetime.fromisoformat(v.strip())
    if isinstance(v, datetime.datetime):
        if v.tzinfo is not None:
            v = v.astimezone(datetime.timezone.utc).replace(tzinfo=None)
        d = v - _EPOCH
        return (d.days * 86400 + d.seconds) * 1_000_000 + d.microseconds
    raise TypeError(f"cannot convert {v!r} to a timestamp")


def micros_to_datetime(us: int) -> datetime.datetime:
    return _EPOCH + datetime.timedelta(microseconds=int(us))


class VectorUDT(DataType):
    simple = "vector"
    torch_dtype = torch.float32


class StructField:
    def __init__(self, name: str, dataType: DataType, nullable: bool = True):  # noqa: N803
        self.name, self.dataType, self.nullable = name, dataType, nullable

    def __repr__(self):
        return f"StructField('{self.name}', {self.dataType!r}, {self.nullable})"


class StructType:
    def __init__(self, fields=None):
        self.fields = list(fields or [])

    def add(self, name, dataType, nullable=True):  # noqa: N803
        self.fields.append(StructField(name, dataType, nullable))
        return self

    @property
    def names(self):
        return [f.name for f in self.fields]

    def __iter__(self):
        return iter(self.fields)

    def __len__(self):
        return len(self.fields)

    def __getitem__(self, k):
        if isinstance(k, str):
            for f in self.fields:
                if f.name == k:
                    return f
            raise KeyError(k)
        return self.fields[k]

    def simpleString(self):  # noqa: N802
        return "struct<" + ",".join(f"{f.name}:{f.dataType.simple}" for f in self.fields) + ">"

    def treeString(self) -> str:  # noqa: N802
        lines = ["root"]
        for f in self.fields:
            lines.append(f" |-- {f.name}: {f.dataType.simple} (nullable = {str(f.nullable).lower()})")
        return "\n".join(lines) + "\n"

    def __repr__(self):
        return f"StructType({self.fields!r})"


NUMERIC = (IntegerType, LongType, DoubleType, FloatType, BooleanType)


def from_sql_decl(decl: str) -> DataType:
    """SQL column declaration -> Spark type, following Spark's JDBC type mapping
    (INT -> int, BIGINT -> bigint, FLOAT/REAL -> float, DOUBLE -> double, DECIMAL -> double here,
    VARCHAR/TEXT -> string, TIMESTAMP/DATETIME -> timestamp, BOOLEAN -> boolean)."""
    d = (decl or "").upper()
    if "BIGINT" in d:
        return LongType()
    if "INT" in d:
        return IntegerType()
    if "DOUBLE" in d or "DEC" in d or "NUMERIC" in d:
        return DoubleType()
    if "FLOAT" in d or "REAL" in d:
        return FloatType()
    if "BOOL" in d:
        return BooleanType()
    if "TIMESTAMP" in d or "DATETIME" in d:
        return TimestampType()
    return StringType()


def from_torch(dt: torch.dtype) -> DataType:
    return {torch.int32: IntegerType(), torch.int64: LongType(), torch.float64: DoubleType(),
            torch.float32: FloatType(), torch.bool: BooleanType(), torch.uint8: BooleanType()}[dt]
