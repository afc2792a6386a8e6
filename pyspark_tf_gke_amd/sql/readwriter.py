"""DataFrameReader / DataFrameWriter.

* CSV: native quote-aware tokenizer + Spark-style schema inference (csrc/host/csv.cpp); each rank
  parses only its contiguous range of records (parallel ingest), string columns are
  dictionary-encoded and the dictionaries unified across ranks (spark_workload_to_cloud_k8s.py:48).
* ``format("jdbc")``: the reference reads MySQL over JDBC with
  partitionColumn/lowerBound/upperBound/numPartitions (google_health_SQL.py:26-37).  The runtime
  ships no MySQL; a real SQL source is SQLite (stdlib): ``jdbc:sqlite:<file>``, or a
  ``jdbc:mysql://host:port/<db>`` URL resolved to ``$PTG_JDBC_ROOT/<db>.sqlite`` (written by
  ``workloads/raw-spark/load_csv.py``).  Partitioned reads follow Spark's JDBC column partitioning
  exactly (stride from the bounds; the first partition also takes ``< lower`` and NULLs, the last
  ``>= upper``) and the partitions are read in parallel, round-robin over the executor ranks.  Option
  ``adaptiveBounds=true`` uses the column's real min/max instead (fixes the reference's
  all-rows-in-partition-0 skew).  Without a database file, ``dbtable`` resolves to an
  exported CSV/Parquet file (``url`` = ``file:<dir>`` or option ``path``).
* Parquet (pyarrow for the file format only), text, JSON lines.
* Writer: one ``part-<partition>-<uuid>.parquet`` / ``.csv`` per non-empty partition (a write task;
  partition p lives on rank p % world) + ``_SUCCESS``; modes
  overwrite / append / error / ignore.
"""
from __future__ import annotations

import ctypes
import glob
import json
import os
import shutil
import uuid

import numpy as np
import torch

from .. import _native
from ..parallel import comm
from . import types as T
from .dataframe import DataFrame
from .table import ColumnVector, Table, column_from_python


def unify_dictionary(cv: ColumnVector) -> ColumnVector:
    """Make a string column's dictionary identical on every rank (union in rank order) and remap
    local codes — required before codes can be compared, shuffled or grouped across ranks."""
    if not comm.distributed() or not isinstance(cv.dtype, T.StringType):
        return cv
    merged = comm.union_strings(cv.dictionary or [])  # tensor collectives: hashes, then new strings' bytes
    idx = {s: i for i, s in enumerate(merged)}
    lut = torch.tensor([idx[s] for s in (cv.dictionary or [])] + [-1], dtype=torch.int32, device=cv.device)
    codes = cv.data.long()
    codes = torch.where(codes < 0, torch.full_like(codes, len(cv.dictionary or [])), codes)
    return ColumnVector(lut[codes], cv.dtype, cv.valid, merged)


def _parse_csv_bytes(buf: bytes, header: bool, infer: bool, sep: str, device, schema=None, rank_split=True):
    lib = _native.host_lib()
    n = len(buf)
    cbuf = ctypes.create_string_buffer(buf, n)
    nrows = ctypes.c_long(0)
    ncols = ctypes.c_int(0)
    lib.ptgh_csv_index(cbuf, n, ord(sep), ctypes.byref(nrows), ctypes.byref(ncols), None, 0)
    R, Cn = nrows.value, ncols.value
    starts = np.zeros(max(R, 1), dtype=np.int64)
    lib.ptgh_csv_index(cbuf, n, ord(sep), ctypes.byref(nrows), ctypes.byref(ncols),
                       starts.ctypes.data_as(ctypes.c_void_p), R)

    def spans(st):
        m = len(st)
        fs = np.zeros(m * Cn, dtype=np.int64)
        fl = np.zeros(m * Cn, dtype=np.int32)
        fq = np.zeros(m * Cn, dtype=np.uint8)
        if m:
            lib.ptgh_csv_fields(cbuf, n, st.ctypes.data_as(ctypes.c_void_p), m, Cn, ord(sep),
                                fs.ctypes.data_as(ctypes.c_void_p), fl.ctypes.data_as(ctypes.c_void_p),
                                fq.ctypes.data_as(ctypes.c_void_p))
        return fs, fl, fq

    if header and R:
        hs, hl, hq = spans(starts[:1].copy())
        names = []
        for j in range(Cn):
            raw = buf[hs[j]:hs[j] + max(hl[j], 0)].decode("utf-8", "replace")
            names.append(raw.replace('""', '"') if hq[j] else raw)
        data_starts = starts[1:R]
    else:
        names = [f"_c{j}" for j in range(Cn)]
        data_starts = starts[:R]
    if isinstance(schema, T.StructType):
        names = schema.names
    total = len(data_starts)
    if rank_split and comm.distributed():
        w, r = comm.world_size(), comm.rank()
        data_starts = data_starts[total * r // w: total * (r + 1) // w]
    st = np.ascontiguousarray(data_starts)
    m = len(st)
    fs, fl, fq = spans(st)
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    types = []
    for j in range(Cn):
        if isinstance(schema, T.StructType):
            dt = schema.fields[j].dataType
            types.append({T.IntegerType: 0, T.LongType: 1, T.DoubleType: 2, T.FloatType: 2, T.BooleanType: 3}.get(type(dt), 4))
            continue
        if not infer:
            types.append(4)
            continue
        tcode = ctypes.c_int(5)
        lib.ptgh_csv_infer(cbuf, p(fs), p(fl), p(fq), m, Cn, j, ctypes.byref(tcode))
        types.append(tcode.value)
    if infer and comm.distributed() and not isinstance(schema, T.StructType):
        allt = [row.tolist() for row in comm.all_gather_v(torch.tensor([types], dtype=torch.int64))[0:]]
        allt = [r[0] for r in allt]
        merged = []
        for j in range(Cn):
            ts = [t[j] for t in allt if t[j] != 5]
            if not ts:
                merged.append(5)
            elif all(t <= 2 for t in ts):
                merged.append(max(ts))
            elif len(set(ts)) == 1:
                merged.append(ts[0])
            else:
                merged.append(4)
        types = merged
    cols = {}
    for j, name in enumerate(names):
        t = types[j]
        if t in (0, 1):
            out = np.zeros(m, dtype=np.int64)
            valid = np.zeros(m, dtype=np.uint8)
            lib.ptgh_csv_parse(cbuf, p(fs), p(fl), m, Cn, j, 0, p(out), p(valid))
            data = torch.from_numpy(out.astype(np.int32) if t == 0 else out)
            dt = T.IntegerType() if t == 0 else T.LongType()
        elif t == 2:
            out = np.zeros(m, dtype=np.float64)
            valid = np.zeros(m, dtype=np.uint8)
            lib.ptgh_csv_parse(cbuf, p(fs), p(fl), m, Cn, j, 1, p(out), p(valid))
            data, dt = torch.from_numpy(out), T.DoubleType()
        elif t == 3:
            out = np.zeros(m, dtype=np.uint8)
            valid = np.zeros(m, dtype=np.uint8)
            lib.ptgh_csv_parse(cbuf, p(fs), p(fl), m, Cn, j, 2, p(out), p(valid))
            data, dt = torch.from_numpy(out.astype(np.bool_)), T.BooleanType()
        else:
            codes = np.zeros(m, dtype=np.int32)
            cap = int(np.maximum(fl[j::Cn], 0).sum()) + 16 if m else 16
            dbytes = ctypes.create_string_buffer(cap)
            doff = np.zeros(m + 2, dtype=np.int64)
            nd, used = ctypes.c_long(0), ctypes.c_long(0)
            rc = lib.ptgh_csv_dict_encode(cbuf, p(fs), p(fl), p(fq), m, Cn, j, p(codes), dbytes, cap, p(doff), m + 1,
                                          ctypes.byref(nd), ctypes.byref(used))
            if rc != 0:
                raise RuntimeError(f"csv dictionary encoding failed ({rc})")
            raw = dbytes.raw[: used.value]
            dictionary = [raw[doff[i]:doff[i + 1]].decode("utf-8", "replace") for i in range(nd.value)]
            cv = ColumnVector(torch.from_numpy(codes).to(device), T.StringType(), None, dictionary)
            cols[name] = unify_dictionary(cv)
            continue
        v = torch.from_numpy(valid)
        cols[name] = ColumnVector(data.to(device), dt, None if bool(valid.all()) else v.to(device))
    return Table(cols, m, device)


class DataFrameReader:
    def __init__(self, session):
        self._s = session
        self._fmt = "parquet"
        self._opts: dict = {}
        self._schema = None

    def format(self, source: str):
        self._fmt = source.lower()
        return self

    def option(self, key, value):
        self._opts[key] = value
        return self

    def options(self, **kw):
        self._opts.update(kw)
        return self

    def schema(self, schema):
        self._schema = schema
        return self

    def load(self, path=None, format=None, **kw):  # noqa: A002
        fmt = (format or self._fmt).lower()
        self._opts.update(kw)
        if fmt == "csv":
            return self.csv(path or self._opts.get("path"))
        if fmt == "parquet":
            return self.parquet(path or self._opts.get("path"))
        if fmt in ("json", "text"):
            return getattr(self, fmt)(path or self._opts.get("path"))
        if fmt == "jdbc":
            return self._jdbc()
        raise ValueError(f"unsupported format {fmt}")

    @staticmethod
    def _truthy(v):
        return str(v).lower() in ("1", "true", "yes", "y")

    def csv(self, path, schema=None, sep=None, header=None, inferSchema=None, **kw):  # noqa: N803
        header = self._truthy(header if header is not None else self._opts.get("header", False))
        infer = self._truthy(inferSchema if inferSchema is not None else self._opts.get("inferSchema", False))
        sep = sep or self._opts.get("sep", self._opts.get("delimiter", ","))
        schema = schema or self._schema
        paths = _expand(path)
        tables = []
        for pth in paths:
            with open(pth, "rb") as fh:
                buf = fh.read()
            tables.append(_parse_csv_bytes(buf, header, infer, sep, self._s.device, schema))
        return DataFrame(Table.concat(tables), self._s)

    def text(self, path, wholetext=False, lineSep=None):  # noqa: N803
        paths = _expand(path)
        lines = []
        for pth in paths:
            with open(pth, "r", encoding="utf-8", errors="replace") as fh:
                lines += [fh.read()] if wholetext else fh.read().splitlines()
        if comm.distributed():
            w, r = comm.world_size(), comm.rank()
            lines = lines[len(lines) * r // w: len(lines) * (r + 1) // w]
        cv = unify_dictionary(column_from_python(lines, T.StringType(), self._s.device))
        return DataFrame(Table({"value": cv}, len(lines), self._s.device), self._s)

    def json(self, path, **kw):
        rows = []
        for pth in _expand(path):
            with open(pth) as fh:
                rows += [json.loads(l) for l in fh if l.strip()]
        return self._s.createDataFrame(rows)

    def parquet(self, *paths):
        import pyarrow.parquet as pq

        files = []
        for p in paths:
            files += _expand(p, exts=(".parquet",))
        files = sorted(files)
        w, r = comm.world_size(), comm.rank()
        mine = [f for i, f in enumerate(files) if i % w == r]
        tables = [_arrow_to_table(pq.read_table(f), self._s.device) for f in mine]
        if not tables and files:
            empty = pq.read_table(files[0]).slice(0, 0)
            tables = [_arrow_to_table(empty, self._s.device)]
        t = Table.concat(tables)
        t = Table({n: unify_dictionary(c) for n, c in t.columns.items()}, t.num_rows, t.device)
        return DataFrame(t, self._s)

    def jdbc(self, url, table, column=None, lowerBound=None, upperBound=None, numPartitions=None,  # noqa: N803
             predicates=None, properties=None):
        self._opts.update({"url": url, "dbtable": table})
        if column:
            self._opts.update({"partitionColumn": column, "lowerBound": lowerBound, "upperBound": upperBound,
                               "numPartitions": numPartitions})
        return self._jdbc()

    def _jdbc(self):
        url = str(self._opts.get("url", ""))
        table = self._opts.get("dbtable")
        db = _sqlite_for_url(url)
        if db is not None:
            return self._jdbc_sqlite(db, table)
        base = self._opts.get("path") or os.environ.get("PTG_JDBC_ROOT")
        if url.startswith("file:"):
            base = url[5:]
        if not base:
            raise RuntimeError(
                f"JDBC source {url!r}: no database engine in this runtime. Point the source at exported table "
                "files with option('path', <dir or file>) or PTG_JDBC_ROOT (looked up as <dir>/<dbtable>.csv|.parquet).")
        cand = [base] if os.path.isfile(base) else [os.path.join(base, f"{table}.parquet"), os.path.join(base, f"{table}.csv")]
        src = next((c for c in cand if os.path.exists(c)), None)
        if src is None:
            raise FileNotFoundError(f"JDBC table {table!r} not found under {base}")
        r = DataFrameReader(self._s)
        df = r.parquet(src) if src.endswith(".parquet") else r.csv(src, header=True, inferSchema=True)
        pc = self._opts.get("partitionColumn")
        if pc and "id" not in [c.lower() for c in df.columns] and pc == "id":
            # MySQL table of load_csv.py has an AUTO_INCREMENT id (load_csv.py:49-63)
            from .functions import monotonically_increasing_id

            df = df.withColumn("id", monotonically_increasing_id() + 1)
        if pc:
            df._num_partitions = int(self._opts.get("numPartitions") or df._num_partitions)
        return df


    def _jdbc_sqlite(self, path, table):
        import sqlite3

        from .session import SparkSession  # noqa: F401  (type context)

        con = sqlite3.connect(f"file:{path}?mode=ro", uri=True)
        try:
            src = table if str(table).lstrip().startswith("(") else f'"{table}"'
            cur = con.execute(f"SELECT * FROM {src} LIMIT 0")
            names = [d[0] for d in cur.description]
            decl = {}
            if not str(table).lstrip().startswith("("):
                decl = {r[1]: r[2] for r in con.execute(f'PRAGMA table_info("{table}")')}
            types = [T.from_sql_decl(decl.get(n, "")) for n in names]
            pc = self._opts.get("partitionColumn")
            w, r = comm.world_size(), comm.rank()
            if pc:
                n = max(1, int(self._opts.get("numPartitions") or 1))
                lo, hi = int(self._opts.get("lowerBound")), int(self._opts.get("upperBound"))
                if self._truthy(self._opts.get("adaptiveBounds", False)):
                    mn, mx = con.execute(f'SELECT MIN("{pc}"), MAX("{pc}") FROM {src}').fetchone()
                    if mn is not None:
                        lo, hi = int(mn), int(mx) + 1
                wheres = jdbc_partition_predicates(pc, lo, hi, n)
                mine = [wh for i, wh in enumerate(wheres) if i % w == r]
            else:
                n = 1
                mine = ["1=1"] if r == 0 else []
            rows = []
            for wh in mine:
                rows += con.execute(f"SELECT * FROM {src} WHERE {wh}").fetchall()
        finally:
            con.close()
        schema = T.StructType([T.StructField(nm, tp) for nm, tp in zip(names, types)])
        df = self._s.createDataFrame(rows, schema, _local=True)
        t = df._t
        df = DataFrame(Table({nm: unify_dictionary(c) for nm, c in t.columns.items()}, t.num_rows, t.device), self._s)
        df._num_partitions = n
        return df


def jdbc_partition_predicates(column: str, lower: int, upper: int, n: int) -> list:
    """WHERE clauses of Spark's JDBC column partitioning (JDBCRelation.columnPartition)."""
    if n <= 1 or upper - lower < 1:
        return ["1=1"]
    n = min(n, upper - lower)
    stride = upper // n - lower // n
    cur, out = lower, []
    for i in range(n):
        lb = f'"{column}" >= {cur}' if i != 0 else None
        cur += stride
        ub = f'"{column}" < {cur}' if i != n - 1 else None
        if ub is None:
            out.append(lb)
        elif lb is None:
            out.append(f'{ub} OR "{column}" IS NULL')
        else:
            out.append(f"{lb} AND {ub}")
    return out


def _sqlite_for_url(url: str):
    """jdbc:sqlite:<file> -> file; jdbc:mysql://host:port/<db> -> $PTG_JDBC_ROOT/<db>.sqlite if present."""
    if url.startswith("jdbc:sqlite:"):
        return url[len("jdbc:sqlite:"):]
    if url.startswith("jdbc:mysql://"):
        rest = url[len("jdbc:mysql://"):]
        dbname = rest.split("/", 1)[1].split("?", 1)[0] if "/" in rest else ""
        root = os.environ.get("PTG_JDBC_ROOT")
        if root and dbname:
            cand = os.path.join(root, f"{dbname}.sqlite")
            if os.path.exists(cand):
                return cand
    return None


def _expand(path, exts=None):
    if isinstance(path, (list, tuple)):
        out = []
        for p in path:
            out += _expand(p, exts)
        return out
    path = str(path)
    if path.startswith("file://"):
        path = path[7:]
    if os.path.isdir(path):
        fs = sorted(f for f in glob.glob(os.path.join(path, "*")) if os.path.isfile(f)
                    and not os.path.basename(f).startswith(("_", ".")))
        return [f for f in fs if not exts or f.endswith(exts)]
    hits = sorted(glob.glob(path))
    if not hits:
        raise FileNotFoundError(path)
    return hits


def _arrow_to_table(at, device) -> Table:
    import pyarrow as pa

    cols = {}
    for name in at.column_names:
        arr = at.column(name).combine_chunks()
        t = arr.type
        valid = None
        if arr.null_count:
            valid = torch.from_numpy(np.asarray(arr.is_valid()).astype(np.uint8)).to(device)
        if pa.types.is_string(t) or pa.types.is_large_string(t) or pa.types.is_dictionary(t):
            enc = arr.dictionary_encode() if not pa.types.is_dictionary(t) else arr
            codes = np.asarray(enc.indices.fill_null(-1)).astype(np.int32)
            cols[name] = ColumnVector(torch.from_numpy(codes).to(device), T.StringType(), None,
                                      [str(s) for s in enc.dictionary.to_pylist()])
        elif pa.types.is_list(t) or pa.types.is_fixed_size_list(t):
            mat = np.stack([np.asarray(v, dtype=np.float32) for v in arr.to_pylist()]) if len(arr) else np.zeros((0, 0), np.float32)
            cols[name] = ColumnVector(torch.from_numpy(mat).to(device), T.VectorUDT())
        elif pa.types.is_boolean(t):
            cols[name] = ColumnVector(torch.from_numpy(np.asarray(arr.fill_null(False)).astype(np.bool_)).to(device),
                                      T.BooleanType(), valid)
        else:
            np_arr = np.asarray(arr.fill_null(0) if arr.null_count else arr)
            if not np_arr.flags.writeable:  # arrow buffers are read-only; torch needs a writable array
                np_arr = np_arr.copy()
            tt = torch.from_numpy(np.ascontiguousarray(np_arr))
            if tt.dtype == torch.int32:
                dt = T.IntegerType()
            elif tt.dtype == torch.int64:
                dt = T.LongType()
            elif tt.dtype == torch.float32:
                dt = T.FloatType()
            else:
                tt, dt = tt.double(), T.DoubleType()
            cols[name] = ColumnVector(tt.to(device), dt, valid)
    return Table(cols, at.num_rows, device)


def table_to_arrow(t: Table):
    import pyarrow as pa

    arrays, names = [], []
    for name, cv in t.columns.items():
        valid = cv.valid_bool().cpu().numpy()
        if isinstance(cv.dtype, T.StringType):
            codes = cv.data.cpu().numpy()
            ok = valid & (codes >= 0)
            d = pa.array(cv.dictionary or [], type=pa.string())
            idx = pa.array(np.where(ok, codes, 0).astype(np.int32), mask=~ok)
            arrays.append(pa.DictionaryArray.from_arrays(idx, d).cast(pa.string()))
        elif isinstance(cv.dtype, T.VectorUDT):
            mat = cv.data.cpu().numpy()
            arrays.append(pa.array([row for row in mat], type=pa.list_(pa.float32())))
        else:
            arr = cv.data.cpu().numpy()
            arrays.append(pa.array(arr, mask=~valid if not valid.all() else None))
        names.append(name)
    return pa.table(arrays, names=names)


class DataFrameWriter:
    def __init__(self, df: DataFrame):
        self._df = df
        self._mode = "errorifexists"
        self._fmt = "parquet"
        self._opts: dict = {}
        self._partition_by = None

    def mode(self, m: str):
        self._mode = m.lower()
        return self

    def format(self, f: str):
        self._fmt = f.lower()
        return self

    def option(self, k, v):
        self._opts[k] = v
        return self

    def partitionBy(self, *cols):  # noqa: N802
        self._partition_by = cols
        return self

    def _prepare(self, path) -> bool:
        exists = os.path.exists(path)
        if comm.rank() == 0:
            if exists and self._mode in ("error", "errorifexists", "default"):
                raise FileExistsError(f"path {path} already exists")
            if exists and self._mode == "overwrite":
                shutil.rmtree(path) if os.path.isdir(path) else os.remove(path)
            os.makedirs(path, exist_ok=True)
        comm.barrier()
        return not (exists and self._mode == "ignore")

    def _finish(self, path):
        comm.barrier()
        if comm.rank() == 0:
            open(os.path.join(path, "_SUCCESS"), "w").close()

    def save(self, path=None):
        return getattr(self, self._fmt)(path or self._opts.get("path"))

    def _tasks(self):
        """(global partition index, Table) of this rank's non-empty partitions - one write task and
        one output file per partition, as Spark writes them (partition p lives on rank p % world).
        A rank whose partitions are all empty writes one empty file when it is rank 0 (the schema)."""
        df = self._df
        world, rank = comm.world_size(), comm.rank()
        parts = df.local_partitions()
        out = [(rank + i * world, t) for i, t in enumerate(parts) if t.num_rows]
        if not out and rank == 0:
            out = [(0, df._t)]
        return out

    def parquet(self, path, mode=None, compression="snappy"):
        import pyarrow.parquet as pq

        if mode:
            self._mode = mode
        if not self._prepare(path):
            return
        for p, t in self._tasks():
            pq.write_table(table_to_arrow(t), os.path.join(path, f"part-{p:05d}-{uuid.uuid4().hex[:12]}.{compression}.parquet"),
                           compression=compression)
        self._finish(path)

    def csv(self, path, mode=None, header=None):
        if mode:
            self._mode = mode
        if not self._prepare(path):
            return
        hdr = DataFrameReader._truthy(header if header is not None else self._opts.get("header", False))
        import csv as pycsv

        for p, t in self._tasks():
            with open(os.path.join(path, f"part-{p:05d}-{uuid.uuid4().hex[:12]}.csv"), "w", newline="") as fh:
                w = pycsv.writer(fh)
                if hdr:
                    w.writerow(self._df.columns)
                for row in t.rows():
                    w.writerow(["" if v is None else v for v in row])
        self._finish(path)

    def json(self, path, mode=None):
        if mode:
            self._mode = mode
        if not self._prepare(path):
            return
        names = self._df.columns
        for p, t in self._tasks():
            with open(os.path.join(path, f"part-{p:05d}-{uuid.uuid4().hex[:12]}.json"), "w") as fh:
                for row in t.rows():
                    fh.write(json.dumps({k: (list(map(float, v)) if hasattr(v, "toArray") else v)
                                         for k, v in zip(names, row)}) + "\n")
        self._finish(path)
