"""DataFrame / ML kernels on the MI355X vs the host (CPU) executor path on identical data."""
import math
import os

import numpy as np
import pytest
import torch

from pyspark_tf_gke_amd.ops import df as D

pytestmark = pytest.mark.gpu

HEALTH = os.path.join(os.path.dirname(__file__), "data", "health.csv")


@pytest.fixture(scope="module")
def spark_gpu(hip_built):
    from pyspark_tf_gke_amd.sql import SparkSession

    s = SparkSession.builder.master("local[1]").config("spark.ptg.device", "cuda").getOrCreate()
    yield s
    s.stop()


def _host(fn):
    from pyspark_tf_gke_amd.sql.session import SparkSession

    s = SparkSession("host", "local[2]", {})
    return fn(s)


def test_compact_and_gather(hip_built):
    n = 1_000_003
    m = (torch.rand(n) < 0.3).to(torch.uint8)
    idx = D.compact(m.cuda())
    ref = torch.nonzero(m).view(-1)
    assert torch.equal(idx.cpu(), ref)
    x = torch.randn(n, 3)
    g = D.gather_rows(x.cuda(), idx)
    assert torch.equal(g.cpu(), x[ref])


def test_reduce_stats(hip_built):
    x = torch.randn(100_000, dtype=torch.float64)
    x[::7] = math.nan
    valid = (torch.rand(100_000) > 0.1).to(torch.uint8)
    g = D.reduce_stats(x.cuda(), valid.cuda())
    h = D.reduce_stats(x, valid)
    assert np.allclose(g, h, rtol=1e-9, equal_nan=True)


@pytest.mark.parametrize("nkeys", [7, 5000, 300_000])
def test_hash_agg_matches_host(hip_built, nkeys):
    n = 2_000_000
    k, v = D.fill_synthetic_kv(n, nkeys, "cpu")
    kg, rg, og = D.hash_agg(k.cuda(), [v.cuda()], [None], True)
    kh, rh, oh = D.hash_agg(k, [v], [None], True)
    order = torch.argsort(kg.cpu())
    assert torch.equal(kg.cpu()[order], kh)
    assert torch.allclose(rg.cpu()[order], rh)
    assert torch.allclose(og[0][0].cpu()[order], oh[0][0], rtol=1e-9)
    assert torch.allclose(og[0][2].cpu()[order], oh[0][2])
    assert torch.allclose(og[0][3].cpu()[order], oh[0][3])


def _sorted_agg(k, r, o):
    order = torch.argsort(k.cpu())
    return k.cpu()[order], r.cpu()[order], [tuple(x.cpu()[order] for x in q) for q in o]


def _assert_agg_equal(got, want, minmax):
    kg, rg, og = _sorted_agg(*got)
    kh, rh, oh = _sorted_agg(*want)
    assert torch.equal(kg, kh)
    assert torch.equal(rg, rh)
    for a, b in zip(og, oh):
        assert torch.allclose(a[0], b[0], rtol=1e-9, atol=1e-9)  # sum
        assert torch.equal(a[1], b[1])  # non-null count
        if minmax:
            assert torch.equal(a[2], b[2]) and torch.equal(a[3], b[3])


@pytest.mark.parametrize("n,nkeys,nv,minmax", [(4_000_000, 1_000_000, 1, False), (8_388_608, 1_000_000, 1, False),
                                               (5_000_000, 3_000, 1, False), (3_000_000, 200_000, 0, False),
                                               (3_000_000, 200_000, 3, True), (700_000, 650_000, 4, True)])
def test_radix_agg_matches_host(hip_built, n, nkeys, nv, minmax):
    """Recursive radix aggregation vs the host path: value columns of mixed types with nulls and
    NaNs, count-only (nv=0), min/max, and very sparse partitions (3,000 keys)."""
    k, v = D.fill_synthetic_kv(n, nkeys, "cuda")
    g = torch.Generator().manual_seed(n + nv)
    cols, valids = [], []
    for j in range(nv):
        if j == 0:
            x = v.clone()
        elif j == 1:
            x = torch.randint(-1000, 1000, (n,), generator=g, dtype=torch.int32).cuda()
        else:
            x = torch.randn(n, generator=g).cuda()
            x[::97] = math.nan
        cols.append(x)
        valids.append((torch.rand(n, generator=g) > 0.2).to(torch.uint8).cuda() if j % 2 == 1 else None)
    got = D.hash_agg_radix(k, cols, valids, minmax)
    want = D.hash_agg(k.cpu(), [c.cpu() for c in cols], [None if x is None else x.cpu() for x in valids], minmax)
    _assert_agg_equal(got, want, minmax)


@pytest.mark.parametrize("lo,span,nv,minmax", [(0, 1_000_000, 1, False), (-5_000_000_000, 1 << 20, 2, False),
                                                (123, 4_000, 0, False), (7, 300_000, 2, False),
                                                (0, 1_000_000, 1, True), (11, 200_000, 4, True),
                                                (-7, 500_000, 3, False)])
def test_range_agg_matches_host(hip_built, lo, span, nv, minmax):
    """Dense small-range keys take the one-level range partition + direct-indexed LDS aggregation
    (range_*_k): sums / non-null counts / min / max with NaN values and validity masks, 0-4 value
    columns, negative keys, and a span of exactly 2^20 whose extremes the sample misses (the window
    is re-planned from the count pass's exact range).  Checked against the host path."""
    n = 6_000_000
    g = torch.Generator().manual_seed(span + nv)
    k = torch.randint(0, span, (n,), generator=g) + lo
    k[17], k[n - 5] = lo, lo + span - 1
    cols, valids = [], []
    for j in range(nv):
        if j == 0:
            x = torch.rand(n, generator=g, dtype=torch.float64)
            x[::101] = math.nan
            vd = None
        else:
            x = torch.randint(-1000, 1000, (n,), generator=g, dtype=torch.int32)
            vd = (torch.rand(n, generator=g) > 0.3).to(torch.uint8)
        cols.append(x)
        valids.append(vd)
    ws = {}
    got = D.hash_agg_radix(k.cuda(), [c.cuda() for c in cols], [None if x is None else x.cuda() for x in valids],
                           minmax, ws=ws)
    assert "rprow" in ws, "range path not taken"
    want = D.hash_agg(k, cols, valids, minmax)
    _assert_agg_equal(got, want, minmax)


@pytest.mark.parametrize("lo,span,nv", [(0, 1 << 21, 1), (-3_000_000_000, 5_000_000, 2), (77, 20_000_000, 0),
                                         (5, 9_000_000, 1)])
def test_range2_agg_matches_host(hip_built, lo, span, nv):
    """Dense keys spanning 2^20..2^28 values take the two-level range path (range2_*: coarse 256-way
    pass with u32 window offsets, fine 256-way pass per coarse partition, direct-indexed LDS
    aggregation per fine window): sums / non-null counts with NaNs and validity masks, 0-2 value
    columns, negative keys, sparse coverage (20M keys over 6M rows).  Checked against the host path."""
    n = 6_000_000
    g = torch.Generator().manual_seed(span + nv + 1)
    k = torch.randint(0, span, (n,), generator=g) + lo
    k[3], k[n - 9] = lo, lo + span - 1
    cols, valids = [], []
    for j in range(nv):
        if j == 0:
            x = torch.rand(n, generator=g, dtype=torch.float64)
            x[::89] = math.nan
            vd = None
        else:
            x = torch.randint(-1000, 1000, (n,), generator=g, dtype=torch.int32)
            vd = (torch.rand(n, generator=g) > 0.3).to(torch.uint8)
        cols.append(x)
        valids.append(vd)
    ws = {}
    got = D.hash_agg_radix(k.cuda(), [c.cuda() for c in cols], [None if x is None else x.cuda() for x in valids],
                           False, ws=ws)
    assert "r2prow" in ws, "two-level range path not taken"
    want = D.hash_agg(k, cols, valids, False)
    _assert_agg_equal(got, want, False)


@pytest.mark.parametrize("lo,span,nv", [(0, 1000, 1), (-70, 3000, 2), (5_000_000_000, 17, 0), (3, 2000, 4)])
def test_small_range_agg_matches_host(hip_built, lo, span, nv):
    """Key spans of a few thousand values skip partitioning (small_range_agg_k: one direct-indexed
    LDS table per workgroup over the whole range); NaN values and validity masks, vs the host path."""
    n = 5_000_000
    g = torch.Generator().manual_seed(span + nv)
    k = torch.randint(0, span, (n,), generator=g) + lo
    cols, valids = [], []
    for j in range(nv):
        if j % 2 == 0:
            x = torch.randn(n, generator=g, dtype=torch.float64)
            x[::89] = math.nan
            vd = None
        else:
            x = torch.randint(-500, 500, (n,), generator=g, dtype=torch.int32)
            vd = (torch.rand(n, generator=g) > 0.25).to(torch.uint8)
        cols.append(x)
        valids.append(vd)
    got = D.hash_agg(k.cuda(), [c.cuda() for c in cols], [None if x is None else x.cuda() for x in valids], False)
    want = D.hash_agg(k, cols, valids, False)
    _assert_agg_equal(got, want, False)


def test_range_agg_off_switch_same_result(hip_built, monkeypatch):
    k, v = D.fill_synthetic_kv(5_000_000, 50_000, "cuda")
    a = D.hash_agg_radix(k, [v], [None], False)
    monkeypatch.setenv("PTG_GROUPBY_RANGE", "0")
    ws = {}
    b = D.hash_agg_radix(k, [v], [None], False, ws=ws)
    assert "rprow" not in ws
    _assert_agg_equal(a, b, False)


def test_repeat_runs_agree(hip_built):
    """Deterministic-mode check: the same groupBy / sort twice.  Keys and counts are
    exact and identical (range path, hash radix path, LDS hash path); f64 sums differ at most by the
    order of LDS atomic adds; the stable radix sort is bitwise identical."""
    k, v = D.fill_synthetic_kv(6_000_000, 700_000, "cuda", seed=5)
    for env in ("1", "0"):
        os.environ["PTG_GROUPBY_RANGE"] = env
        try:
            runs = [_sorted_agg(*D.hash_agg_radix(k, [v], [None], False)) for _ in range(2)]
        finally:
            os.environ.pop("PTG_GROUPBY_RANGE", None)
        (k1, r1, o1), (k2, r2, o2) = runs
        assert torch.equal(k1, k2) and torch.equal(r1, r2) and torch.equal(o1[0][1], o2[0][1])
        assert torch.allclose(o1[0][0], o2[0][0], rtol=1e-12, atol=1e-12)
    small = [_sorted_agg(*D.hash_agg(k[:1_000_000] % 1000, [v[:1_000_000]], [None], False)) for _ in range(2)]
    assert torch.equal(small[0][0], small[1][0]) and torch.equal(small[0][1], small[1][1])
    sk, lo, hi = D.sort_key(k, False)
    a = D.radix_sort_u64(sk, None, lo, hi, row_payload=True)
    b = D.radix_sort_u64(sk, None, lo, hi, row_payload=True)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])


@pytest.mark.parametrize("est", [1_000, 300_000])
def test_radix_agg_spill_recursion(hip_built, est):
    """An estimate far below the real 2M keys sizes the tables too small: partitions spill and are
    re-partitioned one level deeper until every key is emitted exactly once (no lost rows)."""
    k, v = D.fill_synthetic_kv(6_000_000, 2_000_000, "cuda")
    got = D.hash_agg_radix(k, [v], [None], False, est_keys=est)
    want = D.hash_agg(k.cpu(), [v.cpu()], [None], False)
    _assert_agg_equal(got, want, False)


def test_radix_agg_skewed_keys(hip_built):
    """Heavy hitters plus a long tail: one partition holds most rows of a few keys."""
    n = 4_000_000
    g = torch.Generator().manual_seed(7)
    k = torch.where(torch.rand(n, generator=g) < 0.6, torch.randint(0, 3, (n,), generator=g),
                    torch.randint(0, 1 << 40, (n,), generator=g))
    v = torch.rand(n, generator=g, dtype=torch.float64)
    got = D.hash_agg_radix(k.cuda(), [v.cuda()], [None], True)
    want = D.hash_agg(k, [v], [None], True)
    _assert_agg_equal(got, want, True)


@pytest.mark.parametrize("nkeys", [1_000, 1_000_000, 16_000_000, 128_000_000])
def test_groupby_256m_rows_any_cardinality(spark_gpu, nkeys):
    """DataFrame groupBy over 256M rows: sum(count) == n and sum(sum) == sum(values) at every
    cardinality, the group count matches the keys present, and an 8M-row slice is exact vs the
    host path."""
    from pyspark_tf_gke_amd.sql import functions as F
    from pyspark_tf_gke_amd.sql import types as T
    from pyspark_tf_gke_amd.sql.dataframe import DataFrame
    from pyspark_tf_gke_amd.sql.table import ColumnVector, Table

    n = 256 * 1024 * 1024
    k, v = D.fill_synthetic_kv(n, nkeys, "cuda", seed=nkeys)
    df = DataFrame(Table({"key": ColumnVector(k, T.LongType()), "value": ColumnVector(v, T.DoubleType())}, n,
                         k.device), spark_gpu)
    out = df.groupBy("key").agg(F.sum("value").alias("s"), F.count("*").alias("c"))
    c = out._t.column("c").data
    ssum = out._t.column("s").data
    assert int(c.sum().item()) == n
    assert abs(float(ssum.sum().item()) - float(v.sum().item())) <= 1e-9 * n
    present = int(torch.unique(k).numel())
    assert out._t.num_rows == present
    del out, c, ssum
    m = 8 * 1024 * 1024
    got = D.hash_agg_radix(k[:m].contiguous(), [v[:m].contiguous()], [None], True)
    want = D.hash_agg(k[:m].cpu(), [v[:m].cpu()], [None], True)
    _assert_agg_equal(got, want, True)


def test_synthetic_kv_device_matches_host(hip_built):
    kg, vg = D.fill_synthetic_kv(10_000, 1000, "cuda", offset=5, seed=3)
    kh, vh = D.fill_synthetic_kv(10_000, 1000, "cpu", offset=5, seed=3)
    assert torch.equal(kg.cpu(), kh) and torch.allclose(vg.cpu(), vh)


def test_dataframe_pipeline_gpu_vs_host(spark_gpu):
    from pyspark_tf_gke_amd.sql.functions import avg, col, count, isnan, when

    def run(spark):
        df = spark.read.csv(HEALTH, header=True, inferSchema=True)
        df = df.filter(col("measure_name").isNotNull())
        for c in ["value", "lower_ci", "upper_ci"]:
            mv = df.select(c).filter(~isnan(col(c)) & col(c).isNotNull()).agg({c: "avg"}).collect()[0][0]
            df = df.withColumn(c, when(col(c).isNull() | isnan(col(c)), mv).otherwise(col(c)))
        g = df.groupBy("measure_name").agg(count("*").alias("n"), avg("value").alias("m"))
        rows = sorted((r["measure_name"], r["n"], round(r["m"], 6)) for r in g.collect())
        f = df.filter((col("value") > 50) & (col("state_name") == "Texas")).count()
        return rows, f, df.count()

    g = run(spark_gpu)
    h = _host(run)
    assert g == h


def test_kmeans_and_silhouette_gpu_vs_host(spark_gpu):
    from pyspark_tf_gke_amd.ml import ClusteringEvaluator, KMeans, OneHotEncoder, Pipeline, StringIndexer, VectorAssembler
    from pyspark_tf_gke_amd.sql.functions import col

    def run(spark):
        df = spark.read.csv(HEALTH, header=True, inferSchema=True).na.fill(0)
        stages = [StringIndexer(inputCol="measure_name", outputCol="mi", handleInvalid="keep"),
                  OneHotEncoder(inputCol="mi", outputCol="mv"),
                  VectorAssembler(inputCols=["mv"] * 5 + ["value", "lower_ci", "upper_ci"], outputCol="features",
                                  handleInvalid="keep")]
        t = Pipeline(stages=stages).fit(df).transform(df)
        km = KMeans(k=5, seed=1, maxIter=50).fit(t)
        sil = ClusteringEvaluator().evaluate(km.transform(t))
        return km.summary.trainingCost, sil, t._t.column("features").data.float().cpu()

    cg, sg, fg = run(spark_gpu)
    ch, sh, fh = _host(run)
    assert torch.equal(fg, fh)
    assert abs(cg - ch) <= 1e-3 * abs(ch)
    assert abs(sg - sh) <= 1e-3
    _ = col


@pytest.mark.parametrize("n,kind", [(1, "i64"), (2047, "i64"), (2049, "f64"), (1_000_003, "i64"), (3_000_000, "f64"),
                                    (2_500_000, "i32"), (4_000_000, "small"), (1_500_000, "u8")])
@pytest.mark.parametrize("desc", [False, True])
def test_radix_sort_matches_stable_host_sort(hip_built, n, kind, desc):
    """Stable LSD radix sort (sort_key_prep_k / sort_count_k / sort_scatter_k) vs numpy's stable
    argsort of the same orderable keys: identical permutation (ties keep input order)."""
    g = torch.Generator().manual_seed(n)
    if kind == "i64":
        x = torch.randint(-(1 << 62), 1 << 62, (n,), generator=g, dtype=torch.int64)
    elif kind == "f64":
        x = torch.randn(n, generator=g, dtype=torch.float64) * 1e6
        x[::13] = math.nan
        x[::17] = -0.0
        x[::19] = 0.0
        x[::23] = math.inf
    elif kind == "i32":
        x = torch.randint(-(1 << 31), (1 << 31) - 1, (n,), generator=g, dtype=torch.int32)
    elif kind == "small":  # few distinct values in a narrow range: 1 pass, heavy ties
        x = torch.randint(1000, 1037, (n,), generator=g, dtype=torch.int64)
    else:
        x = torch.randint(0, 2, (n,), generator=g, dtype=torch.uint8)
    kg, lo, hi = D.sort_key(x.cuda(), desc)
    kh, loh, hih = D.sort_key(x, desc)
    assert torch.equal(kg.cpu(), kh) and (lo, hi) == (loh, hih)
    sk, perm = D.radix_sort_u64(kg, None, lo, hi)
    want = np.argsort(kh.numpy().view(np.uint64), kind="stable")
    assert torch.equal(perm.cpu(), torch.from_numpy(want.astype(np.int64)))
    assert torch.equal(sk.cpu(), kh[torch.from_numpy(want)])

def test_radix_sort_wide_payload(hip_built):
    """An arbitrary int64 payload (not row ids) keeps the 64-bit scatter path: values above 2^32
    come back intact, in stable key order."""
    n = 300_001
    g = torch.Generator().manual_seed(5)
    k = torch.randint(0, 1 << 20, (n,), generator=g, dtype=torch.int64)
    pay = torch.randint(-(1 << 62), 1 << 62, (n,), generator=g, dtype=torch.int64)
    sk, sv = D.radix_sort_u64(k.cuda(), pay.cuda(), 0, (1 << 20) - 1)
    order = np.argsort(k.numpy(), kind="stable")
    assert torch.equal(sk.cpu(), k[torch.from_numpy(order)])
    assert torch.equal(sv.cpu(), pay[torch.from_numpy(order)])


@pytest.mark.parametrize("n", [1, 4095, 4096 * 3 + 17])
def test_sort_range_count(hip_built, n):
    """df.hip sort_range_count_k: the orderable key range and each tile's raw low-byte histogram in
    one read; the first radix pass's digit counts are that histogram rotated by lo & 255."""
    from pyspark_tf_gke_amd.ops import df as D

    g = torch.Generator().manual_seed(n)
    k = torch.randint(-(1 << 62), 1 << 62, (n,), generator=g, dtype=torch.int64)
    for desc in (False, True):
        m = D.orderable_mask(desc)
        lo, hi, h = D.sort_range_count(k.cuda(), m)
        u = (k ^ m).numpy().view(np.uint64)
        assert lo == int(u.min()) and hi == int(u.max())
        ST = D._native.hip_lib().ptg_sort_tile_rows()
        nt = -(-n // ST)
        want = np.zeros((nt, 256), np.int64)
        for t in range(nt):
            want[t] = np.bincount((u[t * ST:(t + 1) * ST] & np.uint64(255)).astype(np.int64), minlength=256)
        assert np.array_equal(h.cpu().numpy().reshape(nt, 256), want)


@pytest.mark.parametrize("payload,fused", [("1", "1"), ("0", "1"), ("1", "0"), ("0", "0")])
@pytest.mark.parametrize("dtype,asc", [(torch.int64, True), (torch.int64, False), (torch.int32, True)])
def test_orderby_integer_key_output_keys(spark_gpu, dtype, asc, payload, fused, monkeypatch):
    """Single null-free integer sort column: the sorted key column is decoded from the radix
    sort's own output keys (not gathered); the result equals a stable host sort, ties included.
    payload=1: the one value column rides through the radix passes as the payload; 0: row-id
    payload + gather.  fused=1 (int64): the first radix pass reads the raw column and the last writes
    the decoded values (no key prep write, no decode pass)."""
    monkeypatch.setenv("PTG_SORT_VALUE_PAYLOAD", payload)
    monkeypatch.setenv("PTG_SORT_FUSED_KEYS", fused)
    from pyspark_tf_gke_amd.sql import types as T
    from pyspark_tf_gke_amd.sql.dataframe import DataFrame
    from pyspark_tf_gke_amd.sql.table import ColumnVector, Table

    n = 1_000_000
    g = torch.Generator().manual_seed(11)
    info = torch.iinfo(dtype)
    k = torch.randint(info.min, info.max, (n,), generator=g, dtype=dtype)
    k[1::2] = k[0::2]  # ties (n is even)
    k[5], k[6] = info.min, info.max
    v = torch.rand(n, generator=g, dtype=torch.float64)
    lt = T.LongType() if dtype == torch.int64 else T.IntegerType()
    df = DataFrame(Table({"key": ColumnVector(k.cuda(), lt), "value": ColumnVector(v.cuda(), T.DoubleType())}, n,
                         torch.device("cuda")), spark_gpu)
    out = df.orderBy("key", ascending=asc)
    kk = k.numpy()
    if asc:
        order = np.argsort(kk, kind="stable")
    else:  # descending keys, ties in input order
        order = (n - 1) - np.argsort(kk[::-1], kind="stable")[::-1]
    order = torch.as_tensor(np.ascontiguousarray(order, dtype=np.int64))
    assert out._t.column("key").data.dtype == dtype
    assert torch.equal(out._t.column("key").data.cpu(), k[order])
    assert torch.equal(out._t.column("value").data.cpu(), v[order])


def test_argsort_columns_gpu_vs_host(hip_built):
    """Multi-column orderBy permutation (asc/desc, nulls first/last) on the GPU equals the host."""
    n = 500_000
    g = torch.Generator().manual_seed(3)
    a = torch.randint(0, 50, (n,), generator=g, dtype=torch.int64)
    b = torch.randn(n, generator=g, dtype=torch.float64)
    b[::11] = math.nan
    null_a = torch.rand(n, generator=g) < 0.05
    null_b = torch.rand(n, generator=g) < 0.02
    spec = [(a, null_a, True), (b, null_b, False), (torch.arange(n) % 7, None, False)]
    pg = D.argsort_columns([(x.cuda(), None if m is None else m.cuda(), d) for x, m, d in spec])
    ph = D.argsort_columns(spec)
    assert torch.equal(pg.cpu(), ph)


def test_dataframe_orderby_gpu_vs_host(spark_gpu):
    from pyspark_tf_gke_amd.sql.functions import col

    def run(spark):
        df = spark.read.csv(HEALTH, header=True, inferSchema=True)
        o = df.orderBy(col("state_name").desc(), "value", col("measure_name").asc())
        return [tuple(r) for r in o.select("state_name", "value", "measure_name").collect()]

    assert run(spark_gpu) == _host(run)


@pytest.mark.parametrize("n,k,Dm", [(20_000, 100, 153), (7_777, 5, 3), (30_000, 300, 300), (5_000, 40, 600),
                                    (6_000, 25, 623), (4_000, 25, 2048), (3_000, 7, 1031)])
def test_kmeans_mfma_assign_matches_host(hip_built, n, k, Dm):
    """Fused MFMA assignment vs the fp64 host formula: same argmin wherever the best two centers
    are not within f32 rounding, sums/counts/cost to f32 accuracy.  (300 x 300 exceeds the LDS
    accumulator -> global-atomic path; D > KM_DMAX = 576 -> the feature dimension tiled through
    LDS in 512-wide chunks: D = 623 is k_means.py with MEASURE_NAME_WEIGHT = 20, 1031 a ragged
    last chunk.)"""
    g = torch.Generator().manual_seed(k)
    X = torch.randn(n, Dm, generator=g)
    X[:, : Dm // 3] = (X[:, : Dm // 3] > 1.0).float()  # one-hot-like sparse block (skipped zeros)
    C = X[torch.randperm(n, generator=g)[:k]].clone() + 0.01 * torch.randn(k, Dm, generator=g)
    out = {}
    for dev in ("cuda", "cpu"):
        Xd, Cd = X.to(dev), C.to(dev)
        a = torch.empty(n, dtype=torch.int32, device=dev)
        md = torch.empty(n, dtype=torch.float32, device=dev)
        s = torch.zeros(k, Dm, dtype=torch.float32, device=dev)
        c = torch.zeros(k, dtype=torch.float32, device=dev)
        cost = torch.zeros(1, dtype=torch.float64, device=dev)
        D.kmeans_assign_accum(Xd, Cd, assign=a, sums=s, counts=c, cost=cost, mind=md)
        out[dev] = [t.cpu() for t in (a, md, s, c, cost)]
    ag, mg, sg, cg, costg = out["cuda"]
    ah, mh, sh, ch, costh = out["cpu"]
    d = ((X.double()[:, None, :] - C.double()[None]) ** 2).sum(2) if n * k * Dm < 4e8 else None
    if d is not None:
        top2 = torch.topk(d, 2, dim=1, largest=False).values
        clear = (top2[:, 1] - top2[:, 0]) > 1e-4 * top2[:, 1].clamp_min(1.0)
        assert torch.equal(ag[clear], ah[clear])
    assert (ag == ah).float().mean() > 0.999
    # mind = ||x||^2 - 2 x.c + ||c||^2 in f32: the absolute error scales with ||x||^2, not with the
    # (tiny) distance of a row that is itself (almost) a center -> atol relative to the row norms
    atol = max(1e-3, 1e-5 * float((X * X).sum(1).max()))
    assert torch.allclose(mg, mh, rtol=1e-4, atol=atol)
    if bool((ag == ah).all()):
        assert torch.equal(cg, ch)
        assert torch.allclose(sg, sh, rtol=1e-4, atol=1e-3)
    assert abs(float(costg) - float(costh)) <= 1e-5 * abs(float(costh))


def test_kmeans_fit_k100_d153_vs_host_and_sklearn(spark_gpu):
    """KMeans.fit with k=100 on 153-dim features (the reference's one-hot x5 + 3 numeric shape):
    device convergence loop vs the host executor (same seed -> same random init), and one more
    scikit-learn Lloyd step from our centers finds (almost) nothing left to improve."""
    from sklearn.cluster import KMeans as SKM

    from pyspark_tf_gke_amd.ml import KMeans
    from pyspark_tf_gke_amd.sql.table import ColumnVector, Table
    from pyspark_tf_gke_amd.sql import types as T
    from pyspark_tf_gke_amd.sql.dataframe import DataFrame

    g = torch.Generator().manual_seed(5)
    n, Dm = 12_000, 153
    codes = torch.randint(0, 30, (n,), generator=g)
    X = torch.zeros(n, Dm)
    for r in range(5):
        X[torch.arange(n), r * 30 + codes] = 1.0
    X[:, 150:] = torch.randn(n, 3, generator=g) * 3 + codes[:, None].float()

    def fit(dev):
        df = DataFrame(Table({"features": ColumnVector(X.to(dev), T.VectorUDT())}, n, dev), spark_gpu)
        return KMeans(k=100, seed=3, maxIter=30, initMode="random").fit(df)

    mg, mh = fit("cuda"), fit("cpu")
    assert abs(mg.summary.trainingCost - mh.summary.trainingCost) <= 1e-3 * mh.summary.trainingCost
    sk = SKM(n_clusters=100, init=np.asarray(mg.clusterCenters()), n_init=1, max_iter=1).fit(X.numpy().astype(np.float64))
    assert mg.summary.trainingCost <= sk.inertia_ * 1.01
    assert sum(mg.summary.clusterSizes) == n


@pytest.mark.parametrize("n,k,Dm", [(9_000, 37, 153), (5_000, 25, 623), (3_000, 9, 2048)])
def test_silhouette_mfma_matches_host(hip_built, n, k, Dm):
    """Silhouette sum on the matrix cores (D-chunked above 576 features) vs the fp64 host formula."""
    g = torch.Generator().manual_seed(1)
    X = torch.randn(n, Dm, generator=g)
    a = torch.randint(0, k, (n,), generator=g, dtype=torch.int32)
    a[a == 7] = 8  # an empty cluster
    Sg, Qg, cg = D.silhouette_sum(X.cuda(), a.cuda(), k)
    Sh, Qh, ch = D.silhouette_sum(X, a, k)
    assert torch.allclose(Sg.cpu(), Sh, atol=1e-2) and torch.equal(cg.cpu(), ch)
    tg = D.silhouette_points(X.cuda(), a.cuda(), Sg, Qg, cg)
    th = D.silhouette_points(X, a, Sh, Qh, ch)
    assert abs(tg - th) <= 1e-3 * max(1.0, abs(th))


@pytest.mark.parametrize("weight", [20, 66])
def test_kmeans_fit_wide_features_vs_host_and_sklearn(spark_gpu, weight):
    """k_means.py's feature weighting (k_means.py:56-64): the 31-wide one-hot repeated
    MEASURE_NAME_WEIGHT times + 3 numeric columns -> D = 623 (weight 20) / 2049 (weight 66), on the
    HIP path end to end (no host fallback above 576 features): cost vs the host executor, and a
    scikit-learn Lloyd step from our centers finds (almost) nothing to improve."""
    from sklearn.cluster import KMeans as SKM

    from pyspark_tf_gke_amd.ml import ClusteringEvaluator, KMeans
    from pyspark_tf_gke_amd.sql import types as T
    from pyspark_tf_gke_amd.sql.dataframe import DataFrame
    from pyspark_tf_gke_amd.sql.table import ColumnVector, Table

    g = torch.Generator().manual_seed(7)
    n, V = 6_000, 31
    Dm = V * weight + 3
    codes = torch.randint(0, 30, (n,), generator=g)
    X = torch.zeros(n, Dm)
    for r in range(weight):
        X[torch.arange(n), r * V + codes] = 1.0
    X[:, -3:] = torch.randn(n, 3, generator=g) * 3 + codes[:, None].float()

    def fit(dev):
        df = DataFrame(Table({"features": ColumnVector(X.to(dev), T.VectorUDT())}, n, dev), spark_gpu)
        m = KMeans(k=25, seed=1, maxIter=20, initMode="random").fit(df)
        sil = ClusteringEvaluator().evaluate(m.transform(df))
        return m, sil

    (mg, sg), (mh, sh) = fit("cuda"), fit("cpu")
    assert abs(mg.summary.trainingCost - mh.summary.trainingCost) <= 1e-3 * mh.summary.trainingCost
    assert abs(sg - sh) <= 2e-3
    sk = SKM(n_clusters=25, init=np.asarray(mg.clusterCenters()), n_init=1, max_iter=1).fit(X.numpy().astype(np.float64))
    assert mg.summary.trainingCost <= sk.inertia_ * 1.01
    assert sum(mg.summary.clusterSizes) == n


@pytest.mark.parametrize("lo,span", [(-3_000_000_000, 4_000_000_000), (1 << 40, (1 << 32) - 2), (-(1 << 62), 1 << 62)])
def test_radix_agg_key_compression_ranges(hip_built, lo, span):
    """u32-offset key compression (key range < 2^32 - 1, including negative and offset ranges) and the
    i64 fallback (a 2^62 range) give the same groups as the host path."""
    n = 3_000_000
    g = torch.Generator().manual_seed(span % 1000)
    base = torch.randint(0, 300_000, (n,), generator=g, dtype=torch.int64)
    k = lo + (base * (span // 300_000)) % span
    k[:2] = torch.tensor([lo, lo + span - 1])  # both ends of the range
    v = torch.rand(n, generator=g, dtype=torch.float64)
    got = D.hash_agg_radix(k.cuda(), [v.cuda()], [None], True)
    want = D.hash_agg(k, [v], [None], True)
    _assert_agg_equal(got, want, True)


@pytest.mark.parametrize("n", [0, 1, 4095, 4096, 4097, 1 << 20, 5_000_003])
def test_scan_minmax_sample_gather_kernels(hip_built, n):
    """dfutil.hip: exclusive scans (int32 / int64, total slot), int64 min/max over strided views,
    strided sampling and the fixed-row gathers (int64 / u32 indices) vs torch on the host."""
    g = torch.Generator().manual_seed(n)
    x32 = torch.randint(0, 1000, (n,), generator=g, dtype=torch.int32)
    x64 = torch.randint(-(1 << 40), 1 << 40, (n,), generator=g, dtype=torch.int64)
    for x in (x32, x64):
        out = torch.empty(n + 1, dtype=torch.int64, device="cuda")
        D.scan_excl(x.cuda(), out=out[:n], total=out[n:])
        cs = torch.cumsum(x.long(), 0)
        want = torch.cat([torch.zeros(1, dtype=torch.int64), cs])
        assert torch.equal(out.cpu(), want)
    if n:
        assert D.minmax_i64(x64.cuda()) == (int(x64.min()), int(x64.max()))
        pairs = x64[: (n // 2) * 2].view(-1, 2)
        if pairs.numel():
            assert D.minmax_i64(pairs.cuda().contiguous(), n=pairs.shape[0], stride=2, off_min=0, off_max=1) == (
                int(pairs[:, 0].min()), int(pairs[:, 1].max()))
        st = max(1, n // 1000)
        m = (n + st - 1) // st
        assert torch.equal(D.strided_sample(x64.cuda(), st, m).cpu(), x64[::st][:m])
        idx = torch.randint(0, n, (n,), generator=g)
        vals = torch.randn(n, generator=g, dtype=torch.float64)
        assert torch.equal(D.gather_rows(vals.cuda(), idx.cuda()).cpu(), vals[idx])
        assert torch.equal(D.gather_rows(x32.cuda(), idx.to(torch.int32).cuda()).cpu(), x32[idx])


def test_groupby_sparse_keys_hash_path_vs_host(hip_built):
    """1M distinct keys spread over the int64 range (bench extra.groupby_sparse): the sparse fill
    equals its host twin, and the radix-partitioned hash aggregation matches the host groupBy."""
    n, nk = 4_000_000, 1_000_000
    kc, vc = D.fill_synthetic_kv(n, nk, "cpu", sparse=True)
    kg, vg = D.fill_synthetic_kv(n, nk, "cuda", sparse=True)
    assert torch.equal(kg.cpu(), kc) and torch.equal(vg.cpu(), vc)
    assert int(kc.max()) - int(kc.min()) > (1 << 60)
    uk, rows, outs = D.hash_agg_radix(kg, [vg], [None], False)
    order = torch.argsort(uk.cpu())
    hk, hrows, houts = D.hash_agg(kc, [vc], [None], False)
    horder = torch.argsort(hk)
    assert torch.equal(uk.cpu()[order], hk[horder])
    assert torch.equal(rows.cpu()[order], hrows[horder])
    assert torch.allclose(outs[0][0].cpu()[order], houts[0][0][horder], rtol=1e-9, atol=1e-9)


@pytest.mark.parametrize("ntiles", [1, 63, 64, 65, 1000, 5003])
def test_digit_offsets_tile_major(ntiles):
    """dfutil.hip ptg_digit_offsets: the digit-major exclusive scan of tile-major [ntiles][256] counts,
    written tile-major, with the total after the last row."""
    from pyspark_tf_gke_amd.ops import df as D

    torch.manual_seed(ntiles)
    hist = torch.randint(0, 5000, (ntiles, 256), dtype=torch.int32)
    ref = torch.cumsum(hist.t().reshape(-1).long(), 0) - hist.t().reshape(-1).long()  # digit-major
    ref = ref.view(256, ntiles).t().reshape(-1)
    ws = {}

    def buf(name, shape, dtype):
        t = ws.get(name)
        if t is None:
            t = ws[name] = torch.empty(int(np.prod(shape)), dtype=dtype, device="cuda")
        return t.view(shape)

    offs = torch.full((256 * ntiles + 1,), -7, dtype=torch.int64, device="cuda")
    D.digit_offsets(hist.reshape(-1).cuda(), ntiles, offs, buf)
    out = offs.cpu()
    assert torch.equal(out[:-1], ref)
    assert int(out[-1]) == int(hist.long().sum())


def _h9_buf():
    ws = {}

    def buf(name, shape, dtype):
        numel = int(np.prod(shape))
        t = ws.get(name)
        if t is None or t.numel() < numel or t.dtype != dtype:
            t = ws[name] = torch.empty(numel, dtype=dtype, device="cuda")
        return t[:numel].view(shape)
    return buf


@pytest.mark.parametrize("n,nkeys,nv", [(8_388_608, 1_000_000, 1), (6_000_000, 120_000, 2), (5_000_000, 400_000, 0),
                                        (4_500_000, 1_200_000, 1)])
def test_hash9_agg_matches_host(hip_built, n, nkeys, nv):
    """One-level 512-way hash partition + chunked LDS hash tables + per-partition merge (df.hip
    hash9_*_k) vs the host groupBy: sparse int64 keys, f64 and int32 columns with nulls / NaN."""
    k, v = D.fill_synthetic_kv(n, nkeys, "cuda", sparse=True)
    g = torch.Generator().manual_seed(n + nv)
    cols, valids = [], []
    for j in range(nv):
        x = v.clone() if j == 0 else torch.randint(-1000, 1000, (n,), generator=g, dtype=torch.int32).cuda()
        if j == 0:
            x[::101] = math.nan
        cols.append(x)
        valids.append((torch.rand(n, generator=g) > 0.2).to(torch.uint8).cuda() if j == 1 else None)
    pay = [(c.contiguous(), vd) for c, vd in zip(cols, valids)]
    got = D.hash_agg_h9(k, pay, _h9_buf(), nv, nkeys)
    assert got is not None
    want = D.hash_agg(k.cpu(), [c.cpu() for c in cols], [None if x is None else x.cpu() for x in valids], False)
    _assert_agg_equal(got, want, False)
    # and through the planner (sampled distinct-key estimate)
    _assert_agg_equal(D.hash_agg_radix(k, cols, valids, False), want, False)


def test_hash9_overflow_falls_back(hip_built):
    """An estimate 40x too low sizes the LDS tables far too small: the kernels flag the overflow,
    hash_agg_h9 returns None and the planner's recursive path still gives the exact result."""
    n, nk = 4_500_000, 1_000_000
    k, v = D.fill_synthetic_kv(n, nk, "cuda", sparse=True)
    assert D.hash_agg_h9(k, [(v, None)], _h9_buf(), 1, nk // 40) is None
    got = D.hash_agg_radix(k, [v], [None], False, est_keys=nk // 40)
    want = D.hash_agg(k.cpu(), [v.cpu()], [None], False)
    _assert_agg_equal(got, want, False)


@pytest.mark.parametrize("ntiles", [1, 65, 3001])
def test_digit_offsets_512_bins(ntiles):
    """ptg_digit_offsets_b with 512 digits (the hash9 partition) = digit-major exclusive scan."""
    from pyspark_tf_gke_amd.ops._util import hip, ptr

    torch.manual_seed(ntiles)
    B = 512
    hist = torch.randint(0, 3000, (ntiles, B), dtype=torch.int32)
    ref = torch.cumsum(hist.t().reshape(-1).long(), 0) - hist.t().reshape(-1).long()
    ref = ref.view(B, ntiles).t().reshape(-1)
    tpc = D.DIGIT_OFFS_TPC
    nch = -(-ntiles // tpc)
    hg = hist.reshape(-1).cuda()
    csum = torch.empty(B * nch, dtype=torch.int64, device="cuda")
    cbase = torch.empty_like(csum)
    offs = torch.full((B * ntiles + 1,), -7, dtype=torch.int64, device="cuda")
    hip("ptg_digit_offsets_b", 0, ptr(hg), ntiles, tpc, ptr(csum), nch, None, B, 0)
    D.scan_excl(csum, out=cbase, total=offs[B * ntiles:])
    hip("ptg_digit_offsets_b", 1, ptr(hg), ntiles, tpc, ptr(cbase), nch, ptr(offs), B, 0)
    out = offs.cpu()
    assert torch.equal(out[:-1], ref)
    assert int(out[-1]) == int(hist.long().sum())


# ---- multi-column / nullable group keys on our kernels (dfkey.hip) vs pandas -----------------------
def _pd_health():
    import pandas as pd

    return pd.read_csv(HEALTH)


def test_groupby_two_nullable_keys_vs_pandas(spark_gpu):
    """groupBy(measure_name, subpopulation) on health.csv: `subpopulation` has 1,508 empty values
    (null in Spark), so the key is a 2-column nullable tuple packed into one exact int64 key."""
    from pyspark_tf_gke_amd.sql.functions import avg, count, max as fmax, min as fmin, sum as fsum

    df = spark_gpu.read.csv(HEALTH, header=True, inferSchema=True)
    g = df.groupBy("measure_name", "subpopulation").agg(
        count("*").alias("n"), count("value").alias("nv"), avg("value").alias("m"), fsum("value").alias("s"),
        fmin("value").alias("lo"), fmax("upper_ci").alias("hi"))
    got = {(r["measure_name"], r["subpopulation"]): (r["n"], r["nv"], r["m"], r["s"], r["lo"], r["hi"])
           for r in g.collect()}
    p = _pd_health()
    ref = {}
    for (mn, sp), grp in p.groupby(["measure_name", "subpopulation"], dropna=False):
        sp = None if isinstance(sp, float) and math.isnan(sp) else sp
        v = grp["value"].dropna()
        ref[(mn, sp)] = (len(grp), len(v), v.mean() if len(v) else None, v.sum() if len(v) else None,
                         v.min() if len(v) else None, grp["upper_ci"].max())
    assert set(got) == set(ref)
    assert any(k[1] is None for k in got)  # the null group exists
    for k, (n, nv, m, s, lo, hi) in ref.items():
        g_ = got[k]
        assert g_[0] == n and g_[1] == nv, (k, g_, ref[k])
        for a, b in zip(g_[2:], (m, s, lo, hi)):
            assert (a is None and (b is None or b != b)) or math.isclose(a, b, rel_tol=1e-9, abs_tol=1e-9), (k, g_, ref[k])


def test_groupby_three_keys_wide_ranges_vs_host(spark_gpu):
    """Three key columns whose value ranges cannot share 63 bits (two full-range int64 columns):
    the widest switch to rank coding (sorted distinct keys, binary search in the pack kernel)."""
    from pyspark_tf_gke_amd.sql.functions import count, sum as fsum
    from pyspark_tf_gke_amd.sql.session import SparkSession

    rng = np.random.default_rng(3)
    n = 50_000
    a = rng.integers(-(1 << 62), 1 << 62, 40)[rng.integers(0, 40, n)]
    b = rng.integers(-(1 << 62), 1 << 62, 30)[rng.integers(0, 30, n)]
    c = rng.integers(0, 5, n)
    v = rng.normal(size=n)
    rows = [(int(x), int(y), int(z), float(w)) for x, y, z, w in zip(a, b, c, v)]

    def run(spark):
        df = spark.createDataFrame(rows, ["a", "b", "c", "v"])
        out = df.groupBy("a", "b", "c").agg(count("*").alias("n"), fsum("v").alias("s")).collect()
        return sorted((r["a"], r["b"], r["c"], r["n"], round(r["s"], 9)) for r in out)

    assert run(spark_gpu) == _host(run)


def test_count_distinct_and_drop_duplicates_vs_pandas(spark_gpu):
    from pyspark_tf_gke_amd.sql.functions import countDistinct

    df = spark_gpu.read.csv(HEALTH, header=True, inferSchema=True)
    p = _pd_health()
    got = df.agg(countDistinct("subpopulation").alias("a"), countDistinct("value").alias("b"),
                 countDistinct("state_name").alias("c")).collect()[0]
    assert got["a"] == p["subpopulation"].nunique() and got["c"] == p["state_name"].nunique()
    assert got["b"] == p["value"].nunique()
    dd = df.dropDuplicates(["measure_name", "subpopulation"]).collect()
    ref = p.drop_duplicates(["measure_name", "subpopulation"])
    assert len(dd) == len(ref)
    # the surviving rows are the first occurrences, in input order
    assert [r["edition"] for r in dd] == ref["edition"].tolist()
    assert [r["measure_name"] for r in dd] == ref["measure_name"].tolist()
    assert df.select("measure_name", "subpopulation").distinct().count() == len(ref)


def test_groupby_more_than_four_value_columns(spark_gpu):
    from pyspark_tf_gke_amd.sql.functions import avg, max as fmax, sum as fsum

    df = spark_gpu.read.csv(HEALTH, header=True, inferSchema=True)
    g = df.groupBy("state_name").agg(fsum("value").alias("s1"), avg("lower_ci").alias("a2"), fmax("upper_ci").alias("m3"),
                                     fsum("lower_ci").alias("s4"), avg("value").alias("a5"), fmax("value").alias("m6"))
    got = {r["state_name"]: r for r in g.collect()}
    p = _pd_health()
    for st, grp in p.groupby("state_name"):
        r = got[st]
        for name, ref in (("s1", grp["value"].sum()), ("a2", grp["lower_ci"].mean()), ("m3", grp["upper_ci"].max()),
                          ("s4", grp["lower_ci"].sum()), ("a5", grp["value"].mean()), ("m6", grp["value"].max())):
            assert math.isclose(r[name], ref, rel_tol=1e-9, abs_tol=1e-9), (st, name, r[name], ref)


def _spec_launches():
    import ctypes

    from pyspark_tf_gke_amd import _native

    v = ctypes.c_long(0)
    _native.hip_lib().ptg_expr_spec_launches(ctypes.byref(v))
    return v.value


def test_specialised_expressions_match_vm(spark_gpu, monkeypatch):
    """expr_affine_k (one column, one constant, one op, optional int cast, or a comparison) gives
    bit-identical values and null masks to the expression VM, including NaN / inf / out-of-range
    casts and an odd-length tail, for every column and output type; other shapes stay on the VM."""
    from pyspark_tf_gke_amd.sql import types as T
    from pyspark_tf_gke_amd.sql.dataframe import DataFrame
    from pyspark_tf_gke_amd.sql.functions import col
    from pyspark_tf_gke_amd.sql.table import ColumnVector, Table

    n = 100_003
    g = torch.Generator().manual_seed(5)
    v = torch.randn(n, generator=g, dtype=torch.float64) * 1e3
    v[::97] = float("nan")
    v[::101] = float("inf")
    v[::103] = 3e12
    cols = {"v": ColumnVector(v.cuda(), T.DoubleType()),
            "f": ColumnVector(v.float().cuda(), T.FloatType()),
            "i": ColumnVector((torch.randint(-1000, 1000, (n,), generator=g)).int().cuda(), T.IntegerType()),
            "l": ColumnVector((torch.randint(-10**12, 10**12, (n,), generator=g)).cuda(), T.LongType())}
    df = DataFrame(Table(cols, n, torch.device("cuda")), spark_gpu)
    exprs = {"a": (col("v") * 4).cast("int"), "b": col("v") + 1.5, "c": 3 - col("v"), "d": col("v") / 2,
             "e": (col("f") * 0.5).cast("long"), "g": (col("i") - 7).cast("int"), "h": col("l") * 3,
             "k": col("v").cast("int"), "m": col("i") * 2.5, "p": col("v") > 0.5, "q": col("i") == 7,
             "r": 10 <= col("l"), "s": col("v") * col("f")}  # (s: two columns -> the VM)

    def run(flag):
        monkeypatch.setenv("PTG_EXPR_SPECIALIZE", flag)
        out = df.select(*[e.alias(k) for k, e in exprs.items()])
        res = {}
        for k in exprs:
            cv = out._t.column(k)
            res[k] = (cv.data.cpu(), None if cv.valid is None else cv.valid.cpu())
        f = df.filter(col("v") >= 100.0)
        res["filter"] = (f._t.column("l").data.cpu(), None)
        torch.cuda.synchronize()
        return res

    before = _spec_launches()
    spec = run("1")
    used = _spec_launches() - before
    vm = run("0")
    assert _spec_launches() - before == used
    assert used >= len(exprs) - 1, used  # every single-column shape took the specialised kernels
    for k in spec:
        a, b = spec[k], vm[k]
        assert a[0].dtype == b[0].dtype, k
        assert torch.equal(a[0].contiguous().view(torch.uint8), b[0].contiguous().view(torch.uint8)), k  # NaN bits too
        assert (a[1] is None) == (b[1] is None) and (a[1] is None or torch.equal(a[1], b[1])), k
