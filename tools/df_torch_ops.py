"""Which torch (non-framework) device kernels the DataFrame operators of tools/df_ops_profile.py still
launch, and from where: runs the same queries (smaller --rows) under a TorchDispatchMode that records
every aten op touching a CUDA tensor that is not a view / metadata op, with the innermost call site in
pyspark_tf_gke_amd/.  Prints one JSON line per (op, site) with its count."""
import argparse
import collections
import json
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=2_000_000)
ap.add_argument("--multirank", action="store_true",
                help="the multi-rank path on one GPU: a 1-rank RCCL group with PTG_COLLECTIVES_WORLD1, so the "
                     "groupBy / orderBy shuffles (count matrix, p2p exchange, range split) run; only the "
                     "single-int64-key groupBy and the orderBy are recorded")
a = ap.parse_args()
if a.multirank:
    os.environ.update({"PTG_FORCE_PG": "1", "PTG_COLLECTIVES_WORLD1": "1", "RANK": "0", "WORLD_SIZE": "1",
                       "LOCAL_RANK": "0", "LOCAL_WORLD_SIZE": "1", "MASTER_ADDR": "127.0.0.1",
                       "MASTER_PORT": os.environ.get("MASTER_PORT", "29671")})

SKIP = ("view", "_unsafe_view", "alias", "empty", "empty_strided", "as_strided", "detach", "t", "transpose",
        "permute", "expand", "slice", "select", "unsqueeze", "squeeze", "reshape", "_reshape_alias", "split",
        "unbind", "lift_fresh", "_local_scalar_dense", "is_nonzero", "set_", "resize_", "narrow",
        "_to_copy_cpu")
counts: collections.Counter = collections.Counter()
PKG = os.sep + "pyspark_tf_gke_amd" + os.sep


class Rec(TorchDispatchMode):
    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        name = func.overloadpacket.__name__
        dev = any(isinstance(x, torch.Tensor) and x.is_cuda for x in list(args) + list(kwargs.values()))
        out = func(*args, **kwargs)
        outs = out if isinstance(out, (tuple, list)) else [out]
        dev = dev or any(isinstance(x, torch.Tensor) and x.is_cuda for x in outs)
        if dev and name not in SKIP:
            site = "?"
            for fr in reversed(traceback.extract_stack()[:-1]):
                if PKG in fr.filename:
                    site = f"{fr.filename.split(PKG)[-1]}:{fr.lineno} {fr.name}"
                    break
            counts[(name, site)] += 1
        return out


from pyspark_tf_gke_amd.ops import df as D  # noqa: E402
from pyspark_tf_gke_amd.sql import SparkSession  # noqa: E402
from pyspark_tf_gke_amd.sql import types as T  # noqa: E402
from pyspark_tf_gke_amd.sql.dataframe import DataFrame  # noqa: E402
from pyspark_tf_gke_amd.sql.functions import avg, col, count, countDistinct, max as fmax, sum as fsum  # noqa: E402
from pyspark_tf_gke_amd.sql.table import ColumnVector, Table  # noqa: E402

spark = SparkSession.builder.master("local[1]").config("spark.ptg.device", "cuda").getOrCreate()
HEALTH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "data", "health.csv")
df = spark.read.csv(HEALTH, header=True, inferSchema=True)
df.count()
k, v = D.fill_synthetic_kv(a.rows, 1000, "cuda")
big = DataFrame(Table({"k": ColumnVector(k, T.LongType()), "v": ColumnVector(v, T.DoubleType())}, a.rows, k.device),
                spark)
torch.cuda.synchronize()
if a.multirank:
    from pyspark_tf_gke_amd.parallel import comm  # noqa: E402

    comm.init()
    assert comm.distributed()
    big.groupBy("k").agg(count("*").alias("n"), fsum("v").alias("s"))._t.num_rows  # warm (plans, buffers)
    torch.cuda.synchronize()
    with Rec():
        g = big.groupBy("k").agg(count("*").alias("n"), fsum("v").alias("s"))
        g._t.num_rows
        o = big.orderBy(col("v").desc())
        o._t.num_rows
    torch.cuda.synchronize()
    print(json.dumps({"multirank": True, "groups": int(g._t.num_rows), "sorted_rows": int(o._t.num_rows)}))
    for (name, site), c in counts.most_common():
        print(json.dumps({"op": name, "count": c, "site": site}))
    sys.exit(0)
with Rec():
    df.groupBy("measure_name", "subpopulation").agg(count("*").alias("n"), avg("value").alias("m"),
                                                    fsum("value").alias("s"), fmax("upper_ci").alias("hi")).collect()
    df.agg(countDistinct("subpopulation"), countDistinct("value"), countDistinct("state_name")).collect()
    df.dropDuplicates(["measure_name", "subpopulation"]).collect()
    df.select("measure_name", "state_name").distinct().count()
    big.groupBy(col("k"), (col("v") * 4).cast("int").alias("b")).agg(count("*").alias("n"), fsum("v").alias("s")).count()
    big.orderBy("k").limit(5).collect()
for (name, site), c in counts.most_common():
    print(json.dumps({"op": name, "count": c, "site": site}))
