import numpy as np

from pyspark_tf_gke_amd.data import AUTOTUNE, Dataset


def test_from_tensor_slices_batch_repeat_shard():
    X = np.arange(10, dtype=np.float32).reshape(10, 1)
    y = np.arange(10, dtype=np.int32)
    ds = Dataset.from_tensor_slices((X, y))
    assert ds.cardinality() == 10
    b = list(ds.batch(4))
    assert [len(x[1]) for x in b] == [4, 4, 2]
    assert len(list(ds.batch(4, drop_remainder=True))) == 2
    s0 = [int(e[1]) for e in ds.shard(3, 0)]
    s1 = [int(e[1]) for e in ds.shard(3, 1)]
    assert s0 == [0, 3, 6, 9] and s1 == [1, 4, 7]
    it = iter(ds.batch(4).repeat())
    got = [next(it)[1].tolist() for _ in range(4)]
    assert got[3] == [0, 1, 2, 3]


def test_shuffle_is_permutation_and_reshuffles():
    ds = Dataset.range(100).shuffle(30, seed=7)
    a, b = [int(x) for x in ds], [int(x) for x in ds]
    assert sorted(a) == list(range(100)) and sorted(b) == list(range(100))
    assert a != list(range(100)) and a != b


def test_map_parallel_prefetch_zip_take_skip():
    ds = Dataset.range(20).map(lambda x: x * 2, num_parallel_calls=AUTOTUNE).prefetch(2)
    assert [int(x) for x in ds] == [2 * i for i in range(20)]
    z = Dataset.zip((Dataset.range(5), Dataset.range(5).map(lambda v: v + 10)))
    assert [(int(a), int(b)) for a, b in z] == [(i, i + 10) for i in range(5)]
    assert [int(x) for x in Dataset.range(10).skip(3).take(2)] == [3, 4]
    assert [int(x) for x in Dataset.range(10).filter(lambda v: v % 2 == 0)] == [0, 2, 4, 6, 8]
