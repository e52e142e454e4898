"""CPU: pin the oracle (both restatements) against the known-answer tests and golden
fixtures before anything is checked against it."""
import glob
import json
import os
import struct

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import spark_semantics as S


def kats():
    with open(os.path.join(GOLDEN, "kats.json")) as f:
        return json.load(f)


def test_long_hash_kats_python_and_c(oracle_lib):
    L = oracle_lib.lib()
    for k, h in kats()["long_hash"]:
        assert S.java_long_hash(k) == h
        assert L.orc_java_long_hash(k) == h


def test_pid_kats(oracle_lib):
    L = oracle_lib.lib()
    for k, r, p in kats()["hash_pid"]:
        assert S.hash_partition(k, r) == p
        assert L.orc_hash_partition(k, r) == p
    for x, m, v in kats()["non_negative_mod"]:
        assert S.non_negative_mod(x, m) == v
        assert L.orc_non_negative_mod(x, m) == v


def test_edge_pids_c_matches_python(oracle_lib):
    L = oracle_lib.lib()
    for k, r, p in kats()["edge_pids"]:
        assert L.orc_hash_partition(k, r) == p == S.hash_partition(k, r)
        assert 0 <= p < r


def test_scala_hash_is_not_used():
    # Scala's (-1L).## is -1; Java's Long.hashCode(-1) is 0.
    assert S.java_long_hash(-1) == 0
    assert S.hash_partition(-1, 1024) == 0


def test_splitmix_generator_kats(oracle_lib):
    L = oracle_lib.lib()
    for seed, i, v in kats()["splitmix64"]:
        assert S.splitmix64_at(seed, i) == v == L.orc_splitmix64_at(seed, i)


def test_block_id_wire_format():
    for m, r, hx in kats()["block_id_bytes"]:
        assert S.ucx_block_id_bytes(m, r).hex() == hx


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "hash_*.npz"))))
def test_c_oracle_reproduces_hash_fixtures(oracle_lib, path):
    z = np.load(path)
    R = int(z["num_partitions"])
    recs = z["records"]
    assert np.array_equal(oracle_lib.partition_ids(recs, R), z["pids"])
    out, counts = oracle_lib.map_write(recs, R)
    assert np.array_equal(out, z["out"])
    assert np.array_equal(counts * 16, z["lengths"])
    assert oracle_lib.index_bytes(z["lengths"]) == z["index"].tobytes()
    out4, counts4 = oracle_lib.map_write(recs, R, nthreads=4)
    assert np.array_equal(out4, out) and np.array_equal(counts4, counts)


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "range_*.npz"))))
def test_c_oracle_reproduces_range_fixtures(oracle_lib, path):
    z = np.load(path)
    R = int(z["num_partitions"])
    kind = oracle_lib.PART_RANGE_BYTES10 if z["records"].shape[1] == 100 else oracle_lib.PART_RANGE_I64
    pids = oracle_lib.partition_ids(z["records"], R, kind, z["bounds"], bool(z["ascending"]))
    assert np.array_equal(pids, z["pids"])
    out, counts = oracle_lib.map_write(z["records"], R, kind, z["bounds"], bool(z["ascending"]), nthreads=3)
    assert np.array_equal(out, z["out"])
    assert np.array_equal(counts * z["records"].shape[1], z["lengths"])


def test_range_partition_semantics_small():
    b = [10, 20, 30]
    # upper bounds are inclusive: k == bound goes to that bound's partition
    assert [S.range_partition(k, b) for k in (5, 10, 11, 20, 30, 31)] == [0, 0, 1, 1, 2, 3]
    assert [S.range_partition(k, b, ascending=False) for k in (5, 31)] == [3, 0]
    big = list(range(0, 2000, 10))  # > 128 bounds: binary-search path
    assert S.range_partition(10, big) == 1 and S.range_partition(11, big) == 2
    assert S.range_partition(10**9, big) == len(big)


def test_index_layout_and_validation(oracle_lib):
    lengths = np.array([16, 0, 32, 48], np.int64)
    idx = oracle_lib.index_bytes(lengths)
    assert idx == S.index_file_bytes(lengths.tolist())
    assert struct.unpack(">5q", idx) == (0, 16, 16, 48, 96)
    assert S.check_index_and_data(idx, 96, 4) == [16, 0, 32, 48]
    assert S.check_index_and_data(idx, 95, 4) is None
    assert S.check_index_and_data(idx, 96, 3) is None
    assert S.check_index_and_data(struct.pack(">q", 8) + idx[8:], 96, 4) is None
    assert S.block_range(idx, 2, 3) == (16, 32)
    assert S.block_range(idx, 0, 4) == (0, 96)
    assert S.ucx_registered_blocks([16, 0, 32]) == [(0, 0, 16), (2, 16, 32)]


def test_uniform_generator_c_matches_python(oracle_lib):
    a = oracle_lib.gen_uniform16(777, 123, value_base=5)
    b = S.pack_records16(S.gen_uniform_records(777, 123, 5))
    assert a.tobytes() == b


def test_zipf_head_mass(oracle_lib):
    cdf = oracle_lib.zipf_cdf(1.1, 2**16)
    recs = oracle_lib.gen_zipf16(200_000, 9, cdf)
    keys = recs[:, :8].copy().view(np.int64).ravel()
    assert keys.min() >= 1 and keys.max() <= 2**16
    assert abs(np.mean(keys == 1) - cdf[0]) < 0.01


def test_multithreaded_equals_single_threaded(oracle_lib):
    recs = oracle_lib.gen_uniform16(300_001, 77)
    for R in (1, 200, 1024, 4096):
        a, ca = oracle_lib.map_write(recs, R, nthreads=1)
        b, cb = oracle_lib.map_write(recs, R, nthreads=7)
        assert np.array_equal(a, b) and np.array_equal(ca, cb)
        # stability: values (= input index) ascend inside every partition run
        vals = a[:, 8:].copy().view(np.int64).ravel()
        o = oracle_lib.offsets(ca)
        for p in range(0, R, max(1, R // 17)):
            run = vals[o[p]:o[p + 1]]
            assert np.all(np.diff(run) > 0)


def test_range_partitioner_matches_bisect_on_distinct_bounds(oracle_lib):
    """RangePartitioner.getPartition (linear scan up to 128 bounds, Arrays.binarySearch above)
    returns, for Spark's distinct sorted bounds, the first bound >= key -- Python's
    bisect_left, an implementation outside this repository; descending order mirrors it.
    Long keys (signed order) and TeraSort's 10-byte keys (unsigned lexicographic order),
    with exact hits on bounds.  (Duplicate bounds, where the JDK's probe order decides, stay
    pinned by the restatement only.)"""
    import bisect

    rng = np.random.default_rng(17)
    for nb in (1, 7, 128, 129, 1023):
        b = np.unique(rng.integers(-(2**62), 2**62, nb * 2))[:nb].astype(np.int64)
        keys = np.concatenate([rng.integers(-(2**63), 2**63 - 1, 3000, dtype=np.int64), b, b + 1, b - 1])
        recs = np.zeros((len(keys), 16), np.uint8)
        recs[:, :8] = keys.view(np.uint8).reshape(-1, 8)
        for asc in (True, False):
            got = oracle_lib.partition_ids(recs, nb + 1, oracle_lib.PART_RANGE_I64, b, asc)
            want = np.array([bisect.bisect_left(b.tolist(), int(k)) for k in keys])
            assert np.array_equal(got, want if asc else nb - want), (nb, asc)
    for nb in (5, 128, 300):
        raw = rng.integers(0, 256, size=(nb * 3, 10), dtype=np.uint8)
        bl = sorted({bytes(r) for r in raw})[:nb]
        b10 = np.frombuffer(b"".join(bl), np.uint8).reshape(-1, 10)
        recs = oracle_lib.gen_terasort100(4000, nb)
        recs[:nb, :10] = b10  # exact hits
        for asc in (True, False):
            got = oracle_lib.partition_ids(recs, len(bl) + 1, oracle_lib.PART_RANGE_BYTES10, b10, asc)
            want = np.array([bisect.bisect_left(bl, bytes(r[:10])) for r in recs])
            assert np.array_equal(got, want if asc else len(bl) - want), (nb, asc)


def test_stable_group_by_partition_matches_numpy_stable_sort(oracle_lib):
    """a4's stable group-by-partition (ExternalSorter / ShuffleInMemorySorter: partition-
    contiguous, map input order inside a partition) equals numpy's stable argsort of the
    partition ids -- an independent stable sort -- for hash and range partitioners, with and
    without threads; counts equal numpy's bincount."""
    rng = np.random.default_rng(23)
    for n, R in ((1, 1), (1000, 3), (50_000, 200), (200_003, 1024)):
        recs = oracle_lib.gen_uniform16(n, 900 + R)
        recs[: n // 3, :8] = recs[: 1, :8]  # many equal keys: order must come from the input
        for nt in (1, 4):
            out, counts = oracle_lib.map_write(recs, R, nthreads=nt)
            pids = oracle_lib.partition_ids(recs, R)
            order = np.argsort(pids, kind="stable")
            assert np.array_equal(out, recs[order]) and np.array_equal(counts, np.bincount(pids, minlength=R))
    b = np.sort(rng.integers(-(2**62), 2**62, 99)).astype(np.int64)
    recs = oracle_lib.gen_uniform16(30_000, 5)
    out, counts = oracle_lib.map_write(recs, 100, oracle_lib.PART_RANGE_I64, b)
    pids = oracle_lib.partition_ids(recs, 100, oracle_lib.PART_RANGE_I64, b)
    assert np.array_equal(out, recs[np.argsort(pids, kind="stable")])
