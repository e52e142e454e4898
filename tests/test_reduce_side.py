"""Reduce side after the fetch (UcxShuffleReader.scala:137-191): sortByKey / TeraSort
(dep.keyOrdering) and groupByKey / reduceByKey(_ + _) (dep.aggregator, mapSideCombine =
false) on the GPU, against the oracle's restatement (oracle.reduce_sorted /
oracle.reduce_grouped).

CPU tests pin the oracle's reduce-side functions to plain-Python restatements of Spark's
semantics (stable TimSort order; CompactBuffer append order; wrapping Long sums).  GPU tests
(marked gpu) run the engine through the C ABI: bit-exact sorted bytes, identical keys /
group starts / values / sums."""
import numpy as np
import pytest

# ---------------------------------------------------------------- CPU: oracle pinning --


def _py_groupbykey(pairs):
    """ExternalAppendOnlyMap + CompactBuffer, restated with a dict (insertion-ordered values)."""
    d = {}
    for k, v in pairs:
        d.setdefault(k, []).append(v)
    return d


def _records16(keys, vals):
    a = np.empty((len(keys), 16), np.uint8)
    a[:, :8] = np.asarray(keys, dtype="<i8").reshape(-1, 1).view(np.uint8)
    a[:, 8:] = np.asarray(vals, dtype="<i8").reshape(-1, 1).view(np.uint8)
    return a


def test_oracle_sort_is_stable_signed(oracle_lib):
    keys = [3, -1, 3, -(2**63), 2**63 - 1, -1, 0, 3]
    recs = _records16(keys, range(len(keys)))
    got = oracle_lib.reduce_sorted([recs])
    want = sorted(zip(keys, range(len(keys))), key=lambda kv: kv[0])  # Python sort is stable
    assert np.array_equal(got, _records16([k for k, _ in want], [v for _, v in want]))


def test_oracle_sort_terasort_unsigned_lex(oracle_lib):
    rng = np.random.default_rng(5)
    recs = rng.integers(0, 256, size=(300, 100), dtype=np.uint8)
    recs[:40, :10] = recs[0, :10]  # duplicates: stability matters
    recs[40:60, 0] = 0xFF          # high bytes sort last (unsigned)
    got = oracle_lib.reduce_sorted([recs])
    order = sorted(range(len(recs)), key=lambda i: bytes(recs[i, :10]))  # stable
    assert np.array_equal(got, recs[order])


@pytest.mark.parametrize("agg", ["group", "sum"])
def test_oracle_grouped_matches_dict(oracle_lib, agg):
    rng = np.random.default_rng(11)
    seqs = []
    for _ in range(3):
        n = int(rng.integers(0, 200))
        keys = rng.integers(-6, 6, size=n)
        vals = rng.integers(-(2**63), 2**63 - 1, size=n, dtype=np.int64)
        seqs.append(_records16(keys, vals))
    res = oracle_lib.reduce_grouped(seqs, agg)
    base = 0
    for gi, s in enumerate(seqs):
        k = s[:, :8].copy().view("<i8").reshape(-1).tolist()
        v = s[:, 8:].copy().view("<i8").reshape(-1).tolist()
        d = _py_groupbykey(zip(k, v))
        for key in sorted(d):
            if agg == "group":
                keys, starts, vals = res
                g = np.nonzero((starts >= base) & (keys == key))[0][0]
                st = starts[g]
                assert vals[st:st + len(d[key])].tolist() == d[key]
            else:
                keys, sums = res
                total = sum(d[key]) % 2**64
                total = total - 2**64 if total >= 2**63 else total
                idx = [i for i in range(len(keys)) if keys[i] == key]
                assert any(int(sums[i]) == total for i in idx)
        base += len(k)


# ---------------------------------------------------------------- GPU parity ----------
_sid = [5000]


def _run(sgx_lib, oracle_lib, maps, R, kind=0, bounds=None, ascending=True, rng_part=None, agg=None, flags=0):
    """Write `maps` (list of record arrays) as map ids 0..M-1, read [r0, r1) back on the
    GPU (sorted, or grouped with `agg`), compare with the oracle."""
    _sid[0] += 1
    sid = _sid[0]
    rb = maps[0].shape[1]
    r0, r1 = rng_part or (0, R)
    with sgx_lib.ShuffleEngine(device=0, num_chunks=5, flags=flags) as e:
        e.register_shuffle(sid, R, kind, bounds, ascending, rb)
        outs = []
        for mid, recs in enumerate(maps):
            e.write_map(sid, mid, np.ascontiguousarray(recs), len(recs), rb, R)
            outs.append(oracle_lib.map_write(recs, R, kind, bounds, ascending))
        seqs = oracle_lib.canonical_reducer_sequences(outs, R, rb)[r0:r1]
        mids = list(range(len(maps)))
        if agg is None:
            got = e.read_sorted(sid, mids, r0, r1).reshape(-1, rb)
            want = oracle_lib.reduce_sorted(seqs) if seqs else np.empty((0, rb), np.uint8)
            assert got.shape == want.shape
            if not np.array_equal(got, want):
                bad = np.nonzero(np.any(got != want, axis=1))[0]
                pytest.fail(f"{len(bad)} sorted records differ, first at {bad[:5]}")
        else:
            a = sgx_lib.AGG_SUM if agg == "sum" else sgx_lib.AGG_GROUP
            got = e.read_grouped(sid, mids, r0, r1, a)
            want = oracle_lib.reduce_grouped(seqs, agg)
            assert len(got) == len(want)
            for g, w in zip(got, want):
                assert np.array_equal(g, w)
        e.unregister_shuffle(sid)


def _zipfish(rng, n, K=50):
    keys = (rng.zipf(1.3, size=n) % K) - K // 3  # heavy duplicates, negatives
    return _records16(keys, rng.integers(-(2**63), 2**63 - 1, size=n, dtype=np.int64))


@pytest.mark.gpu
@pytest.mark.parametrize("R", [1, 7, 256, 1024, 4096])
def test_sorted_hash_uniform(sgx_lib, oracle_lib, R):
    maps = [oracle_lib.gen_uniform16(n, 100 + i, value_base=i << 32) for i, n in enumerate((30_000, 0, 17_777))]
    _run(sgx_lib, oracle_lib, maps, R)


@pytest.mark.gpu
@pytest.mark.parametrize("R", [3, 1024])
def test_sorted_hash_duplicates_and_signs(sgx_lib, oracle_lib, R):
    rng = np.random.default_rng(R)
    maps = [_zipfish(rng, 20_000), _zipfish(rng, 5_001)]
    maps[0][:3, :8] = np.array([-(2**63), 2**63 - 1, -1], dtype="<i8").reshape(-1, 1).view(np.uint8)
    _run(sgx_lib, oracle_lib, maps, R)
    _run(sgx_lib, oracle_lib, maps, R, rng_part=(1, R) if R > 1 else (0, 1))


@pytest.mark.gpu
@pytest.mark.parametrize("ascending", [True, False])
def test_sorted_range_i64(sgx_lib, oracle_lib, ascending):
    rng = np.random.default_rng(3)
    maps = [_zipfish(rng, 12_000, K=5000), oracle_lib.gen_uniform16(9_000, 7)]
    allk = np.concatenate([m[:, :8].copy().view("<i8").reshape(-1) for m in maps])
    bounds = np.unique(np.sort(rng.choice(allk, 63)))
    _run(sgx_lib, oracle_lib, maps, len(bounds) + 1, sgx_lib.PART_RANGE_I64, bounds, ascending)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["range", "hash"])
def test_sorted_terasort(sgx_lib, oracle_lib, kind):
    maps = [oracle_lib.gen_terasort100(n, 40 + i) for i, n in enumerate((6_000, 2_345))]
    maps[0][100:400, :10] = maps[0][99, :10]  # duplicate keys across a tile: stability
    R = 64
    if kind == "range":
        rng = np.random.default_rng(1)
        sample = np.concatenate(maps)[rng.choice(8345, 20 * R, replace=False), :10]
        sample = sample[np.lexsort(sample.T[::-1])]
        bounds = np.ascontiguousarray(sample[np.linspace(0, len(sample) - 1, R - 1).astype(int)])
        _run(sgx_lib, oracle_lib, maps, R, sgx_lib.PART_RANGE_BYTES10, bounds)
    else:
        _run(sgx_lib, oracle_lib, maps, R)


@pytest.mark.gpu
@pytest.mark.parametrize("agg", ["group", "sum"])
@pytest.mark.parametrize("R", [1, 200, 1024])
def test_grouped(sgx_lib, oracle_lib, agg, R):
    rng = np.random.default_rng(R + len(agg))
    maps = [_zipfish(rng, 40_000, K=3000), oracle_lib.gen_uniform16(10_000, 9), _zipfish(rng, 1)]
    _run(sgx_lib, oracle_lib, maps, R, agg=agg)


@pytest.mark.gpu
@pytest.mark.parametrize("agg", ["group", "sum"])
@pytest.mark.parametrize("shape", ["spanning", "tile_aligned", "unique", "one"])
def test_grouped_tile_shapes(sgx_lib, oracle_lib, agg, shape):
    """The one-pass grouping (k_group_fused: 4096-record tiles, a look-back over tiles) on
    group sizes that stress its tile boundaries: groups spanning several tiles (the sum is
    carried), groups starting exactly on tile boundaries, every key unique, one record.
    Values near +-2^63, so the Long sums wrap."""
    T = 4096
    sizes = {"spanning": [1, T - 1, 3 * T + 17, 5, 2 * T, T + 1, 2, 7 * T - 3, 1],
             "tile_aligned": [T, T, 1, T - 1, 2 * T, T],
             "unique": [1] * (2 * T + 1),
             "one": [1]}[shape]
    rng = np.random.default_rng(len(sizes))
    keys = np.repeat(np.arange(len(sizes), dtype=np.int64) * 7 - 10, sizes)
    vals = rng.integers(2**62, 2**63 - 1, size=len(keys), dtype=np.int64) * rng.choice([-1, 1], size=len(keys))
    perm = rng.permutation(len(keys))
    recs = _records16(keys[perm], vals[perm])
    _run(sgx_lib, oracle_lib, [recs[: len(recs) // 2], recs[len(recs) // 2:]], 1, agg=agg)


@pytest.mark.gpu
def test_grouped_empty_range(sgx_lib, oracle_lib):
    maps = [oracle_lib.gen_uniform16(1000, 1)]
    _run(sgx_lib, oracle_lib, maps, 16, rng_part=(5, 5), agg="group")
    _run(sgx_lib, oracle_lib, maps, 16, rng_part=(5, 5))


@pytest.mark.gpu
def test_reader_dispatch(sgx_lib, oracle_lib, tmp_path):
    """UcxShuffleReader.read picks the path from the dependency (aggregator / keyOrdering)."""
    recs = _zipfish(np.random.default_rng(0), 5000, K=100)
    mgr = sgx_lib.UcxShuffleManager(device=0, localDir=str(tmp_path))
    try:
        out, cnt = oracle_lib.map_write(recs, 8)
        seqs = oracle_lib.canonical_reducer_sequences([(out, cnt)], 8, 16)
        for sid, dep in enumerate([
                sgx_lib.ShuffleDependency(sgx_lib.HashPartitioner(8), 16, keyOrdering=True),
                sgx_lib.ShuffleDependency(sgx_lib.HashPartitioner(8), 16, aggregator=sgx_lib.Aggregator("group")),
                sgx_lib.ShuffleDependency(sgx_lib.HashPartitioner(8), 16, aggregator=sgx_lib.Aggregator("sum"))]):
            h = mgr.registerShuffle(sid, dep)
            w = mgr.getWriter(h, 0)
            w.write(recs)
            w.stop(True)
            got = mgr.getReader(h, 2, 6).read()
            if dep.keyOrdering:
                assert np.array_equal(got, oracle_lib.reduce_sorted(seqs[2:6]))
            else:
                want = oracle_lib.reduce_grouped(seqs[2:6], dep.aggregator.kind)
                for g, wv in zip(got, want):
                    assert np.array_equal(g, wv)
    finally:
        mgr.stop()


@pytest.mark.gpu
@pytest.mark.parametrize("skip", ["1", "0"])
@pytest.mark.parametrize("keys", ["small_nonneg", "all_equal", "two_values_high_byte"])
def test_sorted_trivial_digits(sgx_lib, oracle_lib, skip, keys):
    """Digit passes whose byte is constant over the fetched keys are skipped (the default;
    SGX_FLAG_SORT_ALL_DIGITS runs them all); the result must not depend on it."""
    flags = 0 if skip == "1" else sgx_lib.FLAG_SORT_ALL_DIGITS
    rng = np.random.default_rng(len(keys))
    n = 30_000
    if keys == "small_nonneg":
        k = rng.integers(0, 3000, size=n)
    elif keys == "all_equal":
        k = np.full(n, -12345)
    else:
        k = np.where(rng.random(n) < 0.5, 1 << 56, -(1 << 60)) + 7
    maps = [_records16(k[: n // 2], rng.integers(0, 1 << 62, size=n // 2)),
            _records16(k[n // 2:], rng.integers(0, 1 << 62, size=n - n // 2))]
    for R in (1, 16):
        _run(sgx_lib, oracle_lib, maps, R, flags=flags)
        _run(sgx_lib, oracle_lib, maps, R, agg="group", flags=flags)


@pytest.mark.gpu
@pytest.mark.slow
@pytest.mark.parametrize("codec", ["fixed", "kryo+lz4"])
def test_c0_groupbykey_full_size(sgx_lib, oracle_lib, codec, tmp_path):
    """BASELINE config C0 at its size: groupByKey of 10M (Long, Long) records -- two map
    shards of 5M (the two executors of local-cluster[2,1,2048]) -- to 200 reducers through
    UcxShuffleManager -> getWriter -> getReader().read() (the GroupByTest shapes of
    buildlib/test.sh:163-173; combineValuesByKey, spark_3_0/UcxShuffleReader.scala:155-164),
    with the engine's fixed codec and with Spark's KryoSerializer + spark.shuffle.compress
    (LZ4), against oracle.reduce_grouped."""
    n, R, seed = 10_000_000, 200, 0x5EEDC0DE
    recs = oracle_lib.gen_uniform16(n, seed)
    conf = {"spark.shuffle.compress": "true" if codec != "fixed" else "false"}
    mgr = sgx_lib.UcxShuffleManager(conf=conf, localDir=str(tmp_path))
    try:
        dep = sgx_lib.ShuffleDependency(sgx_lib.HashPartitioner(R), 16, aggregator=sgx_lib.Aggregator("group"),
                                        serializer="fixed" if codec == "fixed" else "kryo")
        h = mgr.registerShuffle(0, dep)
        outs = []
        for m in range(2):
            shard = recs[m * (n // 2):(m + 1) * (n // 2)]
            w = mgr.getWriter(h, m)
            w.write(shard)
            out, counts = oracle_lib.map_write(shard, R, nthreads=8)
            outs.append((out, counts))
            if codec == "fixed":
                assert np.array_equal(w.getPartitionLengths(), counts * 16)
        keys, starts, values = mgr.getReader(h, 0, R).read()
        seqs = oracle_lib.canonical_reducer_sequences(outs, R, 16)
        wk, ws, wv = oracle_lib.reduce_grouped(seqs, "group")
        assert np.array_equal(keys, wk)
        assert np.array_equal(starts, ws)
        assert np.array_equal(values, wv)
        assert len(values) == n
    finally:
        mgr.stop()


@pytest.mark.gpu
def test_size_query_result_reuse_and_invalidation(sgx_lib, oracle_lib):
    """A size query computes the read and the filling call right after it reuses it; any call
    in between on the thread, or any change to the engine's shuffles, makes the filling call
    recompute.  Results always equal the oracle's; device outputs equal host outputs."""
    import ctypes

    from sparkucx_amd._lib import lib

    e = sgx_lib.ShuffleEngine(device=0)
    R = 64
    sid = 71
    e.register_shuffle(sid, R, serializer=sgx_lib.SER_KRYO)
    recs = [oracle_lib.gen_uniform16(40_000, 900 + i, value_base=i << 32) for i in range(2)]
    recs[1][:, :8] = recs[0][:, :8]  # shared keys: real groups
    for i, r in enumerate(recs):
        e.write_map(sid, i, r, len(r), 16)
    outs = [oracle_lib.map_write(r, R) for r in recs]
    seqs = oracle_lib.canonical_reducer_sequences(outs, R, 16)

    def want(r0, r1, agg):
        return oracle_lib.reduce_grouped(seqs[r0:r1], agg)

    m = np.array([0, 1], np.int64)

    def query(r0, r1, agg):
        ng, nv = ctypes.c_int64(), ctypes.c_int64()
        sgx_lib._lib.check(lib().sgx_read_grouped(e.handle, sid, m.ctypes.data, 2, r0, r1, agg, None, None, None,
                                                  0, 0, 0, ctypes.byref(ng), ctypes.byref(nv)), "q")
        return ng.value, nv.value

    def fill(r0, r1, agg, G, V):
        k, s, v = np.empty(G, np.int64), np.empty(G, np.int64), np.empty(V, np.int64)
        ng, nv = ctypes.c_int64(), ctypes.c_int64()
        sgx_lib._lib.check(lib().sgx_read_grouped(e.handle, sid, m.ctypes.data, 2, r0, r1, agg, k.ctypes.data,
                                                  s.ctypes.data, v.ctypes.data, G, V, 0, ctypes.byref(ng),
                                                  ctypes.byref(nv)), "f")
        return (k, s, v) if agg == sgx_lib.AGG_GROUP else (k, v)

    try:
        # reuse: query then fill
        G, V = query(0, 32, sgx_lib.AGG_GROUP)
        for g, w in zip(fill(0, 32, sgx_lib.AGG_GROUP, G, V), want(0, 32, "group")):
            assert np.array_equal(g, w)
        # another call on the thread in between: the fill recomputes its own range
        G, V = query(0, 32, sgx_lib.AGG_SUM)
        query(32, 64, sgx_lib.AGG_SUM)
        for g, w in zip(fill(0, 32, sgx_lib.AGG_SUM, G, V), want(0, 32, "sum")):
            assert np.array_equal(g, w)
        # a write in between (another map id): recomputed, still the two maps asked for
        G, V = query(16, 48, sgx_lib.AGG_GROUP)
        e.write_map(sid, 9, recs[0][:1000], 1000, 16)
        for g, w in zip(fill(16, 48, sgx_lib.AGG_GROUP, G, V), want(16, 48, "group")):
            assert np.array_equal(g, w)
        # the Python wrapper (size query + fill) and device outputs
        for agg in ("group", "sum"):
            a = sgx_lib.AGG_GROUP if agg == "group" else sgx_lib.AGG_SUM
            host = e.read_grouped(sid, [0, 1], 0, R, a)
            dev = e.read_grouped(sid, [0, 1], 0, R, a, device=True)
            try:
                for h, d, w in zip(host, dev, want(0, R, agg)):
                    assert np.array_equal(h, w)
                    assert np.array_equal(d.to_numpy(len(w) * 8).view(np.int64), w)
            finally:
                for d in dev:
                    d.free()
        # sorted / records reads of the Kryo shuffle (size query decodes and keeps the result)
        got = e.read_sorted(sid, [0, 1], 0, R).reshape(-1, 16)
        assert np.array_equal(got, oracle_lib.reduce_sorted(seqs))
        got = e.read_records(sid, [0, 1], 0, R).reshape(-1, 16)
        assert np.array_equal(got, np.concatenate(seqs))
    finally:
        e.close()


@pytest.mark.gpu
# bucket path / SGX_FLAG_NO_BUCKET_SORT (digit passes only) / SGX_FLAG_ASSUME_LDS_DISORDER (every
# pass ballot-ranked on the per-lane kernel: the fallback if the engine-start check fails)
@pytest.mark.parametrize("flags", [0, 64, 128])
@pytest.mark.parametrize("case", ["hash16_R1", "hash16_R7", "hash16_R1024", "hash16_R4096", "range16_asc",
                                  "range16_desc", "tera_range", "tera_hash", "dups_in_bucket", "long_bucket"])
def test_sorted_bucket_path(sgx_lib, oracle_lib, flags, case):
    """The sorted read's bucket path (key-window passes -> partitioner pass -> every (P, window)
    bucket sorted on chip) against the oracle, at sizes where the window takes one or two
    passes, for hash and range partitioners, 16 B and TeraSort 100 B records; equal keys
    inside a bucket (stability on chip), and a bucket longer than the chip's halo (the kernel
    gives up and the digit passes finish from its input)."""
    rng = np.random.default_rng(sum(map(ord, case)))
    if case.startswith("hash16"):
        R = int(case.split("_R")[1])
        maps = [oracle_lib.gen_uniform16(n, 500 + i, value_base=i << 32) for i, n in enumerate((300_001, 77_777))]
        _run(sgx_lib, oracle_lib, maps, R, flags=flags)
    elif case.startswith("range16"):
        maps = [oracle_lib.gen_uniform16(n, 600 + i) for i, n in enumerate((250_000, 50_000))]
        allk = np.concatenate([m[:, :8].copy().view("<i8").reshape(-1) for m in maps])
        bounds = np.unique(np.sort(rng.choice(allk, 255)))
        _run(sgx_lib, oracle_lib, maps, len(bounds) + 1, sgx_lib.PART_RANGE_I64, bounds, case.endswith("asc"),
             flags=flags)
    elif case.startswith("tera"):
        maps = [oracle_lib.gen_terasort100(n, 700 + i) for i, n in enumerate((120_000, 30_001))]
        maps[0][1000:1100, :10] = maps[0][999, :10]  # 101 equal keys: one bucket, stable on chip
        R = 128
        if case == "tera_range":
            sample = np.concatenate(maps)[rng.choice(150_001, 20 * R, replace=False), :10]
            sample = sample[np.lexsort(sample.T[::-1])]
            bounds = np.ascontiguousarray(sample[np.linspace(0, len(sample) - 1, R - 1).astype(int)])
            _run(sgx_lib, oracle_lib, maps, R, sgx_lib.PART_RANGE_BYTES10, bounds, flags=flags)
        else:
            _run(sgx_lib, oracle_lib, maps, R, flags=flags)
    elif case == "dups_in_bucket":
        recs = oracle_lib.gen_uniform16(400_000, 800)
        recs[::7, :8] = recs[1::7][:len(recs[::7]), :8]  # pairs of equal keys everywhere
        recs[5000:5200, :8] = recs[4999, :8]              # 200 equal keys
        _run(sgx_lib, oracle_lib, [recs], 1024, flags=flags)
    else:  # long_bucket: 3000 equal keys in one reducer -> longer than the halo -> fallback
        recs = oracle_lib.gen_uniform16(300_000, 900)
        recs[10_000:13_000, :8] = recs[9_999, :8]
        _run(sgx_lib, oracle_lib, [recs], 256, flags=flags)


@pytest.mark.gpu
@pytest.mark.parametrize("flags", [0, 1024])
@pytest.mark.parametrize("case", ["pieces", "subrange", "many_pieces", "grouped_sum", "empty_partitions"])
def test_sorted_segmented_window(sgx_lib, oracle_lib, flags, case):
    """The sorted read's segmented window pass (one stable pass by the key window inside every
    partition's segment of the gathered records) against the oracle, and the
    LSD form it replaces (SGX_FLAG_NO_SEG_WINDOW = 1024): partitions of several 2^17-record
    pieces, a sub-range of reducers, two partitions of ten pieces each, reduceByKey sums, and
    empty partitions between full ones."""
    if case == "pieces":  # 4 reducers x ~200 K records: two pieces each
        maps = [oracle_lib.gen_uniform16(n, 1000 + i, value_base=i << 32) for i, n in enumerate((500_001, 300_000))]
        _run(sgx_lib, oracle_lib, maps, 4, flags=flags)
    elif case == "subrange":
        maps = [oracle_lib.gen_uniform16(n, 1100 + i, value_base=i << 32) for i, n in enumerate((400_000, 123_457))]
        _run(sgx_lib, oracle_lib, maps, 64, rng_part=(5, 41), flags=flags)
    elif case == "many_pieces":  # 2 reducers x 1.25 M records: 10 pieces each
        maps = [oracle_lib.gen_uniform16(2_500_000, 1200)]
        _run(sgx_lib, oracle_lib, maps, 2, flags=flags)
    elif case == "grouped_sum":
        rng = np.random.default_rng(1300)
        keys = rng.integers(0, 1 << 40, size=600_000, dtype=np.int64)
        keys[::3] = keys[1::3][: len(keys[::3])]
        maps = [_records16(keys, rng.integers(-(2**40), 2**40, size=len(keys), dtype=np.int64))]
        _run(sgx_lib, oracle_lib, maps, 32, agg="sum", flags=flags)
    else:  # keys that hash to 3 of 16 reducers only: 13 empty segments
        rng = np.random.default_rng(1400)
        keys = rng.choice(np.array([1, 2, 3], dtype=np.int64), size=400_000) + 16 * rng.integers(0, 1 << 26, size=400_000)
        maps = [_records16(keys, np.arange(len(keys), dtype=np.int64))]
        _run(sgx_lib, oracle_lib, maps, 16, flags=flags)
