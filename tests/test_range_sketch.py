"""RangePartitioner bounds from the data (§8(f) row 3): RangePartitioner.sketch +
determineBounds (Spark 3.0.1, restated in oracle/spark_semantics.py).

Parity is UNPINNED against Spark itself (no JVM / Spark here, no fixture in the reference):
the GPU sketch (every record's XORShiftRandom draw in parallel by GF(2) jump-ahead) is
checked against the sequential restatement, which is checked here for internal properties
(reservoir = uniform sample semantics, bounds sorted / distinct / balanced)."""
import numpy as np
import pytest


def test_xorshift_jump_matches_sequential(oracle_lib):
    """The engine's jump-ahead relies on XORShiftRandom's step being GF(2)-linear: M^a M^b =
    M^(a+b) on the sequential generator (checked on the Python restatement)."""
    from oracle import spark_semantics as ss

    M64 = ss.M64

    def step(s):
        s ^= (s << 21) & M64
        s ^= s >> 35
        s ^= (s << 4) & M64
        return s

    cols = [step(1 << b) for b in range(64)]

    def apply(c, v):
        r = 0
        for b in range(64):
            if (v >> b) & 1:
                r ^= c[b]
        return r

    s0 = ss.xorshift_hash_seed(12345)
    s = s0
    for _ in range(37):
        s = step(s)
    m = cols
    j = s0
    # 37 = 32 + 4 + 1 via repeated squaring
    pows = [cols]
    for _ in range(6):
        p = pows[-1]
        pows.append([apply(p, apply(p, 1 << b)) for b in range(64)])
    for bit in range(6):
        if (37 >> bit) & 1:
            j = apply(pows[bit], j)
    assert j == s
    del m


def test_reservoir_semantics(oracle_lib):
    from oracle import spark_semantics as ss

    keys = list(range(1000))
    s, n = ss.reservoir_sample_and_count(keys, 50, 7)
    assert n == 1000 and len(s) == 50 and len(set(s)) == 50
    s2, n2 = ss.reservoir_sample_and_count(keys[:30], 50, 7)
    assert n2 == 30 and s2 == keys[:30]


def test_bounds_properties(oracle_lib):
    from oracle import spark_semantics as ss

    rng = np.random.default_rng(0)
    parts = [rng.integers(-(2**40), 2**40, size=3000).tolist() for _ in range(4)]
    b = ss.range_bounds(parts, 16, rdd_id=3)
    assert len(b) == 15 and b == sorted(b) and len(set(b)) == 15
    allk = np.sort(np.concatenate(parts))
    counts = np.diff(np.searchsorted(allk, b, side="right"))
    assert counts.min() > 0.4 * len(allk) / 16 and counts.max() < 1.8 * len(allk) / 16


@pytest.mark.gpu
@pytest.mark.parametrize("rb,R,sizes,rdd", [(16, 64, (20_000, 19_000, 21_000), 5), (16, 200, (50_000, 45_000), 0),
                                            (16, 8, (100, 0, 70), 2), (100, 32, (6_000, 7_000), 9)])
def test_gpu_sketch_matches_restatement(sgx_lib, oracle_lib, rb, R, sizes, rdd):
    from oracle import spark_semantics as ss

    batches = []
    for i, n in enumerate(sizes):
        if rb == 16:
            recs = oracle_lib.gen_uniform16(n, 77 + i)
            recs[: n // 3, :8] = recs[:1, :8]  # duplicates
        else:
            recs = oracle_lib.gen_terasort100(n, 77 + i)
        batches.append(recs)
    with sgx_lib.ShuffleEngine(device=0) as e:
        got = e.range_bounds(batches, list(sizes), rb, R, rdd)
        dev = [e.alloc(max(16, b.nbytes)) for b in batches]
        for d, b in zip(dev, batches):
            d.copy_from(b)
        got_dev = e.range_bounds(dev, list(sizes), rb, R, rdd)
    if rb == 16:
        keys = [b[:, :8].copy().view("<i8").reshape(-1).tolist() for b in batches]
        want = np.array(ss.range_bounds(keys, R, rdd), dtype=np.int64)
    else:
        keys = [[bytes(r[:10]) for r in b] for b in batches]
        want = np.frombuffer(b"".join(ss.range_bounds(keys, R, rdd)), dtype=np.uint8).reshape(-1, 10)
    assert np.array_equal(got, want)
    assert np.array_equal(got_dev, want)


@pytest.mark.gpu
def test_terasort_end_to_end_with_sampled_bounds(sgx_lib, oracle_lib, tmp_path):
    """TeraSort's shape end to end on one GPU: bounds from the data (sketch), map-side
    partition + scatter, then each reducer's records sorted by key: the concatenation of all
    reducers is the globally sorted input (a property that holds at any size)."""
    maps = [oracle_lib.gen_terasort100(n, 300 + i) for i, n in enumerate((40_000, 35_000, 38_000))]
    mgr = sgx_lib.UcxShuffleManager(device=0, localDir=str(tmp_path))
    try:
        part = sgx_lib.RangePartitioner.fromData(mgr.engine, maps, [len(m) for m in maps], 100, 64, rddId=1)
        h = mgr.registerShuffle(0, sgx_lib.ShuffleDependency(part, 100, keyOrdering=True))
        for mid, m in enumerate(maps):
            w = mgr.getWriter(h, mid)
            w.write(m)
        got = mgr.getReader(h, 0, part.numPartitions).read()
        allr = np.concatenate(maps)
        want = allr[np.lexsort(tuple(allr[:, i] for i in range(9, -1, -1)))]
        assert np.array_equal(got, want)
    finally:
        mgr.stop()


def test_murmur3_bytes_hash_pinned_to_scikit_learn():
    """scala.util.hashing.MurmurHash3.bytesHash (the XORShiftRandom seed hash of the sketch)
    is MurmurHash3_x86_32; the restatement agrees with scikit-learn's independent C
    implementation (sklearn.utils.murmurhash3_32) on every tail length, random seeds, Scala's
    arraySeed and the 8-byte big-endian seeds XORShiftRandom hashes.  This pins one building
    block of the sketch to an implementation outside this repository; the rest of the row
    stays unpinned (no JVM here)."""
    from oracle import spark_semantics as semantics

    murmurhash3_32 = pytest.importorskip("sklearn.utils").murmurhash3_32
    rng = np.random.default_rng(7)
    for n in list(range(0, 41)) + [64, 100, 1000]:
        for seed in (0, 1, 0x3C074A61, 0xFFFFFFFF, int(rng.integers(0, 2**32))):
            data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
            want = murmurhash3_32(data, seed=seed, positive=True)
            assert semantics.murmur3_bytes_hash(data, seed) == want, (n, seed)
    for s in (0, 1, -1, 42, 2**40 + 7, -(2**63)):
        b = (s & (2**64 - 1)).to_bytes(8, "big")
        lo = murmurhash3_32(b, seed=0x3C074A61, positive=True)
        hi = murmurhash3_32(b, seed=lo, positive=True)
        assert semantics.xorshift_hash_seed(s) == (hi << 32) | lo


def test_java_random_known_answers():
    """java.util.Random, whose nextLong() seeds each re-sampled partition
    (PartitionwiseSampledRDD.getPartitions): the widely published first values."""
    from oracle import spark_semantics as ss

    assert ss.JavaRandom(42).next_int() == -1170105035
    assert ss.JavaRandom(0).next_long() == -4962768465676381896


def test_bernoulli_sampler_properties():
    """BernoulliSampler restated: deterministic per seed, the kept fraction near f in both
    regimes (gap sampling at f <= 0.4, one draw per item above), order preserved."""
    from oracle import spark_semantics as ss

    items = list(range(200_000))
    for f in (0.01, 0.3, 0.5, 0.9):
        a = ss.bernoulli_sample(items, f, 1234)
        assert a == ss.bernoulli_sample(items, f, 1234) and a == sorted(a)
        assert abs(len(a) - f * len(items)) < 6 * (f * (1 - f) * len(items)) ** 0.5, f
    assert ss.bernoulli_sample(items, 0.0, 1) == [] and ss.bernoulli_sample(items[:10], 1.0, 1) == items[:10]


def test_imbalanced_partitions_are_resampled():
    """A partition holding more than 3 / #partitions of the items is re-sampled (RDD.sample),
    not refused: bounds come out sorted, distinct and still balanced over the data."""
    from oracle import spark_semantics as ss

    rng = np.random.default_rng(5)
    parts = [rng.integers(-(2**40), 2**40, size=n).tolist() for n in (40_000, 500, 500, 500, 500, 500, 500, 500)]
    b = ss.range_bounds(parts, 64, rdd_id=4)
    assert len(b) == 63 and b == sorted(b) and len(set(b)) == 63
    allk = np.sort(np.concatenate(parts))
    counts = np.diff(np.searchsorted(allk, b, side="right"))
    assert counts.min() > 0.3 * len(allk) / 64 and counts.max() < 2.0 * len(allk) / 64


@pytest.mark.gpu
@pytest.mark.parametrize("rb,R,sizes,rdd,parent", [
    (16, 64, (50_000,) + (1_000,) * 7, 6, 5),      # fraction 0.022: gap sampling
    (16, 200, (9_000, 100, 100, 100), 3, 1),       # fraction 0.43: one draw per record (GPU)
    (100, 32, (30_000, 400, 400, 400, 400), 8, 2),  # TeraSort keys, gap sampling
    (16, 16, (2_000, 0, 10), 1, 0),                 # fraction 0.16, an empty partition
])
def test_gpu_resampling_of_imbalanced_partitions(sgx_lib, oracle_lib, rb, R, sizes, rdd, parent):
    """Spark's second pass for imbalanced partitions (RangePartitioner's rangeBounds:
    fraction * n > sampleSizePerPartition -> RDD.sample(false, fraction,
    byteswap32(-rdd.id - 1))) on the GPU path equals the sequential restatement, for host and
    device batches, Long and 10-byte keys, both BernoulliSampler regimes."""
    from oracle import spark_semantics as ss

    batches = []
    for i, n in enumerate(sizes):
        recs = oracle_lib.gen_uniform16(n, 91 + i) if rb == 16 else oracle_lib.gen_terasort100(n, 91 + i)
        batches.append(recs)
    with sgx_lib.ShuffleEngine(device=0) as e:
        got = e.range_bounds(batches, list(sizes), rb, R, rdd, parent_rdd_id=parent)
        dev = [e.alloc(max(16, b.nbytes)) for b in batches]
        for d, b in zip(dev, batches):
            d.copy_from(b)
        got_dev = e.range_bounds(dev, list(sizes), rb, R, rdd, parent_rdd_id=parent)
    if rb == 16:
        keys = [b[:, :8].copy().view("<i8").reshape(-1).tolist() for b in batches]
        want = np.array(ss.range_bounds(keys, R, rdd, parent_rdd_id=parent), dtype=np.int64)
    else:
        keys = [[bytes(r[:10]) for r in b] for b in batches]
        want = np.frombuffer(b"".join(ss.range_bounds(keys, R, rdd, parent_rdd_id=parent)),
                             dtype=np.uint8).reshape(-1, 10)
    assert len(want) > 0
    assert np.array_equal(got, want)
    assert np.array_equal(got_dev, want)
