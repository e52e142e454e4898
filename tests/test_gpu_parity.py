"""GPU parity: the HIP path (through the C ABI) against the oracle and the golden fixtures.

Bit-exact bar (integer/byte work): identical partition lengths (=> identical index
offsets), identical partition-contiguous bytes (=> identical partition ids and per-reducer
record sequences in input order), identical index/data files."""
import glob
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

_sid = [1000]


def next_sid():
    _sid[0] += 1
    return _sid[0]


def run_map(engine, recs, R, kind=0, bounds=None, ascending=True, host=True):
    """Write one map through the C ABI; return (lengths, output bytes as (n, rb))."""
    import sparkucx_amd as sgx

    rb = recs.shape[1] if recs.ndim == 2 else 16
    sid = next_sid()
    engine.register_shuffle(sid, R, kind, bounds, ascending, rb)
    try:
        if host:
            src = np.ascontiguousarray(recs)
        else:
            src = engine.alloc(max(recs.nbytes, 16))
            src.copy_from(recs)
        n = recs.shape[0]
        lengths = engine.write_map(sid, 0, src, n, rb, R)
        out = engine.map_output_bytes(sid, 0).reshape(-1, rb)
        return lengths, out
    finally:
        engine.unregister_shuffle(sid)
        _ = sgx


def check_against_oracle(engine, oracle_lib, recs, R, kind=0, bounds=None, ascending=True, host=True):
    want_out, want_counts = oracle_lib.map_write(recs, R, kind, bounds, ascending, nthreads=8)
    lengths, out = run_map(engine, recs, R, kind, bounds, ascending, host)
    rb = recs.shape[1]
    assert np.array_equal(lengths, want_counts * rb), "partition lengths / index offsets differ"
    assert out.shape == want_out.shape
    if not np.array_equal(out, want_out):
        bad = np.nonzero(np.any(out != want_out, axis=1))[0]
        pytest.fail(f"{len(bad)} records differ, first at {bad[:5]}")


# ---------------------------------------------------------------- golden fixtures ----
@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "hash_*.npz"))))
def test_golden_hash(engine, path):
    z = np.load(path)
    R = int(z["num_partitions"])
    lengths, out = run_map(engine, z["records"], R)
    assert np.array_equal(lengths, z["lengths"])
    assert np.array_equal(out, z["out"])


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "range_*.npz"))))
def test_golden_range(engine, path):
    import sparkucx_amd as sgx

    z = np.load(path)
    R = int(z["num_partitions"])
    kind = sgx.PART_RANGE_BYTES10 if z["records"].shape[1] == 100 else sgx.PART_RANGE_I64
    lengths, out = run_map(engine, z["records"], R, kind, z["bounds"], bool(z["ascending"]))
    assert np.array_equal(lengths, z["lengths"])
    assert np.array_equal(out, z["out"])


# ---------------------------------------------------------------- seeded random ------
@pytest.mark.parametrize("R", [1, 2, 3, 7, 200, 1000, 1024, 2048, 4096, 5000])
@pytest.mark.parametrize("n", [0, 1, 63, 64, 65, 8191, 8192, 8193, 100_003])
def test_hash_random_sizes(engine, oracle_lib, R, n):
    recs = oracle_lib.gen_uniform16(n, 0x5EEDC0DE + R + n)
    check_against_oracle(engine, oracle_lib, recs, R)


@pytest.mark.parametrize("R", [200, 1024, 4096])
def test_hash_device_input_2m(engine, oracle_lib, R):
    recs = oracle_lib.gen_uniform16(2_000_003, R)
    check_against_oracle(engine, oracle_lib, recs, R, host=False)


def test_device_generator_matches_oracle(engine, oracle_lib):
    n = 1_000_001
    buf = engine.alloc(n * 16)
    engine.gen_uniform16(buf, n, 0xABCDEF, value_base=12345)
    assert np.array_equal(buf.to_numpy().reshape(-1, 16), oracle_lib.gen_uniform16(n, 0xABCDEF, 12345))
    cdf = oracle_lib.zipf_cdf(1.1, 2**16)
    engine.gen_zipf16(buf, n, 77, cdf, value_base=3)
    assert np.array_equal(buf.to_numpy().reshape(-1, 16), oracle_lib.gen_zipf16(n, 77, cdf, 3))
    m = 10_001
    tb = engine.alloc(m * 100)
    engine.gen_terasort100(tb, m, 99, 5)
    assert np.array_equal(tb.to_numpy().reshape(-1, 100), oracle_lib.gen_terasort100(m, 99, 5))


def test_edge_keys_all_partition_counts(engine, oracle_lib):
    import json

    kats = json.load(open(os.path.join(GOLDEN, "kats.json")))
    keys = sorted({k for k, _, _ in kats["edge_pids"]})
    recs = np.zeros((len(keys) * 5, 16), np.uint8)
    arr = np.array(keys * 5, dtype=np.int64)
    recs[:, :8] = arr.view(np.uint8).reshape(-1, 8)
    recs[:, 8:] = np.arange(len(arr), dtype=np.int64).view(np.uint8).reshape(-1, 8)
    for R in (1, 2, 3, 7, 200, 1000, 1024, 4096, 5000):
        check_against_oracle(engine, oracle_lib, recs, R)


@pytest.mark.parametrize("R", [1024, 4096])
@pytest.mark.parametrize("num_chunks", [1, 3, 1024, 4096])
def test_chunking_does_not_change_output(sgx_lib, oracle_lib, num_chunks, R):
    recs = oracle_lib.gen_uniform16(300_007, 5)
    with sgx_lib.ShuffleEngine(device=0, num_chunks=num_chunks) as e:
        check_against_oracle(e, oracle_lib, recs, R)


GEOMETRIES = [(4, 16), (8, 16), (12, 10), (14, 9), (16, 7), (4, 12), (8, 8), (4, 8), (8, 4), (4, 4), (4, 2), (4, 1)]


@pytest.mark.parametrize("rank", ["ordered", "match"])
@pytest.mark.parametrize("waves,items", GEOMETRIES)
@pytest.mark.parametrize("R", [7, 200, 1024, 1536, 4096])
def test_every_staged_geometry(sgx_lib, oracle_lib, waves, items, R, rank):
    """Every instantiated K4 geometry of both rankers (lane-ordered atomics, ballot/peer
    table), full tiles + a ragged tail, multiple chunks.  A (waves, items) pair the
    lane-ordered kernel lacks falls back to the match kernel, which is then re-tested."""
    rank_mode = sgx_lib.RANK_MATCH if rank == "match" else sgx_lib.RANK_ORDERED
    tile = waves * items * 64
    n = 5 * tile * 3 + tile // 3 + 7
    recs = oracle_lib.gen_uniform16(n, 0xC0FFEE + R)
    with sgx_lib.ShuffleEngine(device=0, num_chunks=3, scatter_waves=waves, scatter_items=items,
                               rank_mode=rank_mode) as e:
        try:
            check_against_oracle(e, oracle_lib, recs, R)
        except sgx_lib.UnsupportedOperationException:  # geometry's LDS does not fit this R
            pytest.skip(f"geometry {waves}x{items} does not fit R={R}")


@pytest.mark.parametrize("cfg", [dict(hist_mode=1), dict(rank_mode=1), dict(flags=1), dict(hist_mode=1, flags=1),
                                 dict(flags=32), dict(flags=128)])
def test_kernel_choices_are_byte_identical(sgx_lib, oracle_lib, cfg):
    """sgx_config's kernel choices -- the ballot/popcount wave-aggregated histogram
    (SGX_HIST_BALLOT), ballot-matched K4 ranking (SGX_RANK_MATCH), K4 without write-combining
    (SGX_FLAG_NO_WRITE_COMBINING), one lane-ordered pass instead of the two-level split at
    R > 1024 (SGX_FLAG_NO_SPLIT_SCATTER), the fallback taken when the engine-start LDS ordering
    check fails (SGX_FLAG_ASSUME_LDS_DISORDER) -- change speed, never bytes."""
    recs = oracle_lib.gen_uniform16(3 * 8192 * 5 + 1234, 99)
    with sgx_lib.ShuffleEngine(device=0, **cfg) as e:
        for R in (7, 200, 1024, 4096):
            check_against_oracle(e, oracle_lib, recs, R)
    cdf = oracle_lib.zipf_cdf(1.1, 2**20)
    zrecs = oracle_lib.gen_zipf16(300_001, 5, cdf)
    with sgx_lib.ShuffleEngine(device=0, **cfg) as e:
        for R in (1024, 4096):
            check_against_oracle(e, oracle_lib, zrecs, R)


def test_engine_start_lds_order_check(sgx_lib, oracle_lib):
    """sgx_create probes, on the device it runs on, the property the default ranking rests on
    (same-address LDS atomics of one wave return old values in issue order, then lane order);
    it holds on MI355X.  When it does not (forced here by SGX_FLAG_ASSUME_LDS_DISORDER) the
    engine ranks every scatter by ballot matching -- 100 B records included -- same bytes."""
    with sgx_lib.ShuffleEngine(device=0) as e:
        assert e.lds_order_ok
    tera = oracle_lib.gen_terasort100(50_001, 17)
    with sgx_lib.ShuffleEngine(device=0, flags=sgx_lib.FLAG_ASSUME_LDS_DISORDER, num_chunks=5) as e:
        assert not e.lds_order_ok
        for R in (1, 64, 2048):
            check_against_oracle(e, oracle_lib, tera, R)


@pytest.mark.parametrize("R", [200, 585, 586, 1000, 1024, 1025, 2048, 3000, 4096, 5000, 8192])
@pytest.mark.parametrize("group", [7, 15, 1])
def test_write_combining_carry_pressure(sgx_lib, oracle_lib, R, group):
    """Write-combining K4: records arrive in runs of `group` per partition, so most
    partitions end every tile with a 7-record tail; the deferred records then exceed the
    tile's carry capacity and force the flush path, alternating with normal tiles.  Several
    chunks, a ragged last tile; bit-exact against the oracle.  (R > 1024 runs the
    lane-ordered kernel: the same input shapes on that path.)"""
    n = 3 * 4096 * 7 + 1234
    recs = oracle_lib.gen_uniform16(n, 0xCA11 + R + group)
    rng = np.random.default_rng(R * 31 + group)
    pids = np.concatenate([np.repeat(rng.permutation(R), group) for _ in range(n // (R * group) + 1)])[:n]
    keys = (pids + R * rng.integers(0, 1000, n)).astype(np.int64)  # 0 <= key < 2^31: pid = key % R
    recs[:, :8] = keys.view(np.uint8).reshape(-1, 8)
    for chunks in (1, 3):
        with sgx_lib.ShuffleEngine(device=0, num_chunks=chunks) as e:
            check_against_oracle(e, oracle_lib, recs, R)


@pytest.mark.parametrize("R", [2048, 4096, 8192])
@pytest.mark.parametrize("shape", ["uniform", "one_super", "hot_partition", "many_hot", "all_hot", "zipf", "tiny", "empty"])
def test_two_level_split_scatter(sgx_lib, oracle_lib, R, shape):
    """The two-level split K4 (hash, power-of-two R > 1024: S = R/64 super-partitions written
    whole-line, then 64 sub-partitions inside each, over pieces of whole (super, chunk)
    blocks; the hybrid level 1 writes partitions with >= 2x the mean count straight to the
    output): bit-exact against the oracle, and byte-identical to the single lane-ordered pass
    (SGX_FLAG_NO_SPLIT_SCATTER), for uniform keys, every key in ONE super-partition (one piece
    per chunk, all other supers empty), one hot partition holding most records, more hot
    partitions than the hybrid's 192 hot streams, every record hot (level 2 empty), Zipf(1.1),
    a map smaller than one tile, and an empty map; 1, 5 and the default number of chunks."""
    n = {"tiny": 1000, "empty": 0}.get(shape, 400_003)
    recs = oracle_lib.gen_uniform16(max(n, 1), 0x5B1 + R)[:n]
    rng = np.random.default_rng(R)
    if shape == "one_super":  # pid in [64 s, 64 s + 64) for one s
        pid = 64 * 3 + rng.integers(0, 64, n)
        recs[:, :8] = (pid + R * rng.integers(0, 1 << 20, n)).astype(np.int64).view(np.uint8).reshape(-1, 8)
    elif shape == "hot_partition":
        pid = np.where(rng.random(n) < 0.8, 5, rng.integers(0, R, n))
        recs[:, :8] = (pid + R * rng.integers(0, 1 << 20, n)).astype(np.int64).view(np.uint8).reshape(-1, 8)
    elif shape == "many_hot":  # the hybrid's hot streams: more qualifying partitions than SPLIT_HOT_CAP (192)
        pid = np.where(rng.random(n) < 0.7, rng.integers(0, 300, n) * (R // 300), rng.integers(0, R, n))
        recs[:, :8] = (pid + R * rng.integers(0, 1 << 20, n)).astype(np.int64).view(np.uint8).reshape(-1, 8)
    elif shape == "all_hot":  # every record in a hot partition: level 2 gets no records
        pid = rng.integers(0, 8, n) * 37 % R
        recs[:, :8] = (pid + R * rng.integers(0, 1 << 20, n)).astype(np.int64).view(np.uint8).reshape(-1, 8)
    elif shape == "zipf":
        recs = oracle_lib.gen_zipf16(n, 0x5B1 + R, oracle_lib.zipf_cdf(1.1, 2**24))
    for chunks in (0, 1, 5):
        for flags in (0, sgx_lib.FLAG_NO_SPLIT_SCATTER):  # both bit-exact: byte-identical to each other
            with sgx_lib.ShuffleEngine(device=0, num_chunks=chunks, flags=flags) as e:
                check_against_oracle(e, oracle_lib, recs, R)


def test_zipf_skew_r4096(engine, oracle_lib):
    cdf = oracle_lib.zipf_cdf(1.1, 2**24)
    recs = oracle_lib.gen_zipf16(1_000_000, 11, cdf)
    check_against_oracle(engine, oracle_lib, recs, 4096)


@pytest.mark.parametrize("distinct", [2, 5, 64, 300])
@pytest.mark.parametrize("R", [7, 1024, 4096])
def test_heavy_collisions(engine, oracle_lib, distinct, R):
    """Few distinct keys: many lanes of one ranking atomic hit the same counter dword, the
    case where stability rests on lane-ordered LDS atomics."""
    recs = oracle_lib.gen_uniform16(300_001, distinct * 7 + R)
    keys = np.arange(distinct, dtype=np.int64) * 7919 - 3
    pick = np.random.default_rng(distinct).integers(0, distinct, len(recs))
    recs[:, :8] = keys[pick].view(np.uint8).reshape(-1, 8)
    check_against_oracle(engine, oracle_lib, recs, R)


@pytest.mark.parametrize("R", [1024, 4096, 6144])
def test_all_records_one_partition(engine, oracle_lib, R):
    recs = oracle_lib.gen_uniform16(200_000, 1)
    recs[:, :8] = np.frombuffer(np.int64(4242).tobytes(), np.uint8)  # same key everywhere
    check_against_oracle(engine, oracle_lib, recs, R)


@pytest.mark.parametrize("R", [1025, 1536, 1537, 2048, 3072, 4096, 5000, 6144, 6145])
@pytest.mark.parametrize("shape", ["uniform", "sorted", "edges", "hot"])
def test_large_r_shapes(sgx_lib, oracle_lib, R, shape):
    """R > 1024: the K4 shapes that stress a large-R scatter -- uniform keys; keys sorted by
    partition (every chunk sees a different narrow band of partitions); only the first and
    last partitions; one hot partition holding half the records -- over several chunk
    counts and a ragged size, bit-exact against the oracle.  (These shapes were written
    for the split write-combining K4 that was measured and rejected; they
    run the lane-ordered kernel.)"""
    n = 700_001
    recs = oracle_lib.gen_uniform16(n, 0x5917 + R)
    rng = np.random.default_rng(R)
    if shape == "sorted":
        pids = (np.arange(n, dtype=np.int64) * R) // n
    elif shape == "edges":
        pids = np.where(rng.integers(0, 2, n) == 0, 0, R - 1)
    elif shape == "hot":
        pids = np.where(rng.integers(0, 2, n) == 0, R // 3, rng.integers(0, R, n))
    else:
        pids = None
    if pids is not None:  # 0 <= key < 2^31: HashPartitioner gives key % R
        keys = (pids + R * rng.integers(0, 1000, n)).astype(np.int64)
        recs[:, :8] = keys.view(np.uint8).reshape(-1, 8)
    for chunks in (0, 5, 64):
        with sgx_lib.ShuffleEngine(device=0, num_chunks=chunks) as e:
            check_against_oracle(e, oracle_lib, recs, R)


# ---------------------------------------------------------------- range partitioners --
@pytest.mark.parametrize("nb", [1, 50, 128, 129, 1023, 4095])
@pytest.mark.parametrize("asc", [True, False])
def test_range_i64_random(engine, oracle_lib, nb, asc):
    import sparkucx_amd as sgx

    rng = np.random.default_rng(nb)
    recs = oracle_lib.gen_uniform16(50_000, nb + 3)
    keys = recs[:, :8].copy().view(np.int64).ravel()
    bounds = np.sort(rng.choice(keys, nb, replace=False))
    recs[:nb, :8] = bounds.view(np.uint8).reshape(-1, 8)  # exact hits on bounds
    check_against_oracle(engine, oracle_lib, recs, nb + 1, sgx.PART_RANGE_I64, bounds, asc)


@pytest.mark.parametrize("nb", [63, 1023])
def test_terasort_bytes10(engine, oracle_lib, nb):
    import sparkucx_amd as sgx

    recs = oracle_lib.gen_terasort100(60_000, nb)
    rng = np.random.default_rng(nb)
    sample = recs[rng.choice(len(recs), 20 * (nb + 1), replace=False), :10]
    order = np.lexsort(sample.T[::-1])
    sample = sample[order]
    step = len(sample) / (nb + 1)
    bounds = np.ascontiguousarray(sample[[int(step * (i + 1)) for i in range(nb)]])
    check_against_oracle(engine, oracle_lib, recs, nb + 1, sgx.PART_RANGE_BYTES10, bounds)


@pytest.mark.parametrize("shape", ["one_bucket", "two_buckets", "dups_linear", "dups_jdk", "extremes"])
@pytest.mark.parametrize("rb", [16, 100])
def test_range_directory_edges(engine, oracle_lib, shape, rb):
    """The bounds' top-bits directory (sgx_register_shuffle, range_pid_*): every bound sharing
    the key's top 10 bits (one directory bucket holding the whole search), bounds split over
    two buckets, duplicate bounds on Spark's linear branch (<= 128: a lower bound, directory
    used) and on its binary search (> 128: the exact JDK loop, no directory), and keys at the
    extremes of the key space -- every key also hitting a bound exactly -- against the oracle,
    both orders, 16 B Long keys and 100 B TeraSort keys, on every scatter kernel."""
    import sparkucx_amd as sgx

    rng = np.random.default_rng(len(shape) * 100 + rb)
    n = 40_000
    recs = oracle_lib.gen_uniform16(n, 77) if rb == 16 else oracle_lib.gen_terasort100(n, 77)
    if rb == 16:
        kind = sgx.PART_RANGE_I64
        top = np.int64(0x1230000000000000)
        if shape == "one_bucket":
            b = np.unique(top + rng.integers(0, 1 << 40, 700))
        elif shape == "two_buckets":
            b = np.unique(np.concatenate([top + rng.integers(0, 1 << 40, 300), -top + rng.integers(0, 1 << 40, 300)]))
        elif shape == "dups_linear":
            b = np.sort(np.repeat(rng.integers(-(1 << 62), 1 << 62, 40), 3))[:120]
        elif shape == "dups_jdk":
            b = np.sort(np.repeat(rng.integers(-(1 << 62), 1 << 62, 100), 3))
        else:
            b = np.array([-(1 << 63), -(1 << 63) + 1, -1, 0, 1, (1 << 63) - 2, (1 << 63) - 1], dtype=np.int64)
        b = np.sort(b.astype(np.int64))
        keys = recs[:, :8].copy().view(np.int64).ravel()
        keys[:len(b)] = b  # exact hits
        if shape == "one_bucket" or shape == "two_buckets":
            keys[len(b):len(b) + 20000] = top + rng.integers(-(1 << 41), 1 << 41, 20000)
        keys[-4:] = [-(1 << 63), (1 << 63) - 1, 0, -1]
        recs[:, :8] = keys.view(np.uint8).reshape(-1, 8)  # (the strided view's ravel is a copy)
        bounds = b
    else:
        kind = sgx.PART_RANGE_BYTES10
        keys = recs[:, :10]
        if shape == "one_bucket":
            b = rng.integers(0, 256, (700, 10), dtype=np.uint8)
            b[:, 0], b[:, 1] = 0x12, 0x30
        elif shape == "two_buckets":
            b = rng.integers(0, 256, (600, 10), dtype=np.uint8)
            b[:300, 0], b[:300, 1], b[300:, 0], b[300:, 1] = 0x12, 0x30, 0xF0, 0x00
        elif shape == "dups_linear":
            b = np.repeat(rng.integers(0, 256, (40, 10), dtype=np.uint8), 3, axis=0)[:120]
        elif shape == "dups_jdk":
            b = np.repeat(rng.integers(0, 256, (100, 10), dtype=np.uint8), 3, axis=0)
        else:
            b = np.array([[0] * 10, [0] * 9 + [1], [0x7F] + [0xFF] * 9, [0xFF] * 9 + [0xFE], [0xFF] * 10], np.uint8)
        b = b[np.lexsort(b.T[::-1])]
        if shape in ("one_bucket", "two_buckets"):
            b = np.unique(b, axis=0)
        bounds = np.ascontiguousarray(b)
        keys[:len(b)] = bounds
        if shape in ("one_bucket", "two_buckets"):
            keys[len(b):len(b) + 20000, 0], keys[len(b):len(b) + 20000, 1] = 0x12, 0x30
        keys[-2:] = [[0] * 10, [0xFF] * 10]
    for asc in (True, False):
        check_against_oracle(engine, oracle_lib, recs, len(bounds) + 1, kind, bounds, asc)


@pytest.mark.parametrize("wide2", ["1", "0"])
@pytest.mark.parametrize("R", [1, 7, 1000, 2048, 4096])
@pytest.mark.parametrize("n", [1, 1023, 1024, 5 * 1024 + 77, 3 * 4096 + 1001])
def test_wide_records_every_path(sgx_lib, oracle_lib, wide2, R, n):
    """100 B records: the LDS-staged K4 (R <= 2048) and the per-lane kernel
    (SGX_FLAG_NO_WIDE_STAGED, and R = 4096), hash and range partitioners, partial tiles and
    several chunks."""
    flags = 0 if wide2 == "1" else sgx_lib.FLAG_NO_WIDE_STAGED
    recs = oracle_lib.gen_terasort100(n, R + n)
    with sgx_lib.ShuffleEngine(device=0, num_chunks=3, flags=flags) as e:
        check_against_oracle(e, oracle_lib, recs, R)
        if R > 1:
            rng = np.random.default_rng(R)
            sample = recs[rng.choice(n, min(n, 8 * R), replace=n < 8 * R), :10]
            sample = sample[np.lexsort(sample.T[::-1])]
            bounds = np.ascontiguousarray(sample[np.linspace(0, len(sample) - 1, R - 1).astype(int)])
            check_against_oracle(e, oracle_lib, recs, R, sgx_lib.PART_RANGE_BYTES10, bounds)


def test_hash_on_wide_records(engine, oracle_lib):
    recs = oracle_lib.gen_terasort100(30_000, 4)
    check_against_oracle(engine, oracle_lib, recs, 1024)


# ---------------------------------------------------------------- plugin API ----------
def test_manager_writer_resolver_reader(sgx_lib, oracle_lib, tmp_path):
    R, n = 1024, 250_000
    mgr = sgx_lib.UcxShuffleManager(localDir=str(tmp_path))
    try:
        h = mgr.registerShuffle(5, sgx_lib.ShuffleDependency(sgx_lib.HashPartitioner(R)))
        maps = {}
        for m in (3, 1, 2):
            recs = oracle_lib.gen_uniform16(n + m, 100 + m, value_base=m << 40)
            w = mgr.getWriter(h, m)
            w.write(recs)
            out, counts = oracle_lib.map_write(recs, R)
            maps[m] = (out, counts)
            assert np.array_equal(w.getPartitionLengths(), counts * 16)
            st = w.stop(True)
            assert st.mapId == m
        # index + data files (IndexShuffleBlockResolver layout)
        res = mgr.shuffleBlockResolver
        lengths = maps[1][1] * 16
        res.writeIndexFileAndCommit(5, 1, lengths)
        assert open(res.getIndexFile(5, 1), "rb").read() == oracle_lib.index_bytes(lengths)
        assert open(res.getDataFile(5, 1), "rb").read() == maps[1][0].tobytes()
        assert np.array_equal(res.checkIndexAndDataFile(res.getIndexFile(5, 1), res.getDataFile(5, 1), R),
                              lengths)
        off = oracle_lib.offsets(maps[1][1])
        assert res.getBlockData("shuffle_5_1_17") == maps[1][0][off[17]:off[18]].tobytes()
        assert res.getBlockData((5, 1, 10, 20)) == maps[1][0][off[10]:off[20]].tobytes()
        # reader: canonical order (reducer, then map ascending)
        got = mgr.getReader(h, 100, 103).read()
        want = []
        for r in range(100, 103):
            for m in sorted(maps):
                o = oracle_lib.offsets(maps[m][1])
                want.append(maps[m][0][o[r]:o[r + 1]])
        assert np.array_equal(got, np.concatenate(want))
    finally:
        mgr.stop()


def test_existing_attempt_wins(sgx_lib, oracle_lib, tmp_path):
    R = 200
    mgr = sgx_lib.UcxShuffleManager(localDir=str(tmp_path))
    try:
        h = mgr.registerShuffle(1, sgx_lib.ShuffleDependency(sgx_lib.HashPartitioner(R)))
        a = oracle_lib.gen_uniform16(10_000, 1)
        w = mgr.getWriter(h, 0)
        w.write(a)
        la = w.getPartitionLengths().copy()
        mgr.shuffleBlockResolver.writeIndexFileAndCommit(1, 0, la.copy())
        # a second attempt with different data: the committed first attempt wins
        b = oracle_lib.gen_uniform16(12_000, 2)
        w2 = mgr.getWriter(h, 0)
        w2.write(b)
        lb = w2.getPartitionLengths().copy()
        mgr.shuffleBlockResolver.writeIndexFileAndCommit(1, 0, lb)
        assert np.array_equal(lb, la)
        assert open(mgr.shuffleBlockResolver.getDataFile(1, 0), "rb").read() == oracle_lib.map_write(a, R)[0].tobytes()
        # a corrupt index is replaced by the new attempt
        with open(mgr.shuffleBlockResolver.getIndexFile(1, 0), "r+b") as f:
            f.write(b"\x01")
        lc = w2.getPartitionLengths().copy()
        mgr.shuffleBlockResolver.writeIndexFileAndCommit(1, 0, lc)
        assert open(mgr.shuffleBlockResolver.getDataFile(1, 0), "rb").read() == oracle_lib.map_write(b, R)[0].tobytes()
    finally:
        mgr.stop()


def test_fetch_blocks_and_errors(sgx_lib, oracle_lib, engine):
    R = 1024
    recs = oracle_lib.gen_uniform16(123_457, 3)
    out, counts = oracle_lib.map_write(recs, R)
    o = oracle_lib.offsets(counts) * 16
    flat = out.reshape(-1)
    sid = next_sid()
    engine.register_shuffle(sid, R)
    engine.write_map(sid, 9, recs, len(recs), 16, R)
    rng = np.random.default_rng(0)
    rids = rng.integers(0, R, 300)
    data, lens = engine.fetch_blocks(sid, [9] * len(rids), rids)
    want = np.concatenate([flat[o[r]:o[r + 1]] for r in rids])
    assert np.array_equal(data, want)
    assert np.array_equal(lens, (counts * 16)[rids])
    dev = engine.alloc(int(lens.sum()))
    engine.fetch_blocks(sid, [9] * len(rids), rids, dst=dev)
    assert np.array_equal(dev.to_numpy(), want)
    with pytest.raises(sgx_lib.BlockNotFoundException):
        engine.fetch_blocks(sid, [8], [0])
    with pytest.raises(sgx_lib.IllegalArgumentException):
        engine.fetch_blocks(sid, [9], [R])
    with pytest.raises(sgx_lib.IllegalArgumentException):
        engine.fetch_blocks(sid, [9, 9], [1, 2], dst=np.empty(1, np.uint8))
    engine.unregister_shuffle(sid)
    with pytest.raises(sgx_lib.IllegalStateException):
        engine.fetch_blocks(sid, [9], [0])
    with pytest.raises(sgx_lib.IllegalStateException):
        engine.write_map(sid, 0, recs, 10, 16)


def test_registration_errors(sgx_lib, engine):
    with pytest.raises(sgx_lib.IllegalArgumentException):
        engine.register_shuffle(next_sid(), 0)
    with pytest.raises(sgx_lib.UnsupportedOperationException):
        engine.register_shuffle(next_sid(), 1_000_000)
    with pytest.raises(sgx_lib.IllegalArgumentException):
        engine.register_shuffle(next_sid(), 10, sgx_lib.PART_RANGE_I64, np.arange(3), True)
    sid = next_sid()
    engine.register_shuffle(sid, 10)
    with pytest.raises(sgx_lib.IllegalStateException):
        engine.register_shuffle(sid, 10)
    with pytest.raises(sgx_lib.IllegalArgumentException):
        engine.write_map(sid, 0, np.zeros((4, 100), np.uint8), 4, 100)
    engine.unregister_shuffle(sid)


def test_transport_fetch_blocks_by_block_ids(sgx_lib, oracle_lib):
    import ctypes

    R = 64
    mgr = sgx_lib.UcxShuffleManager()
    try:
        h = mgr.registerShuffle(2, sgx_lib.ShuffleDependency(sgx_lib.HashPartitioner(R)))
        recs = oracle_lib.gen_uniform16(5000, 8)
        mgr.getWriter(h, 4).write(recs)
        out, counts = oracle_lib.map_write(recs, R)
        o = oracle_lib.offsets(counts) * 16
        pool = []

        def alloc(size):
            buf = ctypes.create_string_buffer(max(int(size), 1))
            pool.append(buf)
            return sgx_lib.MemoryBlock(ctypes.addressof(buf), int(size))

        got = {}
        ids = [sgx_lib.UcxShuffleBlockId(2, 4, r) for r in (0, 5, 63)] + [sgx_lib.UcxShuffleBlockId(2, 99, 0)]

        def cb_for(i):
            def cb(res):
                got[i] = res
            return cb

        t = mgr.getTransport()
        reqs = t.fetchBlocksByBlockIds(1, ids, alloc, [cb_for(i) for i in range(len(ids))])
        assert not any(r.isCompleted() for r in reqs)
        t.progress()
        assert all(r.isCompleted() for r in reqs)
        for i, r in enumerate((0, 5, 63)):
            res = got[i]
            assert res.getStatus() == sgx_lib.OperationStatus.SUCCESS
            mb = res.getData()
            assert ctypes.string_at(mb.address, mb.size) == out.reshape(-1)[o[r]:o[r + 1]].tobytes()
            mb.close()
        assert got[3].getStatus() == sgx_lib.OperationStatus.FAILURE
    finally:
        mgr.stop()


# ---------------------------------------------------------------- exchange -----------
def test_exchange_single_rank_over_rccl(sgx_lib, oracle_lib):
    R = 1024
    with sgx_lib.ShuffleEngine(device=0) as e:
        e.comm_init(1, 0, sgx_lib.get_unique_id())
        e.register_shuffle(1, R)
        recs = oracle_lib.gen_uniform16(400_000, 21)
        e.write_map(1, 6, recs, len(recs), 16, R)
        e.exchange(1)
        e.sync()
        data, lens = e.fetch_blocks(1, [6] * R, list(range(R)))
        out, counts = oracle_lib.map_write(recs, R)
        assert np.array_equal(data.reshape(-1, 16), out)
        st = e.stats()
        assert st.count["alltoall"] >= 1 and st.count["regroup"] >= 1


@pytest.mark.parametrize("nmaps,n", [(64, 3_000), (96, 20_001), (3, 600_000)])
def test_exchange_many_maps_one_rank_over_rccl(sgx_lib, oracle_lib, nmaps, n):
    """Spark's map counts: one executor holding many map outputs of a shuffle.  Small pieces
    (64 / 96 maps) go out packed -- one RCCL send per destination, gathered on the device --
    large ones (3 maps of 600 K records) one send per (map, destination); both land in the
    same receive layout and every block equals the oracle's, in the canonical order."""
    R = 512
    with sgx_lib.ShuffleEngine(device=0) as e:
        e.comm_init(1, 0, sgx_lib.get_unique_id())
        e.register_shuffle(1, R)
        outs = []
        for m in range(nmaps):
            recs = oracle_lib.gen_uniform16(n + 37 * m, 500 + m, value_base=m << 32)
            e.write_map(1, m, recs, len(recs), 16)
            outs.append(oracle_lib.map_write(recs, R))
        e.exchange(1)
        e.sync()
        seqs = oracle_lib.canonical_reducer_sequences(outs, R, 16)
        for r0, r1 in ((0, 3), (250, 251), (R - 2, R)):
            mids = [m for r in range(r0, r1) for m in range(nmaps)]
            rids = [r for r in range(r0, r1) for _ in range(nmaps)]
            data, _ = e.fetch_blocks(1, mids, rids)
            assert np.array_equal(data.reshape(-1, 16), np.concatenate(seqs[r0:r1]))
        got = e.read_records(1, list(range(nmaps)), 0, R).reshape(-1, 16)
        assert np.array_equal(got, np.concatenate(seqs))
        assert e.stats().count["alltoall"] == 1


@pytest.mark.parametrize("P", [2, 4, 8])
def test_regroup_kernel_multi_rank_plan(sgx_lib, oracle_lib, engine, P):
    """Simulate the receive side of a P-rank exchange on one GPU: build each source rank's
    map output with the oracle, lay the receive buffer out exactly as ncclAllToAllv would,
    run the K5 regroup kernel with the engine's plan and compare with the canonical
    per-reducer sequences."""
    R = 1024
    outs = []
    for s in range(P):
        recs = oracle_lib.gen_uniform16(50_000 + 17 * s, 1000 + s, value_base=s << 40)
        outs.append(oracle_lib.map_write(recs, R))
    L = np.stack([c * 16 for _, c in outs])
    for rank in range(P):
        sc, sd, rc, rd, items = sgx_lib.plan_exchange(L, rank, 64 * 1024)
        # what each source sends to `rank`: its contiguous slice of my reducers
        recv = []
        for s in range(P):
            s_sc, s_sd, _, _, _ = sgx_lib.plan_exchange(L, s, 0)
            flat = outs[s][0].reshape(-1)
            recv.append(flat[s_sd[rank]:s_sd[rank] + s_sc[rank]])
        recv = np.concatenate(recv) if recv else np.zeros(0, np.uint8)
        assert recv.nbytes == rc.sum()
        src = engine.alloc(max(recv.nbytes, 16))
        src.copy_from(recv)
        dst = engine.alloc(max(recv.nbytes, 16))
        engine.copy_items(src, dst, items, 16)
        got = dst.to_numpy(recv.nbytes)
        seqs = oracle_lib.canonical_reducer_sequences(outs, R, 16)
        mine = [r for r in range(R) if (r * P) // R == rank]
        want = np.concatenate([seqs[r] for r in mine]).reshape(-1)
        assert np.array_equal(got, want)


# ---------------------------------------------------------------- determinism / size --
def test_repeatable_bitwise(engine, oracle_lib):
    recs = oracle_lib.gen_uniform16(1_000_000, 31)
    a = run_map(engine, recs, 1024, host=False)
    b = run_map(engine, recs, 1024, host=False)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


@pytest.mark.slow
def test_full_c1_size_bit_exact(engine, oracle_lib):
    """BASELINE config C1 at full size: 2^28 uniform 16 B records, R = 1024, on-device
    input; compared byte for byte with the multi-threaded oracle."""
    n, R, seed = 1 << 28, 1024, 0x5EEDC0DE
    buf = engine.alloc(n * 16)
    engine.gen_uniform16(buf, n, seed)
    sid = next_sid()
    engine.register_shuffle(sid, R)
    lengths = engine.write_map(sid, 0, buf, n, 16, R)
    got = engine.map_output_bytes(sid, 0)
    engine.unregister_shuffle(sid)
    buf.free()
    recs = oracle_lib.gen_uniform16(n, seed)
    want, counts = oracle_lib.map_write(recs, R, nthreads=16)
    del recs
    assert np.array_equal(lengths, counts * 16)
    assert np.array_equal(got, want.reshape(-1))


@pytest.mark.slow
def test_full_c3_shard_zipf_r4096_bit_exact(engine, oracle_lib):
    """Config C3's per-GPU share at full size: 2^31 / 8 = 2^28 Zipf(1.1) records over
    K = 2^24 ranks, R = 4096 (hot reducer ~11.5 % of the records), on-device input."""
    import sparkucx_amd as sgx  # noqa: F401

    n, R, seed = 1 << 28, 4096, 0x5EEDC0DE + 3
    cdf = oracle_lib.zipf_cdf(1.1, 1 << 24)
    buf = engine.alloc(n * 16)
    engine.gen_zipf16(buf, n, seed, cdf)
    sid = next_sid()
    engine.register_shuffle(sid, R)
    lengths = engine.write_map(sid, 0, buf, n, 16, R)
    got = engine.map_output_bytes(sid, 0)
    engine.unregister_shuffle(sid)
    buf.free()
    recs = oracle_lib.gen_zipf16(n, seed, cdf)
    want, counts = oracle_lib.map_write(recs, R, nthreads=16)
    del recs
    assert counts[1] > 0.1 * n  # the hot reducer (rank 1 -> pid 1)
    assert np.array_equal(lengths, counts * 16)
    assert np.array_equal(got, want.reshape(-1))


@pytest.mark.slow
def test_full_c4_shard_terasort_bit_exact(engine, oracle_lib):
    """Config C4's record shape at one GPU's full share of bytes (2^28 x 16 B = 4.3 GB of
    100 B TeraSort records), 1023 sampled bounds, RangePartitioner over 10-byte keys."""
    import sparkucx_amd as sgx

    n, R, seed = (1 << 28) * 16 // 100, 1024, 0x7E7A
    buf = engine.alloc(n * 100)
    engine.gen_terasort100(buf, n, seed)
    recs = oracle_lib.gen_terasort100(n, seed)
    rng = np.random.default_rng(4)
    sample = recs[rng.choice(n, 20 * R, replace=False), :10]
    sample = sample[np.lexsort(sample.T[::-1])]
    bounds = np.ascontiguousarray(sample[np.linspace(0, len(sample) - 1, R - 1).astype(int)])
    sid = next_sid()
    engine.register_shuffle(sid, R, sgx.PART_RANGE_BYTES10, bounds, True, 100)
    lengths = engine.write_map(sid, 0, buf, n, 100, R)
    got = engine.map_output_bytes(sid, 0)
    engine.unregister_shuffle(sid)
    buf.free()
    want, counts = oracle_lib.map_write(recs, R, sgx.PART_RANGE_BYTES10, bounds, nthreads=16)
    del recs
    assert np.array_equal(lengths, counts * 100)
    assert np.array_equal(got, want.reshape(-1))


def test_shuffle_client_fetch_blocks_split_and_listener(sgx_lib, oracle_lib):
    """UcxShuffleClient.fetchBlocks (spark_3_0/UcxShuffleClient.scala:49-91): 130 block ids are
    split into requests of at most maxBlocksPerRequest (default 50, :53-58), every block
    reaches onBlockFetchSuccess with its bytes, and a request holding an unknown block
    reports onBlockFetchFailure for each of its blocks (the reference never does)."""
    R = 64
    mgr = sgx_lib.UcxShuffleManager(conf={"spark.shuffle.ucx.maxBlocksPerRequest": "50"})
    try:
        h = mgr.registerShuffle(3, sgx_lib.ShuffleDependency(sgx_lib.HashPartitioner(R)))
        outs = {}
        for m in (0, 1, 2):
            recs = oracle_lib.gen_uniform16(20_000 + m, 50 + m)
            mgr.getWriter(h, m).write(recs)
            outs[m] = oracle_lib.map_write(recs, R)

        class Listener(sgx_lib.BlockFetchingListener):
            def __init__(self):
                self.ok, self.failed = {}, {}

            def onBlockFetchSuccess(self, blockId, data):
                self.ok[blockId] = bytes(data)

            def onBlockFetchFailure(self, blockId, exception):
                self.failed[blockId] = exception

        ids = [f"shuffle_3_{m}_{r}" for r in range(R) for m in (0, 1, 2)][:130]
        lst = Listener()
        client = mgr.shuffleClient
        client.fetchBlocks("localhost", 1338, "1", ids, lst)
        # the reference's recursive halving: 130 -> 65 + 65 -> 32 + 33 + 32 + 33
        assert client.requests == 4 and client.request_sizes == [32, 33, 32, 33] and not lst.failed
        for b in ids:
            _, m, r = sgx_lib.parse_block_id(b)
            out, counts = outs[m]
            o = oracle_lib.offsets(counts)
            assert lst.ok[b] == out[o[r]:o[r + 1]].tobytes()
        bad = Listener()
        client.fetchBlocks("localhost", 1338, "1", ["shuffle_3_0_1", "shuffle_3_9_1"], bad)
        assert set(bad.failed) == {"shuffle_3_0_1", "shuffle_3_9_1"} and not bad.ok
        assert isinstance(bad.failed["shuffle_3_9_1"], sgx_lib.BlockNotFoundException)
    finally:
        mgr.stop()


def test_memory_pool_size_classes_and_reuse(sgx_lib, oracle_lib):
    """MemoryPool (memory/MemoryPool.scala:34-147): power-of-two classes from 4 KiB, close()
    returns a block to its class, preallocation fills a class; pool blocks serve as the
    fetch allocator of fetchBlocksByBlockIds."""
    import ctypes

    mgr = sgx_lib.UcxShuffleManager()
    try:
        pool = mgr.getTransport().hostBounceBufferMemoryPool
        a = pool.get(1)
        assert a.size == 4096 and a.isHostMemory
        b = pool.get(4097)
        assert b.size == 8192
        ctypes.memset(b.address, 7, b.size)  # host-visible pinned memory
        addr = b.address
        b.close()
        c = pool.get(5000)
        assert c.address == addr  # reused from the class's free list
        pool.preallocate(70_000, 3)
        alloc, idle = pool.stats()
        assert idle == 3 * 131072 and alloc >= idle + 4096 + 8192
        d = pool.get(100_000, host=False)
        assert d.size == 131072 and not d.isHostMemory
        for blk in (a, c, d):
            blk.close()
        # as the fetch allocator
        h = mgr.registerShuffle(4, sgx_lib.ShuffleDependency(sgx_lib.HashPartitioner(16)))
        recs = oracle_lib.gen_uniform16(3000, 4)
        mgr.getWriter(h, 0).write(recs)
        out, counts = oracle_lib.map_write(recs, 16)
        got = {}
        t = mgr.getTransport()
        t.fetchBlocksByBlockIds(1, [sgx_lib.UcxShuffleBlockId(4, 0, 5)], pool.get,
                                [lambda res: got.setdefault("r", res)])
        t.progress()
        mb = got["r"].getData()
        o = oracle_lib.offsets(counts) * 16
        assert ctypes.string_at(mb.address, mb.size) == out.reshape(-1)[o[5]:o[6]].tobytes()
        mb.close()
    finally:
        mgr.stop()


@pytest.mark.parametrize("workload", ["c3", "c4"])
def test_bench_other_workloads_json_line(workload):
    """bench.py --workload c3 | c4 at a small size: one JSON line with the contract's keys,
    the verified lengths, and the workload's record width and partition count."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--workload", workload, "--records", str(1 << 20),
           "--steps", "2", "--warmup", "1", "--no-cpu-baseline"]
    p = subprocess.run(cmd, cwd=root, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "ms_per_step", "roofline", "roofline_map_side", "config"):
        assert k in d, k
    assert d["verified_lengths_sum"] is True and d["value"] > 0
    assert d["config"]["record_bytes"] == (100 if workload == "c4" else 16)
    assert d["config"]["partitions"] == (4096 if workload == "c3" else 1024)
    assert d["roofline"]["algo_bytes_per_record"] == 2 * d["config"]["record_bytes"]
