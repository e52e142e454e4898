"""GPU parity of the single-pass padded map write (sgx_map_layout).

The padded write replaces the map side's full histogram by a sampled one: every
(partition, chunk) stream is written into a sub-bin sized from the sample, and the streams'
true counts give the lengths and index offsets.  Whatever the layout in HBM, every result the
engine hands out must equal the oracle's (identical partition lengths, index
offsets and per-block / per-reducer record sequences), read three ways: block fetches
(gathered from the fragments), the map's contiguous bytes (sgx_map_data, built on first use)
and the reduce-side reads.  A map whose keys defeat the sample overflows a sub-bin: the
device-side two-pass fallback must produce the same bytes."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

_sid = [5000]


def next_sid():
    _sid[0] += 1
    return _sid[0]


@pytest.fixture(scope="module")
def pad_engine(sgx_lib):
    """An engine that writes every hash map padded, whatever its size."""
    eng = sgx_lib.ShuffleEngine(device=0, flags=sgx_lib.FLAG_PAD_ANY_SIZE)
    yield eng
    eng.close()


def all_blocks(engine, sid, mid, R, dst=None):
    data, lens = engine.fetch_blocks(sid, [mid] * R, list(range(R)), dst=dst)
    return data, lens


def check_map(engine, oracle_lib, recs, R, sid, mid, want_layout, kind=0, bounds=None):
    rb = recs.shape[1]
    want, counts = oracle_lib.map_write(recs, R, kind, bounds, nthreads=8)
    lengths = engine.map_lengths(sid, mid, R)
    assert np.array_equal(lengths, counts * rb), "partition lengths / index offsets differ"
    assert engine.map_layout(sid, mid) == want_layout
    # block fetches, reducer by reducer, straight from the fragments
    data, lens = all_blocks(engine, sid, mid, R)
    assert np.array_equal(lens, counts * rb)
    assert np.array_equal(data.reshape(-1, rb), want)
    # a random subset of blocks, repeated and out of order, into device memory
    rng = np.random.default_rng(R)
    rids = rng.integers(0, R, 97)
    o = oracle_lib.offsets(counts) * rb
    flat = want.reshape(-1)
    sub = np.concatenate([flat[o[r]:o[r + 1]] for r in rids])
    dev = engine.alloc(max(int(sub.size), 16))
    engine.fetch_blocks(sid, [mid] * len(rids), rids, dst=dev)
    assert np.array_equal(dev.to_numpy(sub.size), sub)
    dev.free()
    # the contiguous bytes (built once), and the layout query is unchanged by them
    assert np.array_equal(engine.map_output_bytes(sid, mid).reshape(-1, rb), want)
    assert engine.map_layout(sid, mid) == want_layout


@pytest.mark.parametrize("R", [2, 3, 7, 200, 1000, 1024])
@pytest.mark.parametrize("n", [1, 8, 63, 8193, 100_003, 1_000_003])
def test_padded_random_sizes(sgx_lib, pad_engine, oracle_lib, R, n):
    recs = oracle_lib.gen_uniform16(n, 0xBADD + R * 7 + n)
    sid = next_sid()
    pad_engine.register_shuffle(sid, R)
    try:
        pad_engine.write_map(sid, 3, recs, n, 16, R)
        check_map(pad_engine, oracle_lib, recs, R, sid, 3, sgx_lib.LAYOUT_PADDED)
    finally:
        pad_engine.unregister_shuffle(sid)


def test_padded_is_the_default_from_2_20_records(sgx_lib, engine, oracle_lib):
    R = 1024
    sid = next_sid()
    engine.register_shuffle(sid, R)
    try:
        small = oracle_lib.gen_uniform16((1 << 20) - 1, 1)
        engine.write_map(sid, 0, small, len(small), 16, R)
        big = oracle_lib.gen_uniform16((1 << 20) + 5, 2)
        engine.write_map(sid, 1, big, len(big), 16, R)
        check_map(engine, oracle_lib, small, R, sid, 0, sgx_lib.LAYOUT_CONTIGUOUS)
        check_map(engine, oracle_lib, big, R, sid, 1, sgx_lib.LAYOUT_PADDED)
    finally:
        engine.unregister_shuffle(sid)
    with sgx_lib.ShuffleEngine(device=0, flags=sgx_lib.FLAG_NO_PADDED_MAP) as e:
        e.register_shuffle(1, R)
        e.write_map(1, 0, big, len(big), 16, R)
        check_map(e, oracle_lib, big, R, 1, 0, sgx_lib.LAYOUT_CONTIGUOUS)


@pytest.mark.parametrize("R", [200, 1024])
def test_padded_zipf_and_collisions(sgx_lib, pad_engine, oracle_lib, R):
    """Skewed keys (Zipf(1.1): one partition holds ~11.5 % of the records) and few distinct
    keys: the sample sizes the hot sub-bins from their share."""
    cdf = oracle_lib.zipf_cdf(1.1, 1 << 20)
    z = oracle_lib.gen_zipf16(2_000_003, 11, cdf)
    few = oracle_lib.gen_uniform16(300_001, 12)
    few[:, :8] = (np.arange(len(few)) % 5).astype(np.int64).view(np.uint8).reshape(-1, 8)
    for recs in (z, few):
        sid = next_sid()
        pad_engine.register_shuffle(sid, R)
        try:
            pad_engine.write_map(sid, 0, recs, len(recs), 16, R)
            check_map(pad_engine, oracle_lib, recs, R, sid, 0, sgx_lib.LAYOUT_PADDED)
        finally:
            pad_engine.unregister_shuffle(sid)


@pytest.mark.parametrize("shape", ["sorted_by_chunk", "one_partition_late"])
def test_padded_overflow_falls_back_bit_exact(sgx_lib, pad_engine, oracle_lib, shape):
    """Keys the systematic sample cannot see coming: sorted so each chunk holds one
    partition (every sub-bin overflows), or one partition absent from the sampled lines and
    dense elsewhere.  The guarded two-pass kernels rewrite the map on the device: the layout
    is contiguous and every byte equals the oracle's; the shuffle's next map skips the
    padded attempt and is still exact."""
    R, n = 1024, 1_500_000
    recs = oracle_lib.gen_uniform16(n, 77)
    if shape == "sorted_by_chunk":
        k = (np.arange(n) * 300 // n).astype(np.int64)
    else:
        # partition 5 in every line except the sampled ones (the sample reads line 0 of
        # every `stride` lines; stride is 2 here, so odd lines are never sampled)
        line = np.arange(n) // 8
        k = np.where(line % 2 == 1, 5, np.arange(n) % 1024).astype(np.int64)
    recs[:, :8] = k.view(np.uint8).reshape(-1, 8)
    sid = next_sid()
    pad_engine.register_shuffle(sid, R)
    try:
        pad_engine.write_map(sid, 0, recs, n, 16, R)
        check_map(pad_engine, oracle_lib, recs, R, sid, 0, sgx_lib.LAYOUT_CONTIGUOUS)
        again = oracle_lib.gen_uniform16(n, 78)
        pad_engine.write_map(sid, 1, again, n, 16, R)
        check_map(pad_engine, oracle_lib, again, R, sid, 1, sgx_lib.LAYOUT_CONTIGUOUS)
    finally:
        pad_engine.unregister_shuffle(sid)


def test_async_host_writes_behind_an_overflowing_map(sgx_lib, pad_engine, oracle_lib):
    """Two asynchronous writes of host batches on one thread, the first overflowing its
    sub-bins: its guarded fallback runs on the tail stream and reads the staged input, which
    the second write stages its own records into -- the second copy must wait for that tail
    (Ctx::stage_input).  Both maps must equal the oracle's."""
    R, n = 1024, 1_500_000
    first = oracle_lib.gen_uniform16(n, 91)
    first[:, :8] = (np.arange(n) * 300 // n).astype(np.int64).view(np.uint8).reshape(-1, 8)
    second = oracle_lib.gen_uniform16(n, 92)
    sid1, sid2 = next_sid(), next_sid()  # two shuffles: the second's maps still try padded
    pad_engine.register_shuffle(sid1, R)
    pad_engine.register_shuffle(sid2, R)
    try:
        for _ in range(2):
            pad_engine.write_map(sid1, 0, first, n, 16)   # asynchronous (no lengths asked)
            pad_engine.write_map(sid2, 0, second, n, 16)
            check_map(pad_engine, oracle_lib, first, R, sid1, 0, sgx_lib.LAYOUT_CONTIGUOUS)
            check_map(pad_engine, oracle_lib, second, R, sid2, 0, sgx_lib.LAYOUT_PADDED)
    finally:
        pad_engine.unregister_shuffle(sid1)
        pad_engine.unregister_shuffle(sid2)


@pytest.mark.parametrize("R", [2048, 4096])
@pytest.mark.parametrize("shape", ["uniform", "zipf", "one_super", "hot_partition", "few_keys", "tiny"])
def test_padded_split_r_over_1024(sgx_lib, pad_engine, oracle_lib, R, shape):
    """R > 1024 (config C3's 4096): the padded two-level split -- hot partitions chosen from
    the sample stream from level 1 into their final sub-bins, the rest through their
    super-partition's scratch sub-bins and level 2's (super, chunk) fragments."""
    n = 2_000_003 if shape != "tiny" else 777
    if shape == "zipf":
        recs = oracle_lib.gen_zipf16(n, 5, oracle_lib.zipf_cdf(1.1, 1 << 20))
    else:
        recs = oracle_lib.gen_uniform16(n, 6 + R)
        k = recs[:, :8].copy().view("<i8").reshape(-1)
        if shape == "one_super":  # every key in super-partition 3 (64 partitions)
            k = 3 * 64 + (k & 63)
        elif shape == "hot_partition":  # one partition holds ~40 % of the records
            k = np.where(np.arange(n) % 5 < 2, 17, k)
        elif shape == "few_keys":
            k = k % 7
        recs[:, :8] = k.astype(np.int64).view(np.uint8).reshape(-1, 8)
    sid = next_sid()
    pad_engine.register_shuffle(sid, R)
    try:
        pad_engine.write_map(sid, 0, recs, n, 16, R)
        check_map(pad_engine, oracle_lib, recs, R, sid, 0, sgx_lib.LAYOUT_PADDED)
    finally:
        pad_engine.unregister_shuffle(sid)


def test_padded_split_sorted_input_falls_back(sgx_lib, pad_engine, oracle_lib):
    """Sorted keys at R = 4096: sub-bins overflow, the single-pass lane-ordered fallback runs."""
    R, n = 4096, 1_000_000
    recs = oracle_lib.gen_uniform16(n, 8)
    recs[:, :8] = (np.arange(n) * R // n).astype(np.int64).view(np.uint8).reshape(-1, 8)
    sid = next_sid()
    pad_engine.register_shuffle(sid, R)
    try:
        pad_engine.write_map(sid, 0, recs, n, 16, R)
        check_map(pad_engine, oracle_lib, recs, R, sid, 0, sgx_lib.LAYOUT_CONTIGUOUS)
    finally:
        pad_engine.unregister_shuffle(sid)


def terasort_bounds(oracle_lib, R, seed=0xC4):
    sample = oracle_lib.gen_terasort100(20 * R, seed)[:, :10]
    sample = sample[np.lexsort(sample.T[::-1])]
    return np.ascontiguousarray(sample[[int(len(sample) / R * (i + 1)) for i in range(R - 1)]])


@pytest.mark.parametrize("R", [2, 64, 1024])
@pytest.mark.parametrize("n", [1, 999, 50_001, 600_003])
def test_padded_terasort_records(sgx_lib, pad_engine, oracle_lib, R, n):
    """TeraSort's 100 B records under a RangePartitioner over 10-byte keys (config C4): the
    sampled histogram searches the bounds, the LDS-staged wide-record K4 writes the sub-bins."""
    recs = oracle_lib.gen_terasort100(n, 0x7E + n + R)
    bounds = terasort_bounds(oracle_lib, R)
    sid = next_sid()
    pad_engine.register_shuffle(sid, R, sgx_lib.PART_RANGE_BYTES10, bounds, True, 100)
    try:
        pad_engine.write_map(sid, 0, recs, n, 100, R)
        check_map(pad_engine, oracle_lib, recs, R, sid, 0, sgx_lib.LAYOUT_PADDED, sgx_lib.PART_RANGE_BYTES10, bounds)
    finally:
        pad_engine.unregister_shuffle(sid)


def test_padded_terasort_sorted_input_falls_back(sgx_lib, pad_engine, oracle_lib):
    """Records already sorted by key: each chunk holds a few partitions, every sub-bin of them
    overflows and the wide-record two-pass fallback rewrites the map on the device."""
    R, n = 256, 400_000
    recs = oracle_lib.gen_terasort100(n, 31)
    recs = np.ascontiguousarray(recs[np.lexsort(recs[:, :10].T[::-1])])
    bounds = terasort_bounds(oracle_lib, R)
    sid = next_sid()
    pad_engine.register_shuffle(sid, R, sgx_lib.PART_RANGE_BYTES10, bounds, True, 100)
    try:
        pad_engine.write_map(sid, 0, recs, n, 100, R)
        check_map(pad_engine, oracle_lib, recs, R, sid, 0, sgx_lib.LAYOUT_CONTIGUOUS, sgx_lib.PART_RANGE_BYTES10,
                  bounds)
    finally:
        pad_engine.unregister_shuffle(sid)


def test_padded_reads_index_and_reattempt(sgx_lib, pad_engine, oracle_lib, tmp_path):
    """Several padded maps of one shuffle: the reduce-side reads (records, sorted, grouped,
    summed) over all of them, the index + data files of one, and a re-attempt of a map with
    another size (the slot's buffers are reused)."""
    import struct

    R = 256
    sid = next_sid()
    pad_engine.register_shuffle(sid, R)
    try:
        outs = []
        for m in range(3):
            recs = oracle_lib.gen_uniform16(200_000 + 1000 * m, 90 + m)
            recs[:, :8] = (recs[:, :8].view("<i8") % 50_000).view(np.uint8)  # repeated keys
            pad_engine.write_map(sid, m, recs, len(recs), 16, R)
            outs.append(oracle_lib.map_write(recs, R))
        # re-attempt of map 1 with other records
        recs = oracle_lib.gen_uniform16(150_001, 99)
        pad_engine.write_map(sid, 1, recs, len(recs), 16, R)
        outs[1] = oracle_lib.map_write(recs, R)
        for m in range(3):
            assert pad_engine.map_layout(sid, m) == sgx_lib.LAYOUT_PADDED
        seqs = oracle_lib.canonical_reducer_sequences(outs, R, 16)
        r0, r1 = 10, 200
        got = pad_engine.read_records(sid, [0, 1, 2], r0, r1)
        assert np.array_equal(got.reshape(-1, 16), np.concatenate(seqs[r0:r1]))
        got = pad_engine.read_sorted(sid, [0, 1, 2], r0, r1)
        assert np.array_equal(got.reshape(-1, 16), oracle_lib.reduce_sorted(seqs[r0:r1]))
        k, st, v = pad_engine.read_grouped(sid, [0, 1, 2], r0, r1, sgx_lib.AGG_GROUP)
        wk, wst, wv = oracle_lib.reduce_grouped(seqs[r0:r1], "group")
        assert np.array_equal(k, wk) and np.array_equal(st, wst) and np.array_equal(v, wv)
        k, s = pad_engine.read_grouped(sid, [0, 1, 2], r0, r1, sgx_lib.AGG_SUM)
        wk, ws = oracle_lib.reduce_grouped(seqs[r0:r1], "sum")
        assert np.array_equal(k, wk) and np.array_equal(s, ws)
        idx, dat = str(tmp_path / "s.index"), str(tmp_path / "s.data")
        pad_engine.write_index(sid, 2, idx, dat, R)
        out, counts = outs[2]
        assert open(dat, "rb").read() == out.tobytes()
        raw = open(idx, "rb").read()
        offs = struct.unpack(">%dq" % (R + 1), raw)
        assert list(offs) == list(oracle_lib.offsets(counts) * 16)
    finally:
        pad_engine.unregister_shuffle(sid)


def test_padded_fetch_into_unaligned_device_memory(sgx_lib, pad_engine, oracle_lib):
    """The fragment gather copies 16 B at a time: a destination that is not 16-byte aligned
    is served from the map's contiguous copy instead -- same bytes."""
    class DeviceView:
        """A device-tensor-like view 4 bytes into an engine allocation (no torch: its own HIP
        runtime and the engine's do not share a process here)."""

        is_cuda = True

        def __init__(self, buf, off, n):
            self.buf, self.off, self.n = buf, off, n

        def data_ptr(self):
            return self.buf.ptr + self.off

        def is_contiguous(self):
            return True

        def numel(self):
            return self.n

        def element_size(self):
            return 1

    R = 100
    recs = oracle_lib.gen_uniform16(50_001, 5)
    want, counts = oracle_lib.map_write(recs, R)
    sid = next_sid()
    pad_engine.register_shuffle(sid, R)
    try:
        pad_engine.write_map(sid, 0, recs, len(recs), 16, R)
        buf = pad_engine.alloc(recs.nbytes + 64)
        pad_engine.fetch_blocks(sid, [0] * R, list(range(R)), dst=DeviceView(buf, 4, recs.nbytes))
        assert np.array_equal(buf.to_numpy(recs.nbytes, offset=4), want.reshape(-1))
        assert pad_engine.map_layout(sid, 0) == sgx_lib.LAYOUT_PADDED
        buf.free()
    finally:
        pad_engine.unregister_shuffle(sid)


@pytest.mark.parametrize("p2p", [True, False])
def test_padded_exchange_one_rank(sgx_lib, oracle_lib, p2p):
    """A one-rank communicator (the self-exchange stand-in for the multi-rank path).  With the
    direct peer gather (the default) maps written after it stay single-pass (padded) and the
    exchange gathers their blocks from the fragments; with SGX_FLAG_NO_P2P_EXCHANGE they are
    written contiguous for RCCL's send / recv, and a map written padded before the
    communicator existed is exchanged through its contiguous copy.  Every way gives the
    oracle's blocks, and the exchange moves exactly the published bytes."""
    R = 1024
    flags = sgx_lib.FLAG_PAD_ANY_SIZE | (0 if p2p else sgx_lib.FLAG_NO_P2P_EXCHANGE)
    with sgx_lib.ShuffleEngine(device=0, flags=flags) as e:
        e.register_shuffle(1, R)
        early = oracle_lib.gen_uniform16(300_000, 22)
        e.write_map(1, 5, early, len(early), 16, R)
        assert e.map_layout(1, 5) == sgx_lib.LAYOUT_PADDED
        e.comm_init(1, 0, sgx_lib.get_unique_id())
        recs = oracle_lib.gen_uniform16(400_000, 23)
        e.write_map(1, 6, recs, len(recs), 16, R)
        assert e.map_layout(1, 6) == (sgx_lib.LAYOUT_PADDED if p2p else sgx_lib.LAYOUT_CONTIGUOUS)
        e.stats_reset()
        e.exchange(1)
        e.sync()
        assert e.exchange_bytes() == {"sent": 0, "kept": 16 * (len(early) + len(recs)), "rounds": 1}
        for mid, src in ((5, early), (6, recs)):
            data, lens = e.fetch_blocks(1, [mid] * R, list(range(R)))
            out, counts = oracle_lib.map_write(src, R)
            assert np.array_equal(data.reshape(-1, 16), out)
            assert np.array_equal(np.asarray(lens), counts * 16)


def test_padded_concurrent_writers(sgx_lib, pad_engine, oracle_lib):
    """Map tasks on several threads (one stream and scratch each) writing padded maps of one
    shuffle at once."""
    import threading

    R = 512
    sid = next_sid()
    pad_engine.register_shuffle(sid, R)
    recs = [oracle_lib.gen_uniform16(300_000 + 13 * m, 300 + m) for m in range(6)]
    errs = []

    def work(m):
        try:
            pad_engine.write_map(sid, m, recs[m], len(recs[m]), 16, R)
        except Exception as ex:  # pragma: no cover - reported below
            errs.append(ex)
        finally:
            pad_engine.release_thread()

    th = [threading.Thread(target=work, args=(m,)) for m in range(6)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    try:
        assert not errs, errs
        for m in range(6):
            check_map(pad_engine, oracle_lib, recs[m], R, sid, m, sgx_lib.LAYOUT_PADDED)
    finally:
        pad_engine.unregister_shuffle(sid)


@pytest.mark.slow
def test_full_c1_padded_fetch_bit_exact(sgx_lib, engine, oracle_lib):
    """Config C1 at full size through the default engine: the map is written padded (one pass
    over the records) and every block, gathered from the fragments reducer by reducer into
    device memory, equals the oracle's partition-contiguous output."""
    n, R, seed = 1 << 28, 1024, 0x5EEDC0DE
    buf = engine.alloc(n * 16)
    engine.gen_uniform16(buf, n, seed)
    sid = next_sid()
    engine.register_shuffle(sid, R)
    lengths = engine.write_map(sid, 0, buf, n, 16, R)
    assert engine.map_layout(sid, 0) == sgx_lib.LAYOUT_PADDED
    engine.fetch_blocks(sid, [0] * R, list(range(R)), dst=buf)
    got = buf.to_numpy()
    engine.unregister_shuffle(sid)
    buf.free()
    recs = oracle_lib.gen_uniform16(n, seed)
    want, counts = oracle_lib.map_write(recs, R, nthreads=16)
    del recs
    assert np.array_equal(lengths, counts * 16)
    assert np.array_equal(got, want.reshape(-1))


@pytest.mark.parametrize("overlap", [False, True])
@pytest.mark.parametrize("R", [1024, 4096])
def test_back_to_back_async_writes(sgx_lib, oracle_lib, R, overlap):
    """Asynchronous writes issued back to back from one thread (the
    tail on a second stream, the split's front on a third; by default consecutive writes also
    alternate between two streams, SGX_FLAG_NO_OVERLAP_WRITES keeps them on one): host and device inputs mixed, a
    map id written twice (the second attempt wins), every map checked after one sync."""
    n = 300_007
    sid = next_sid()
    pad_engine = sgx_lib.ShuffleEngine(
        device=0, flags=sgx_lib.FLAG_PAD_ANY_SIZE | (0 if overlap else sgx_lib.FLAG_NO_OVERLAP_WRITES))
    pad_engine.register_shuffle(sid, R)
    bufs = []
    try:
        want = {}
        plan = [(0, "host"), (1, "dev"), (2, "host"), (0, "dev"), (3, "dev"), (4, "host")]
        for k, (mid, kind) in enumerate(plan):
            recs = oracle_lib.gen_zipf16(n, 0x7A0 + k, oracle_lib.zipf_cdf(1.1, 1 << 16)) if k % 2 else \
                oracle_lib.gen_uniform16(n, 0x7A0 + k)
            if kind == "dev":
                b = pad_engine.alloc(recs.nbytes)
                b.copy_from(recs)
                bufs.append(b)  # kept alive until the writes have run
                pad_engine.write_map(sid, mid, b, n, 16)
            else:
                pad_engine.write_map(sid, mid, recs, n, 16)
            want[mid] = recs
        pad_engine.sync()
        for mid, recs in want.items():
            check_map(pad_engine, oracle_lib, recs, R, sid, mid, sgx_lib.LAYOUT_PADDED)
    finally:
        pad_engine.unregister_shuffle(sid)
        for b in bufs:
            b.free()
        pad_engine.close()
