"""GPU parity of the one-pass streaming commit: sgx_map_append only lands each
batch in HBM (host batches through PCIe, device batches copied, SGX_MEM_DEVICE_RETAINED batches
read in place) and sgx_map_commit partitions every batch in one pass through a chunk table --
the padded single-pass write when sgx_write_map would take it, else the two-pass write.  The
reference's writer receives the records as unbounded partition streams and merges spills in
spill order (ucx/NvkvShuffleMapOutputWriter.scala:106-148); whatever the batches, the lengths,
index offsets, blocks and reads must equal the oracle's map_write of all records in append
order, and sgx_write_map of the concatenation."""
import numpy as np
import pytest

from tests.test_padded import check_map, terasort_bounds

pytestmark = pytest.mark.gpu

_sid = [7000]


def next_sid():
    _sid[0] += 1
    return _sid[0]


def append_batches(e, sid, mid, recs, sizes, modes):
    """Append recs in batches of `sizes` records, batch k as modes[k % len(modes)]: "host",
    "device" (copied by the engine), "retained" (a slice of one device buffer, read in place
    at the commit).  Returns the device buffer the retained batches live in."""
    rb = recs.shape[1]
    dev = e.alloc(max(recs.nbytes, 16))
    dev.copy_from(np.ascontiguousarray(recs).reshape(-1))
    e.map_begin(sid, mid)
    pos = 0
    for k, sz in enumerate(sizes):
        mode = modes[k % len(modes)]
        part = np.ascontiguousarray(recs[pos:pos + sz])
        if mode == "host":
            e.map_append(sid, mid, part, sz, rb)
        elif mode == "device":
            tmp = e.alloc(max(part.nbytes, 16))
            tmp.copy_from(part.reshape(-1))
            e.map_append(sid, mid, tmp, sz, rb)
            tmp.free()  # the engine copied it
        else:
            e.map_append(sid, mid, dev, sz, rb, offset=pos * rb, retained=True)
        pos += sz
    assert pos == len(recs)
    return dev


def sizes_for(n, k, seed):
    rng = np.random.default_rng(seed)
    cuts = np.sort(rng.integers(0, n + 1, k - 1))
    s = np.diff(np.concatenate([[0], cuts, [n]])).tolist()
    return s


@pytest.mark.parametrize("R", [200, 1024])
@pytest.mark.parametrize("modes", [("retained",), ("host", "device", "retained")])
def test_commit_is_one_padded_pass(sgx_lib, engine, oracle_lib, R, modes):
    n = 1_300_007
    recs = oracle_lib.gen_uniform16(n, 0x51 + R)
    sizes = [0, 1, 4096] + sizes_for(n - 4097 - 3, 9, R) + [3, 0]
    sid = next_sid()
    engine.register_shuffle(sid, R)
    try:
        dev = append_batches(engine, sid, 0, recs, sizes, modes)
        lengths = engine.map_commit(sid, 0, R)
        dev.free()  # the commit returned: the retained batches are the caller's again
        check_map(engine, oracle_lib, recs, R, sid, 0, sgx_lib.LAYOUT_PADDED)
        engine.write_map(sid, 1, recs, n, 16, R)
        assert np.array_equal(lengths, engine.map_lengths(sid, 1, R))
        assert np.array_equal(engine.map_output_bytes(sid, 0), engine.map_output_bytes(sid, 1))
    finally:
        engine.unregister_shuffle(sid)


def test_async_commit_retained_until_lengths(sgx_lib, engine, oracle_lib):
    """An asynchronous commit (no lengths asked) only enqueues its pass, which reads the
    retained batches in place: the caller keeps them until the map's lengths are known
    (sgx_map_lengths here; sgx.h, SGX_MEM_DEVICE_RETAINED) and may then overwrite them."""
    R, n = 1024, 1_200_000
    recs = oracle_lib.gen_uniform16(n, 0x77)
    sid = next_sid()
    engine.register_shuffle(sid, R)
    try:
        dev = append_batches(engine, sid, 0, recs, sizes_for(n, 4, 5), ("retained",))
        assert engine.map_commit(sid, 0) is None
        engine.map_lengths(sid, 0, R)
        engine.gen_uniform16(dev, n, 0x78)  # the caller reuses its buffer
        dev.free()
        check_map(engine, oracle_lib, recs, R, sid, 0, sgx_lib.LAYOUT_PADDED)
    finally:
        engine.unregister_shuffle(sid)


@pytest.mark.parametrize("R", [2, 7, 1000])
@pytest.mark.parametrize("n,k", [(1, 1), (5, 3), (70_001, 5), (300_000, 300)])
def test_commit_padded_any_size_and_many_batches(sgx_lib, oracle_lib, R, n, k):
    """Small maps written padded (SGX_FLAG_PAD_ANY_SIZE), up to 300 batches = 300 chunks."""
    recs = oracle_lib.gen_uniform16(n, 0x52 + n + R)
    with sgx_lib.ShuffleEngine(device=0, flags=sgx_lib.FLAG_PAD_ANY_SIZE) as e:
        sid = next_sid()
        e.register_shuffle(sid, R)
        dev = append_batches(e, sid, 0, recs, sizes_for(n, k, n + R), ("retained", "host", "device"))
        e.map_commit(sid, 0, R)
        dev.free()
        check_map(e, oracle_lib, recs, R, sid, 0, sgx_lib.LAYOUT_PADDED)


def test_host_batches_land_packed(sgx_lib, engine, oracle_lib):
    """The writer Spark drives: pageable host batches, staged through the engine's two pinned
    buffers (a batch above one 64 MiB piece goes in several) and landed back to back, so 400
    batches still commit as one pass over ~one chunk per CU.  Bytes as one write's."""
    R = 1024
    sizes = [5_000_000] + [3_000] * 400 + [1, 0, 777_777]
    n = sum(sizes)
    recs = oracle_lib.gen_uniform16(n, 0x5A)
    sid = next_sid()
    engine.register_shuffle(sid, R)
    try:
        dev = append_batches(engine, sid, 0, recs, sizes, ("host",))
        dev.free()
        lengths = engine.map_commit(sid, 0, R)
        check_map(engine, oracle_lib, recs, R, sid, 0, sgx_lib.LAYOUT_PADDED)
        engine.write_map(sid, 1, recs, n, 16, R)
        assert np.array_equal(lengths, engine.map_lengths(sid, 1, R))
    finally:
        engine.unregister_shuffle(sid)


@pytest.mark.parametrize("shape", ["sorted_by_chunk", "one_partition_late"])
def test_commit_overflow_falls_back_bit_exact(sgx_lib, engine, oracle_lib, shape):
    """Keys the per-chunk sample cannot see coming: the guarded two-pass kernels rewrite the map
    through the same chunk table, contiguous and exact."""
    R, n = 1024, 1_500_000
    recs = oracle_lib.gen_uniform16(n, 79)
    if shape == "sorted_by_chunk":
        k = (np.arange(n) * 300 // n).astype(np.int64)
    else:
        line = np.arange(n) // 8
        k = np.where(line % 2 == 1, 5, np.arange(n) % 1024).astype(np.int64)
    recs[:, :8] = k.view(np.uint8).reshape(-1, 8)
    sid = next_sid()
    engine.register_shuffle(sid, R)
    try:
        dev = append_batches(engine, sid, 0, recs, sizes_for(n, 6, 3), ("retained", "host"))
        engine.map_commit(sid, 0, R)
        dev.free()
        check_map(engine, oracle_lib, recs, R, sid, 0, sgx_lib.LAYOUT_CONTIGUOUS)
    finally:
        engine.unregister_shuffle(sid)


@pytest.mark.parametrize("flags", ["NO_PADDED_MAP", "NO_DEFERRED_APPEND"])
@pytest.mark.parametrize("R", [3, 1024])
def test_commit_two_pass_and_per_batch_forms(sgx_lib, oracle_lib, flags, R):
    """The two-pass write over the chunk table (no padded map), and the round-4 form that
    partitions every batch on arrival (SGX_FLAG_NO_DEFERRED_APPEND): the same bytes."""
    n = 1_100_003
    recs = oracle_lib.gen_uniform16(n, 0x53 + R)
    with sgx_lib.ShuffleEngine(device=0, flags=getattr(sgx_lib, "FLAG_" + flags)) as e:
        sid = next_sid()
        e.register_shuffle(sid, R)
        dev = append_batches(e, sid, 0, recs, sizes_for(n, 7, R), ("retained", "device", "host"))
        e.map_commit(sid, 0, R)
        dev.free()
        check_map(e, oracle_lib, recs, R, sid, 0, sgx_lib.LAYOUT_CONTIGUOUS)


@pytest.mark.parametrize("R", [64, 1024])
@pytest.mark.parametrize("n,k", [(999, 3), (1_200_001, 7)])
def test_commit_terasort_records(sgx_lib, engine, oracle_lib, R, n, k):
    """100 B TeraSort records under the RangePartitioner over 10-byte keys: retained batches at
    offsets that are not 16 B-aligned are copied by the engine; the rest are read in place."""
    recs = oracle_lib.gen_terasort100(n, 0x54 + n + R)
    bounds = terasort_bounds(oracle_lib, R)
    sid = next_sid()
    engine.register_shuffle(sid, R, sgx_lib.PART_RANGE_BYTES10, bounds, True, 100)
    try:
        dev = append_batches(engine, sid, 0, recs, sizes_for(n, k, R), ("retained", "host", "retained", "device"))
        engine.map_commit(sid, 0, R)
        dev.free()
        want = sgx_lib.LAYOUT_PADDED if n >= (1 << 20) else sgx_lib.LAYOUT_CONTIGUOUS
        check_map(engine, oracle_lib, recs, R, sid, 0, want, sgx_lib.PART_RANGE_BYTES10, bounds)
    finally:
        engine.unregister_shuffle(sid)


def test_commit_terasort_sorted_input_falls_back(sgx_lib, oracle_lib):
    R, n = 256, 400_000
    recs = oracle_lib.gen_terasort100(n, 32)
    recs = np.ascontiguousarray(recs[np.lexsort(recs[:, :10].T[::-1])])
    bounds = terasort_bounds(oracle_lib, R)
    with sgx_lib.ShuffleEngine(device=0, flags=sgx_lib.FLAG_PAD_ANY_SIZE) as e:
        sid = next_sid()
        e.register_shuffle(sid, R, sgx_lib.PART_RANGE_BYTES10, bounds, True, 100)
        dev = append_batches(e, sid, 0, recs, sizes_for(n, 5, 9), ("retained", "host"))
        e.map_commit(sid, 0, R)
        dev.free()
        check_map(e, oracle_lib, recs, R, sid, 0, sgx_lib.LAYOUT_CONTIGUOUS, sgx_lib.PART_RANGE_BYTES10, bounds)


@pytest.mark.parametrize("codec", ["kryo", "kryo+lz4"])
def test_commit_kryo_padded_and_reads(sgx_lib, engine, oracle_lib, codec):
    """A Kryo shuffle's streaming map: the commit writes the records padded and the serializer
    reads them through the fragment table; lengths, bytes and reads equal one batch's."""
    R, n = 1024, 1_200_001
    recs = oracle_lib.gen_uniform16(n, 0x55)
    sid = next_sid()
    engine.register_shuffle(sid, R, serializer=sgx_lib.SER_KRYO)
    if codec == "kryo+lz4":
        engine.set_compression(sid, "lz4", 32768)
    try:
        dev = append_batches(engine, sid, 0, recs, sizes_for(n, 4, 1), ("retained", "host"))
        many = engine.map_commit(sid, 0, R)
        dev.free()
        assert engine.map_layout(sid, 0) == sgx_lib.LAYOUT_SERIALIZED_PADDED
        one = engine.write_map(sid, 1, recs, n, 16, R)
        assert np.array_equal(one, many)
        assert np.array_equal(engine.map_output_bytes(sid, 0), engine.map_output_bytes(sid, 1))
        seqs = oracle_lib.canonical_reducer_sequences([oracle_lib.map_write(recs, R)], R, 16)
        got = engine.read_records(sid, [0], 100, 300).reshape(-1, 16)
        assert np.array_equal(got, np.concatenate(seqs[100:300]))
    finally:
        engine.unregister_shuffle(sid)


def test_retained_batch_is_read_at_the_commit(sgx_lib, engine, oracle_lib):
    """A retained batch is read in place at the commit: what it holds THEN is what is written."""
    R, n = 200, 50_000
    a = oracle_lib.gen_uniform16(n, 1)
    b = oracle_lib.gen_uniform16(n, 2)
    sid = next_sid()
    engine.register_shuffle(sid, R)
    try:
        dev = engine.alloc(a.nbytes)
        dev.copy_from(a.reshape(-1))
        engine.map_begin(sid, 0)
        engine.map_append(sid, 0, dev, n, 16, retained=True)
        dev.copy_from(b.reshape(-1))  # still the caller's: the engine has not read it yet
        engine.map_commit(sid, 0, R)
        dev.free()
        check_map(engine, oracle_lib, b, R, sid, 0, sgx_lib.LAYOUT_CONTIGUOUS)
    finally:
        engine.unregister_shuffle(sid)
