"""Kryo-framed map output: Spark's KryoSerializer stream of (Long,
Long) records with spark.shuffle.compress=false, written and read back on the GPU.

CPU tests pin the two oracle restatements (pure Python, numpy) to the hand-computed known
answers and to each other.  GPU tests compare the HIP path, through the C ABI, with the
oracle and the golden fixtures byte for byte: partition lengths (= index offsets), the
partition-contiguous Kryo stream, the index and data files, fetched blocks, and the
decoded records / sorted / grouped reads of a Kryo shuffle against the fixed-codec ones.
Parity against a JVM is unpinned (no JVM here)."""
import glob
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN


def _edge_records(n, seed):
    rng = np.random.default_rng(seed)
    k = rng.integers(-2**63, 2**63 - 1, size=n, dtype=np.int64, endpoint=True)
    v = rng.integers(-2**63, 2**63 - 1, size=n, dtype=np.int64, endpoint=True)
    sh = rng.integers(0, 64, size=n)
    k = np.where(np.arange(n) % 3 == 0, k, k >> sh)
    v = np.where(np.arange(n) % 2 == 0, v >> rng.integers(0, 64, size=n), v)
    kv = np.stack([k, v], axis=1)
    return np.ascontiguousarray(kv).view(np.uint8).reshape(-1, 16)


# --------------------------------------------------------------------------- CPU ----
def test_kats_python_restatement():
    from oracle import spark_semantics as S

    with open(os.path.join(GOLDEN, "kats_kryo.json")) as f:
        kats = json.load(f)
    for v, h in kats["varlong"]:
        assert S.kryo_write_var_long(v).hex() == h
        assert S.kryo_read_var_long(bytes.fromhex(h), 0) == (v, len(h) // 2)
    for kv, h in kats["record"]:
        assert S.kryo_serialize_pairs([tuple(kv)]).hex() == h
        assert S.kryo_deserialize_pairs(bytes.fromhex(h)) == [tuple(kv)]


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_numpy_restatement_matches_python(seed):
    import oracle
    from oracle import spark_semantics as S

    recs = _edge_records(2000 + seed, seed)
    pairs = [tuple(map(int, r)) for r in recs.view(np.int64).reshape(-1, 2)]
    want = S.kryo_serialize_pairs(pairs)
    assert oracle.kryo_serialize(recs).tobytes() == want
    assert int(oracle.kryo_record_lengths(recs).sum()) == len(want)
    assert S.kryo_deserialize_pairs(want) == pairs


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "kryo_*.npz"))))
def test_golden_fixtures_consistent(path, oracle_lib):
    z = np.load(path)
    R = int(z["num_partitions"])
    out, counts = oracle_lib.map_write(z["records"], R)
    assert np.array_equal(oracle_lib.kryo_serialize(out), z["kryo_stream"])
    off = oracle_lib.kryo_partition_offsets(out, counts)
    assert np.array_equal(np.diff(off), z["kryo_lengths"])
    assert oracle_lib.index_bytes(z["kryo_lengths"]) == z["index"].tobytes()


def test_dependency_rejects_kryo_on_wide_records(sgx_lib):
    with pytest.raises(sgx_lib.UnsupportedOperationException):
        sgx_lib.ShuffleDependency(sgx_lib.HashPartitioner(4), 100, serializer="kryo")
    with pytest.raises(sgx_lib.IllegalArgumentException):
        sgx_lib.ShuffleDependency(sgx_lib.HashPartitioner(4), 16, serializer="java")


# --------------------------------------------------------------------------- GPU ----
_sid = [5000]


def _next_sid():
    _sid[0] += 1
    return _sid[0]


def _kryo_map(engine, recs, R, map_id=0, sid=None, device=False):
    import sparkucx_amd as sgx

    if sid is None:
        sid = _next_sid()
        engine.register_shuffle(sid, R, serializer=sgx.SER_KRYO)
    src = np.ascontiguousarray(recs)
    if device:
        buf = engine.alloc(max(src.nbytes, 16))
        buf.copy_from(src)
        src = buf
    lengths = engine.write_map(sid, map_id, src, recs.shape[0], 16, R)
    return sid, lengths


@pytest.mark.gpu
@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "kryo_*.npz"))))
def test_gpu_golden_kryo(engine, path, tmp_path):
    z = np.load(path)
    R = int(z["num_partitions"])
    sid, lengths = _kryo_map(engine, z["records"], R)
    try:
        assert np.array_equal(lengths, z["kryo_lengths"]), "Kryo partition lengths differ"
        assert np.array_equal(engine.map_output_bytes(sid, 0), z["kryo_stream"]), "Kryo stream differs"
        idx, dat = str(tmp_path / "i"), str(tmp_path / "d")
        engine.write_index(sid, 0, idx, dat, R)
        assert open(idx, "rb").read() == z["index"].tobytes()
        assert open(dat, "rb").read() == z["kryo_stream"].tobytes()
    finally:
        engine.unregister_shuffle(sid)


@pytest.mark.gpu
@pytest.mark.parametrize("n,R,seed", [(0, 16, 0), (1, 1, 1), (2047, 7, 2), (2048, 1024, 3), (2049, 200, 4),
                                      (100_003, 1024, 5), (1 << 20, 1024, 6), (300_001, 4096, 7)])
def test_gpu_kryo_vs_oracle(engine, oracle_lib, n, R, seed):
    recs = _edge_records(n, seed) if seed % 2 else oracle_lib.gen_uniform16(n, 0x5EEDC0DE + seed)
    out, counts = oracle_lib.map_write(recs, R, nthreads=8)
    want = oracle_lib.kryo_serialize(out)
    off = oracle_lib.kryo_partition_offsets(out, counts)
    sid, lengths = _kryo_map(engine, recs, R, device=bool(seed & 2))
    try:
        assert np.array_equal(lengths, np.diff(off))
        got = engine.map_output_bytes(sid, 0)
        if not np.array_equal(got, want):
            bad = np.nonzero(got != want)[0] if got.shape == want.shape else [-1]
            pytest.fail(f"Kryo stream differs ({got.size} vs {want.size} bytes), first at {bad[:5]}")
    finally:
        engine.unregister_shuffle(sid)


@pytest.mark.gpu
def test_gpu_kryo_fetch_and_reduce_side(engine, oracle_lib):
    """Blocks of several maps: fetched bytes are the Kryo slices (byte-granular gather);
    read_records decodes them on the GPU to the canonical records; sorted and grouped reads
    of the Kryo shuffle equal those of the same data under the fixed codec."""
    import sparkucx_amd as sgx

    R, nmaps = 64, 3
    maps = [(_edge_records(5000 + 37 * m, 11 + m) if m == 1 else oracle_lib.gen_uniform16(5000 + 37 * m, 99 + m))
            for m in range(nmaps)]
    sk, sf = _next_sid(), _next_sid()
    engine.register_shuffle(sk, R, serializer=sgx.SER_KRYO)
    engine.register_shuffle(sf, R)
    try:
        outs = []
        for m, recs in enumerate(maps):
            _kryo_map(engine, recs, R, map_id=m, sid=sk)
            engine.write_map(sf, m, np.ascontiguousarray(recs), recs.shape[0], 16, R)
            outs.append(oracle_lib.map_write(recs, R))
        # fetch: arbitrary block order, byte-exact slices of each map's Kryo stream
        mids = [2, 0, 1, 1, 0, 2]
        rids = [5, 63, 0, 17, 17, 40]
        data, lens = engine.fetch_blocks(sk, mids, rids)
        pos = 0
        for m, r, L in zip(mids, rids, lens):
            out, counts = outs[m]
            o = oracle_lib.offsets(counts)
            want = oracle_lib.kryo_serialize(out[o[r]:o[r + 1]])
            assert L == want.size
            assert np.array_equal(data[pos:pos + L], want)
            pos += L
        # decoded records, canonical order, against the fixed-codec blocks
        for r0, r1 in [(0, R), (5, 6), (10, 40)]:
            got = engine.read_records(sk, list(range(nmaps)), r0, r1)
            want = engine.read_records(sf, list(range(nmaps)), r0, r1)
            assert np.array_equal(got, want)
            assert np.array_equal(engine.read_sorted(sk, list(range(nmaps)), r0, r1),
                                  engine.read_sorted(sf, list(range(nmaps)), r0, r1))
            for agg in (sgx.AGG_GROUP, sgx.AGG_SUM):
                a = engine.read_grouped(sk, list(range(nmaps)), r0, r1, agg)
                b = engine.read_grouped(sf, list(range(nmaps)), r0, r1, agg)
                for x, y in zip(a, b):
                    assert np.array_equal(x, y)
        assert engine.read_records(sk, [0], 3, 3).size == 0
    finally:
        engine.unregister_shuffle(sk)
        engine.unregister_shuffle(sf)


@pytest.mark.gpu
def test_gpu_kryo_plugin_mirror(tmp_path, oracle_lib):
    """The plugin mirror end to end with serializer="kryo": writer lengths, index file
    through the resolver, and the reader's records."""
    import sparkucx_amd as sgx

    R = 200
    recs = oracle_lib.gen_uniform16(20_000, 7)
    out, counts = oracle_lib.map_write(recs, R)
    off = oracle_lib.kryo_partition_offsets(out, counts)
    mgr = sgx.UcxShuffleManager(conf={"spark.shuffle.compress": "false"}, device=0, localDir=str(tmp_path))
    try:
        h = mgr.registerShuffle(3, sgx.ShuffleDependency(sgx.HashPartitioner(R), 16, serializer="kryo"))
        w = mgr.getWriter(h, 0)
        w.write(recs)
        assert np.array_equal(w.getPartitionLengths(), np.diff(off))
        got = mgr.getReader(h, 0, R).read()
        assert np.array_equal(got, out)
    finally:
        mgr.stop()


@pytest.mark.gpu
def test_gpu_set_serializer_state_rules(engine):
    import sparkucx_amd as sgx

    sid = _next_sid()
    engine.register_shuffle(sid, 8)
    try:
        engine.write_map(sid, 0, np.zeros((4, 16), np.uint8), 4, 16, 8)
        with pytest.raises(sgx.IllegalStateException):
            engine.set_serializer(sid, sgx.SER_KRYO)
    finally:
        engine.unregister_shuffle(sid)
    sid = _next_sid()
    engine.register_shuffle(sid, 8, record_bytes=100)
    try:
        with pytest.raises(sgx.UnsupportedOperationException):
            engine.set_serializer(sid, sgx.SER_KRYO)
    finally:
        engine.unregister_shuffle(sid)


@pytest.mark.gpu
def test_gpu_kryo_multi_block_scan_round_trip(engine, oracle_lib):
    """> 4096 tiles on both sides (two-level tile scan): 5M records framed and decoded."""
    import sparkucx_amd as sgx

    n, R = 5_000_000, 1024
    recs = oracle_lib.gen_uniform16(n, 1234)
    out, counts = oracle_lib.map_write(recs, R, nthreads=8)
    off = oracle_lib.kryo_partition_offsets(out, counts)
    sid, lengths = _kryo_map(engine, recs, R, device=True)
    try:
        assert np.array_equal(lengths, np.diff(off))
        assert np.array_equal(engine.map_output_bytes(sid, 0), oracle_lib.kryo_serialize(out))
        got = engine.read_records(sid, [0], 0, R).reshape(-1, 16)
        assert np.array_equal(got, out)
    finally:
        engine.unregister_shuffle(sid)
        _ = sgx


@pytest.mark.gpu
def test_gpu_kryo_exchange_single_rank(engine, oracle_lib):
    """sgx_exchange on a Kryo shuffle (one rank, no communicator: the received blocks alias
    the map's Kryo stream); fetched blocks and decoded records come from the round."""
    import sparkucx_amd as sgx

    R = 32
    recs = _edge_records(20_000, 77)
    out, counts = oracle_lib.map_write(recs, R)
    o = oracle_lib.offsets(counts)
    sid, lengths = _kryo_map(engine, recs, R, map_id=4)
    try:
        engine.exchange(sid)
        engine.sync()
        data, lens = engine.fetch_blocks(sid, [4, 4], [31, 0])
        want = np.concatenate([oracle_lib.kryo_serialize(out[o[31]:o[32]]), oracle_lib.kryo_serialize(out[o[0]:o[1]])])
        assert np.array_equal(data, want)
        assert np.array_equal(engine.read_records(sid, [4], 0, R).reshape(-1, 16), out)
    finally:
        engine.unregister_shuffle(sid)
        _ = sgx


def test_varlong_pinned_to_protobuf_sint64():
    """Kryo 4's writeVarLong(v, optimizePositive=false) is zigzag + little-endian base-128
    groups, like protobuf's sint64 varint, except that Kryo stops at 9 bytes (the 9th holds
    8 bits).  Below 2^56 after zigzag -- encodings of 1..8 bytes -- the two must agree byte for
    byte: the restatement (and the numpy oracle the GPU tests compare with) is checked
    against protobuf's independent encoder there; the 9-byte form stays restated."""
    pb = pytest.importorskip("google.protobuf.internal.encoder")
    wf = pytest.importorskip("google.protobuf.internal.wire_format")
    from oracle import spark_semantics as ss

    import oracle as orc

    rng = np.random.default_rng(3)
    vals = [0, 1, -1, 63, -64, 64, -65, 2**55 - 1, -(2**55)]
    for bits in range(1, 56):
        vals += [int(x) for x in rng.integers(-(2**bits), 2**bits, 20)]
    for v in vals:
        z = wf.ZigZagEncode(v)
        assert z < 2**56
        want = pb._VarintBytes(z)
        assert ss.kryo_write_var_long(v) == want, v
    recs = np.zeros((len(vals), 2), dtype=np.int64)
    recs[:, 0] = vals
    recs[:, 1] = vals[::-1]
    stream = orc.kryo_serialize(recs.view(np.uint8).reshape(-1, 16)).tobytes()
    want = b"".join(b"\x09" + pb._VarintBytes(wf.ZigZagEncode(int(k))) + b"\x09" + pb._VarintBytes(wf.ZigZagEncode(int(x)))
                    for k, x in recs)
    assert stream == want


@pytest.mark.gpu
@pytest.mark.parametrize("R,shape", [(1024, "uniform"), (200, "uniform"), (4096, "uniform"), (1024, "overflow"),
                                     (64, "lz4"), (2, "uniform"), (1024, "tiny"), (1024, "zipf"), (4096, "zipf")])
def test_gpu_kryo_padded_write(sgx_lib, oracle_lib, R, shape):
    """A Kryo shuffle's map written padded: the serializer reads the records
    through the fragment table and publishes the same stream, lengths, blocks and LZ4 frames
    as the two-pass write; keys the sample misses ("overflow") overflow a sub-bin and the
    serializer reads the fallback's contiguous records; R = 4096 goes through the padded split."""
    import sparkucx_amd as sgx

    n = {"overflow": 1_500_000, "tiny": 7}.get(shape, 300_001)
    recs = oracle_lib.gen_uniform16(n, 0xAB + R)
    if shape == "zipf":
        ranks = np.arange(1, (1 << 16) + 1, dtype=np.float64)
        cdf = np.cumsum(ranks ** -1.1)
        recs = oracle_lib.gen_zipf16(n, 0xAB + R, cdf / cdf[-1])
    if shape == "overflow":
        # one partition dense in every line the sample skips (stride 2 at this size,
        # test_padded.py::test_padded_overflow_falls_back_bit_exact): its sub-bins overflow
        line = np.arange(n) // 8
        k = np.where(line % 2 == 1, 5, np.arange(n) % 1024).astype(np.int64)
        recs[:, :8] = k.view(np.uint8).reshape(-1, 8)
    out, counts = oracle_lib.map_write(recs, R, nthreads=8)
    want = oracle_lib.kryo_serialize(out)
    off = oracle_lib.kryo_partition_offsets(out, counts)
    with sgx_lib.ShuffleEngine(device=0, flags=sgx.FLAG_PAD_ANY_SIZE) as e:
        sid = _next_sid()
        e.register_shuffle(sid, R, serializer=sgx.SER_KRYO)
        if shape == "lz4":
            e.set_compression(sid, "lz4")
        lengths = e.write_map(sid, 0, np.ascontiguousarray(recs), n, 16, R)
        # the records went through the sub-bins unless sorted keys overflowed them
        if shape != "zipf":  # (skewed keys may or may not fit the sampled sub-bins)
            want_layout = sgx.LAYOUT_CONTIGUOUS if shape == "overflow" else sgx.LAYOUT_SERIALIZED_PADDED
            assert e.map_layout(sid, 0) == want_layout
        if shape == "lz4":
            framed, wl = oracle_lib.lz4_frame_partitions(want, off)
            assert np.array_equal(lengths, wl)
            assert np.array_equal(e.map_output_bytes(sid, 0), framed)
            o = oracle_lib.offsets(counts)
            assert e.read_records(sid, [0], 3, 40).tobytes() == out[o[3]:o[40]].tobytes()
        else:
            assert np.array_equal(lengths, np.diff(off))
            assert np.array_equal(e.map_output_bytes(sid, 0), want)
            rids = [R - 1, 0, R // 2, 1]
            data, lens = e.fetch_blocks(sid, [0] * len(rids), rids)
            pos = 0
            for r, L in zip(rids, lens):
                assert np.array_equal(data[pos:pos + L], want[off[r]:off[r + 1]])
                pos += L
            # the reduce side decodes the published stream: sorted and grouped reads
            seqs = oracle_lib.canonical_reducer_sequences([(out, counts)], R, 16)
            assert e.read_sorted(sid, [0], 0, R).tobytes() == oracle_lib.reduce_sorted(seqs).tobytes()
            ks, ss = e.read_grouped(sid, [0], 0, R, sgx.AGG_SUM)
            wk, wsum = oracle_lib.reduce_grouped(seqs, "sum")
            assert np.array_equal(ks, wk) and np.array_equal(ss, wsum)
