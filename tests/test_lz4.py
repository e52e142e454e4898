"""spark.shuffle.compress=true with the lz4 codec (compression half).

CPU: the oracle's restatement (oracle/lz4_oracle.c) is pinned against the system liblz4
(LZ4_compress_default / LZ4_decompress_safe, 1.9.x) and the `xxhash` module, and against the
golden fixtures tests/golden/lz4_*.npz (made by make_golden_lz4.py from liblz4 + xxhash, not
from the oracle).  GPU: sgx_lz4_frame_partitions (k_lz4_blocks / k_lz4_gather) must be byte
identical to the oracle and the fixtures: every frame header, checksum, payload and end mark.
"""
import ctypes
import glob
import os

import numpy as np
import pytest

from conftest import GOLDEN

FIXTURES = sorted(glob.glob(os.path.join(GOLDEN, "lz4_*.npz")))
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _liblz4():
    try:
        L = ctypes.CDLL("liblz4.so.1")
    except OSError:
        pytest.skip("system liblz4 not present")
    L.LZ4_compress_default.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_int]
    L.LZ4_decompress_safe.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_int]
    return L


def _cases(oracle):
    rng = np.random.default_rng(7)
    recs = oracle.gen_uniform16(20000, 0x5EEDC0DE)
    kry = oracle.kryo_serialize(recs).tobytes()
    out = [b"", b"a", b"abcabcabcabcabcabc", bytes(1000), kry[:32768], kry[5:30005],
           rng.integers(0, 256, 32768, dtype=np.uint8).tobytes(),
           rng.integers(0, 4, 30000, dtype=np.uint8).tobytes(), (b"xyz" * 20000)[:32768]]
    out += [rng.integers(0, 3, n, dtype=np.uint8).tobytes() for n in range(0, 40)]
    # shapes for the wave-parallel search (64 iterations per batch, lane-parallel counts,
    # catch-ups and literal runs): incompressible runs long enough to reach large skip
    # steps before a repeat, matches longer than 64 x 4 bytes, literal runs past 15 / 270,
    # periods around the wave width, and random splices of earlier bytes
    rnd = rng.integers(0, 256, 32768, dtype=np.uint8).tobytes()
    out += [rnd[:20000] + rnd[3000:6000] + rnd[20000:29000], bytes(32768), rnd[:300] + bytes(5000) + rnd[:300]]
    out += [(rnd[:p] * (32768 // p + 1))[:32768] for p in (7, 63, 64, 65, 255, 257, 1000)]
    out += [b"".join(rnd[i * 700:i * 700 + L] + bytes(40) for i, L in enumerate((14, 15, 16, 269, 270, 271, 600)))]
    spl, cur = bytearray(rnd[:64]), 64
    while len(spl) < 32768:
        spl += rnd[cur:cur + int(rng.integers(1, 100))]
        cur = (cur + 100) % 32000
        L, o = int(rng.integers(4, 300)), int(rng.integers(0, len(spl)))
        spl += bytes(spl[o:o + L])
    out += [bytes(spl[:32768]), bytes(spl[:32768])[::-1]]
    low = oracle.gen_uniform16(2048, 0x10E)
    low[:, :8] = (np.arange(2048, dtype=np.int64) % 97).view(np.uint8).reshape(-1, 8)
    out += [oracle.kryo_serialize(low).tobytes()[:32768]]
    return out


def parse_frames(buf: bytes):
    """-> list of (token, compressed_len, original_len, checksum, payload); stops at end mark."""
    frames, p = [], 0
    while p < len(buf):
        assert buf[p:p + 8] == b"LZ4Block"
        tok = buf[p + 8]
        cl, ol, ck = (int.from_bytes(buf[p + 9 + 4 * i:p + 13 + 4 * i], "little") for i in range(3))
        frames.append((tok, cl, ol, ck, buf[p + 21:p + 21 + cl]))
        p += 21 + cl
    return frames


def test_oracle_block_matches_liblz4(oracle_lib):
    L = _liblz4()
    for c in _cases(oracle_lib):
        out = ctypes.create_string_buffer(len(c) + len(c) // 255 + 64)
        n = L.LZ4_compress_default(c, out, len(c), len(out))
        assert oracle_lib.lz4_compress_block(c) == out.raw[:n], len(c)


def test_oracle_xxh32_matches_xxhash(oracle_lib):
    xxhash = pytest.importorskip("xxhash")
    for c in _cases(oracle_lib):
        for seed in (0, 0x9747B28C):
            assert oracle_lib.xxh32(c, seed) == xxhash.xxh32_intdigest(c, seed)
    # published known answer: XXH32 of the empty input, seed 0
    assert oracle_lib.xxh32(b"", 0) == 0x02CC5D05



@pytest.fixture(scope="module", params=["wave-decode", "lane-decode"])
def dec_engine(request, sgx_lib):
    """An engine per LZ4 decoder.  wave-decode (the default): compressed frames go through
    k_lz4_decode (one wave per frame) below 32768 frames, and RAW frames through
    k_lz4_raw_lanes (one lane per frame) from 2048 frames on (k_lz4_decode below that);
    lane-decode (SGX_FLAG_LZ4_LANE_DECODE): every compressed frame through k_lz4_decode_lanes."""
    flags = sgx_lib.FLAG_LZ4_LANE_DECODE if request.param == "lane-decode" else 0
    with sgx_lib.ShuffleEngine(device=0, flags=flags) as e:
        yield e

@pytest.mark.parametrize("path", FIXTURES, ids=os.path.basename)
def test_oracle_matches_golden(path, oracle_lib):
    g = np.load(path)
    framed, lens = oracle_lib.lz4_frame_partitions(g["stream"], g["offsets"], int(g["block_size"]))
    assert np.array_equal(lens, g["lengths"])
    assert framed.tobytes() == g["framed"].tobytes()


@pytest.mark.parametrize("path", FIXTURES, ids=os.path.basename)
def test_golden_frames_decode(path):
    """Frames round-trip: LZ4_decompress_safe of each payload (or the RAW bytes) with a valid
    masked XXH32, the partition streams restored byte for byte, one end mark per stream."""
    L = _liblz4()
    xxhash = pytest.importorskip("xxhash")
    g = np.load(path)
    stream, offs, framed, lens = g["stream"].tobytes(), g["offsets"], g["framed"].tobytes(), g["lengths"]
    pos = 0
    for r in range(len(lens)):
        part = framed[pos:pos + lens[r]]
        pos += lens[r]
        want = stream[offs[r]:offs[r + 1]]
        if not want:
            assert lens[r] == 0
            continue
        frames = parse_frames(part)
        assert frames[-1][1:4] == (0, 0, 0) and frames[-1][0] & 0xF0 == 0x10
        got = b""
        for tok, cl, ol, ck, pay in frames[:-1]:
            if tok & 0xF0 == 0x10:
                blk = pay
            else:
                out = ctypes.create_string_buffer(ol)
                assert L.LZ4_decompress_safe(pay, out, cl, ol) == ol
                blk = out.raw
            assert ck == xxhash.xxh32_intdigest(blk, 0x9747B28C) & 0x0FFFFFFF
            got += blk
        assert got == want


def test_unsafe_writer_fast_merge_restatement(oracle_lib):
    """oracle.unsafe_writer_map_output (UnsafeShuffleWriter, fast spill merge): decoding each
    partition with LZ4BlockInputStream's rules -- liblz4 per block, every XXH32 checked, an end
    mark followed by more bytes starts the next concatenated stream -- gives the partition's
    canonical Kryo stream; every spill segment holds one end mark; one spill equals the
    SortShuffleWriter framing (oracle.lz4_frame_partitions of the whole map)."""
    L = _liblz4()
    xxhash = pytest.importorskip("xxhash")
    R, block = 7, 4096
    sizes = [3000, 0, 1, 5000, 17]
    recs = oracle_lib.gen_uniform16(sum(sizes), 0x7700)
    spills = np.split(recs, np.cumsum(sizes)[:-1])
    data, lens = oracle_lib.unsafe_writer_map_output(spills, R, block_size=block)
    out, counts = oracle_lib.map_write(recs, R)
    kry = oracle_lib.kryo_serialize(out).tobytes()
    koff = oracle_lib.kryo_partition_offsets(out, counts)
    per_spill = [oracle_lib.map_write(sp, R)[1] for sp in spills]
    pos = 0
    for r in range(R):
        part = data[pos:pos + lens[r]].tobytes()
        pos += lens[r]
        got, nend, p = b"", 0, 0
        while p < len(part):  # LZ4BlockInputStream with concatenation (Spark 3.0.1's codec)
            tok = part[p + 8]
            cl, ol, ck = (int.from_bytes(part[p + 9 + 4 * i:p + 13 + 4 * i], "little") for i in range(3))
            pay = part[p + 21:p + 21 + cl]
            p += 21 + cl
            if ol == 0:
                nend += 1
                continue
            if tok & 0xF0 == 0x10:
                blk = pay
            else:
                buf = ctypes.create_string_buffer(ol)
                assert L.LZ4_decompress_safe(pay, buf, cl, ol) == ol
                blk = buf.raw
            assert ck == xxhash.xxh32_intdigest(blk, 0x9747B28C) & 0x0FFFFFFF
            got += blk
        assert got == kry[koff[r]:koff[r + 1]]
        assert nend == sum(1 for c in per_spill if c[r] > 0)
    one, one_len = oracle_lib.unsafe_writer_map_output([recs], R, block_size=block)
    canon, canon_len = oracle_lib.lz4_frame_partitions(np.frombuffer(kry, np.uint8), koff, block)
    assert np.array_equal(one_len, canon_len) and np.array_equal(one, canon)


# ------------------------------------------------------------------------ GPU ------
def _to_device(engine, data: bytes):
    buf = engine.alloc(max(len(data), 1))
    if data:
        buf.copy_from(np.frombuffer(data, np.uint8))
    return buf


@pytest.mark.gpu
@pytest.mark.parametrize("path", FIXTURES, ids=os.path.basename)
def test_gpu_matches_golden(path, engine):
    g = np.load(path)
    buf = _to_device(engine, g["stream"].tobytes())
    try:
        framed, lens = engine.lz4_frame(buf.ptr, g["offsets"], int(g["block_size"]))
    finally:
        buf.free()
    assert np.array_equal(lens, g["lengths"])
    assert framed.tobytes() == g["framed"].tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("block_size", [32768, 4096, 64])
def test_gpu_matches_oracle_mixed_partitions(engine, oracle_lib, block_size):
    cases = _cases(oracle_lib)
    stream = b"".join(cases)
    offs = np.zeros(len(cases) + 1, dtype=np.int64)
    np.cumsum([len(c) for c in cases], out=offs[1:])
    buf = _to_device(engine, stream)
    try:
        framed, lens = engine.lz4_frame(buf.ptr, offs, block_size)
    finally:
        buf.free()
    want, wlens = oracle_lib.lz4_frame_partitions(np.frombuffer(stream, np.uint8), offs, block_size)
    assert np.array_equal(lens, wlens)
    assert framed.tobytes() == want.tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("block_size", [4096, 64])
def test_gpu_tiny_blocks_at_every_byte_phase(dec_engine, oracle_lib, block_size):
    """Partitions whose tail block (and whole partitions) of 1..5 bytes start at every byte
    phase of a dword: a block of n < 4 - phase bytes is staged from g[-phase..n) (the
    regression of round 2's multi-rank LZ4 fault, a 1-byte tail at an odd offset)."""
    rng = np.random.default_rng(17)
    plen = []
    for phase in range(4):
        for tail in range(1, 6):
            pad = (phase - sum(plen)) % 4  # next partition starts at `phase` mod 4
            plen += [pad + 4, block_size + tail, tail]
    stream = rng.integers(0, 256, size=sum(plen), dtype=np.uint8)
    offs = np.zeros(len(plen) + 1, dtype=np.int64)
    np.cumsum(plen, out=offs[1:])
    buf = _to_device(dec_engine, stream.tobytes())
    try:
        framed, lens = dec_engine.lz4_frame(buf.ptr, offs, block_size)
    finally:
        buf.free()
    want, wlens = oracle_lib.lz4_frame_partitions(stream, offs, block_size)
    assert np.array_equal(lens, wlens)
    assert framed.tobytes() == want.tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("R", [1, 200])
def test_gpu_kryo_map_output_compressed(engine, oracle_lib, R):
    """A Kryo (Long, Long) map output written by the engine, then LZ4-framed on the GPU: the
    bytes Spark commits to the data file with spark.shuffle.compress=true."""
    sid = 900 + R
    n = 300_000
    recs = oracle_lib.gen_uniform16(n, 0x5EEDC0DE)
    # low-entropy keys as well, so blocks compress (values = record index)
    recs[n // 2:, :8] = (np.arange(n - n // 2, dtype=np.int64) % 777).view(np.uint8).reshape(-1, 8)
    engine.register_shuffle(sid, R)
    try:
        engine.set_serializer(sid, 1)
        engine.write_map(sid, 0, recs, n, 16, num_partitions=R)
        framed, lens = engine.lz4_frame_map(sid, 0, R)
        out, counts = oracle_lib.map_write(recs, R)
        kry = oracle_lib.kryo_serialize(out)
        koffs = oracle_lib.kryo_partition_offsets(out, counts)
        want, wlens = oracle_lib.lz4_frame_partitions(kry, koffs)
        assert np.array_equal(lens, wlens)
        assert framed.tobytes() == want.tobytes()
        assert int(wlens.sum()) < int(koffs[-1])  # the low-entropy half compresses
    finally:
        engine.unregister_shuffle(sid)


@pytest.mark.gpu
def test_gpu_rejects_bad_block_size(engine, sgx_lib):
    buf = _to_device(engine, b"x" * 100)
    try:
        with pytest.raises(sgx_lib._lib.UnsupportedOperationException):
            engine.lz4_frame(buf.ptr, np.array([0, 100], np.int64), 65536)
    finally:
        buf.free()


# ------------------------------------------------------------- GPU decode (reduce side) --
@pytest.mark.gpu
@pytest.mark.parametrize("path", FIXTURES, ids=os.path.basename)
def test_gpu_unframe_golden(path, dec_engine):
    """LZ4BlockInputStream on the GPU over all partitions' frames back to back = the stream."""
    g = np.load(path)
    got = dec_engine.lz4_unframe(g["framed"])
    assert got.tobytes() == g["stream"].tobytes()


@pytest.mark.gpu
def test_gpu_frame_unframe_round_trip(dec_engine, oracle_lib):
    cases = _cases(oracle_lib)
    stream = b"".join(cases)
    offs = np.zeros(len(cases) + 1, dtype=np.int64)
    np.cumsum([len(c) for c in cases], out=offs[1:])
    buf = _to_device(dec_engine, stream)
    try:
        framed, lens = dec_engine.lz4_frame(buf.ptr, offs, 4096)
    finally:
        buf.free()
    assert dec_engine.lz4_unframe(framed).tobytes() == stream
    # any subset of partitions (fetched blocks in any order) decodes to those streams
    fo = np.zeros(len(lens) + 1, dtype=np.int64)
    np.cumsum(lens, out=fo[1:])
    pick = [7, 3, 5, 0, 8]
    sub = b"".join(framed[fo[r]:fo[r + 1]].tobytes() for r in pick)
    assert dec_engine.lz4_unframe(sub).tobytes() == b"".join(cases[r] for r in pick)


@pytest.mark.gpu
def test_gpu_unframe_rejects_corrupt(dec_engine, sgx_lib):
    g = np.load(FIXTURES[0])
    framed = bytearray(g["framed"].tobytes())
    bad_magic = bytes(framed)
    bad_magic = b"X" + bad_magic[1:]
    with pytest.raises(sgx_lib._lib.IllegalArgumentException):
        dec_engine.lz4_unframe(bad_magic)
    flipped = bytearray(framed)
    flipped[30] ^= 0x5A  # inside the first payload
    with pytest.raises(sgx_lib._lib.IllegalArgumentException):
        dec_engine.lz4_unframe(bytes(flipped))
    with pytest.raises(sgx_lib._lib.IllegalArgumentException):
        dec_engine.lz4_unframe(bytes(framed[:-5]))  # truncated end mark


@pytest.mark.gpu
def test_gpu_unframe_dense_frames(dec_engine, oracle_lib):
    """5000 tiny partition streams: more frames than the first walk's table holds (re-walk)."""
    rng = np.random.default_rng(3)
    parts = [rng.integers(0, 256, int(rng.integers(1, 9)), dtype=np.uint8).tobytes() for _ in range(5000)]
    stream = b"".join(parts)
    offs = np.zeros(len(parts) + 1, dtype=np.int64)
    np.cumsum([len(p) for p in parts], out=offs[1:])
    want, _ = oracle_lib.lz4_frame_partitions(np.frombuffer(stream, np.uint8), offs)
    assert dec_engine.lz4_unframe(want).tobytes() == stream


@pytest.mark.gpu
def test_gpu_unframe_mixed_raw_and_compressed_many_frames(dec_engine, oracle_lib):
    """>= 2048 frames mixing RAW frames (incompressible blocks) and LZ4 ones (repetitive
    blocks) in one buffer: in the default engine the RAW ones take k_lz4_raw_lanes while the
    compressed ones take k_lz4_decode with the RAW frames skipped -- both kernels write the
    same output buffer; the result must equal the stream, also through the per-stream walks."""
    rng = np.random.default_rng(21)
    parts = []
    for i in range(900):  # ~2.7 frames of 1 KiB blocks per stream -> ~2400 frames
        blocks = []
        for k in range(int(rng.integers(2, 5))):
            if (i + k) % 3 == 0:  # incompressible: a RAW frame
                blocks.append(rng.integers(0, 256, 1024, dtype=np.uint8).tobytes())
            else:  # periodic: an LZ4 frame
                pat = rng.integers(0, 256, int(rng.integers(1, 40)), dtype=np.uint8).tobytes()
                blocks.append((pat * (1024 // len(pat) + 1))[:1024])
        parts.append(b"".join(blocks)[: int(rng.integers(1500, 4097))])
    stream = b"".join(parts)
    offs = np.zeros(len(parts) + 1, dtype=np.int64)
    np.cumsum([len(p) for p in parts], out=offs[1:])
    framed, lens = oracle_lib.lz4_frame_partitions(np.frombuffer(stream, np.uint8), offs, 1024)
    frames = [f for r in range(len(lens)) for f in parse_frames(
        framed.tobytes()[int(lens[:r].sum()):int(lens[:r + 1].sum())])[:-1]]
    methods = {f[0] & 0xF0 for f in frames}
    assert len(frames) >= 2048 and methods == {0x10, 0x20}, (len(frames), methods)
    assert dec_engine.lz4_unframe(framed).tobytes() == stream
    assert dec_engine.lz4_unframe(framed, stream_lens=lens).tobytes() == stream


def _overlap_cases():
    """Streams whose LZ4 blocks are full of self-overlapping matches (offsets 1..130, the
    lane-parallel copy's i mod off path and its off >= 64 path), matches around and past the
    lane decoder's 256 B history ring (periods 248..520), long match-length runs, long
    literal runs, and mixtures -- each its own partition stream."""
    rng = np.random.default_rng(11)
    out = [bytes(40000), b"\x07" * 33000]
    for period in (2, 3, 5, 7, 16, 31, 63, 64, 65, 100, 130, 248, 255, 256, 257, 263, 300, 520):
        pat = rng.integers(0, 256, period, dtype=np.uint8).tobytes()
        out.append((pat * (70000 // period + 1))[:70000])
    mixed = bytearray()
    while len(mixed) < 100000:
        k = int(rng.integers(0, 4))
        if k == 0:
            mixed += rng.integers(0, 256, int(rng.integers(1, 300)), dtype=np.uint8).tobytes()
        elif k == 1:
            mixed += bytes([int(rng.integers(0, 256))]) * int(rng.integers(1, 2000))
        elif k == 2 and len(mixed) > 70:
            s = int(rng.integers(max(0, len(mixed) - 600), len(mixed) - 64))
            mixed += mixed[s:s + int(rng.integers(4, 64))]
        else:
            mixed += (rng.integers(0, 256, 3, dtype=np.uint8).tobytes() * 50)
    out.append(bytes(mixed))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("per_stream", [False, True], ids=["one-walk", "per-stream-walk"])
def test_gpu_unframe_overlapping_matches(dec_engine, oracle_lib, per_stream):
    """The in-place, lane-parallel decoder against the streams themselves (frames from the
    oracle, whose compressor is pinned to liblz4), through the single walk and the per-stream
    walks of sgx_lz4_unframe_streams."""
    parts = _overlap_cases()
    stream = b"".join(parts)
    offs = np.zeros(len(parts) + 1, dtype=np.int64)
    np.cumsum([len(p) for p in parts], out=offs[1:])
    for bs in (32768, 4096, 64):
        framed, flens = oracle_lib.lz4_frame_partitions(np.frombuffer(stream, np.uint8), offs, bs)
        if bs >= 4096:
            assert len(framed) < len(stream)  # the blocks really are compressed
        got = dec_engine.lz4_unframe(framed, flens if per_stream else None)
        assert got.tobytes() == stream, bs


@pytest.mark.gpu
def test_gpu_unframe_streams_errors(dec_engine, oracle_lib, sgx_lib):
    parts = _overlap_cases()[:4]
    stream = b"".join(parts)
    offs = np.zeros(len(parts) + 1, dtype=np.int64)
    np.cumsum([len(p) for p in parts], out=offs[1:])
    framed, flens = oracle_lib.lz4_frame_partitions(np.frombuffer(stream, np.uint8), offs, 32768)
    fb = bytearray(framed.tobytes())
    # the stream lengths must cover the buffer
    with pytest.raises(sgx_lib._lib.IllegalArgumentException):
        dec_engine.lz4_unframe(bytes(fb), np.concatenate([flens[:-1], [flens[-1] - 1]]))
    # a bad magic in the third stream is reported at its byte position
    pos = int(flens[:2].sum())
    bad = bytearray(fb)
    bad[pos] = ord("X")
    with pytest.raises(sgx_lib._lib.IllegalArgumentException, match=f"bad magic at byte {pos}"):
        dec_engine.lz4_unframe(bytes(bad), flens)
    # a flipped payload byte fails the block (corrupt sequence or checksum)
    bad = bytearray(fb)
    bad[pos + 40] ^= 0x5A
    with pytest.raises(sgx_lib._lib.IllegalArgumentException):
        dec_engine.lz4_unframe(bytes(bad), flens)
    # a block cut short inside the second stream
    with pytest.raises(sgx_lib._lib.IllegalArgumentException):
        dec_engine.lz4_unframe(bytes(fb), np.concatenate([[flens[0] + flens[1] - 5, 5], flens[2:]]))
    assert dec_engine.lz4_unframe(bytes(fb), flens).tobytes() == stream


# ------------------------------------------------- shuffle-level compression (engine) --
@pytest.mark.gpu
def test_gpu_compressed_shuffle_publishes_lz4_frames(dec_engine, oracle_lib, sgx_lib, tmp_path):
    """sgx_set_compression(LZ4) on a Kryo shuffle: lengths, map bytes, fetched blocks and the
    committed index/data files are the LZ4BlockOutputStream bytes Spark writes with
    spark.shuffle.compress=true."""
    sid, R, n = 950, 64, 200_000
    recs = oracle_lib.gen_uniform16(n, 0x5EEDC0DE)
    recs[::2, :8] = (np.arange(0, n, 2, dtype=np.int64) % 999).view(np.uint8).reshape(-1, 8)
    dec_engine.register_shuffle(sid, R)
    try:
        dec_engine.set_serializer(sid, 1)
        dec_engine.set_compression(sid, "lz4")
        lens = dec_engine.write_map(sid, 0, recs, n, 16, num_partitions=R)
        out, counts = oracle_lib.map_write(recs, R)
        want, wlens = oracle_lib.lz4_frame_partitions(oracle_lib.kryo_serialize(out),
                                                      oracle_lib.kryo_partition_offsets(out, counts))
        assert np.array_equal(lens, wlens)
        assert dec_engine.map_output_bytes(sid, 0).tobytes() == want.tobytes()
        fo = oracle_lib.offsets(wlens)
        pick = [5, 0, 63, 17]
        got, glens = dec_engine.fetch_blocks(sid, [0] * len(pick), pick)
        assert got.tobytes() == b"".join(want[fo[r]:fo[r + 1]].tobytes() for r in pick)
        # the reduce side decodes what it fetched: LZ4 -> Kryo stream of those partitions
        kry = oracle_lib.kryo_serialize(out)
        ko = oracle_lib.kryo_partition_offsets(out, counts)
        assert dec_engine.lz4_unframe(got).tobytes() == b"".join(kry[ko[r]:ko[r + 1]].tobytes() for r in pick)
        idx, dat = str(tmp_path / "s.index"), str(tmp_path / "s.data")
        committed = dec_engine.write_index(sid, 0, idx, dat, R)
        assert np.array_equal(committed, wlens)
        assert open(dat, "rb").read() == want.tobytes()
        assert open(idx, "rb").read() == oracle_lib.index_bytes(wlens)
        # reduce side: fetch -> LZ4 decompress -> Kryo decode, all on the GPU
        recs_read = dec_engine.read_records(sid, [0], 3, 40)
        o = oracle_lib.offsets(counts)
        assert recs_read.tobytes() == out[o[3]:o[40]].tobytes()
        ks, ss = dec_engine.read_grouped(sid, [0], 0, R, sgx_lib._lib.AGG_SUM)
        wk, wsum = oracle_lib.reduce_grouped(oracle_lib.canonical_reducer_sequences([(out, counts)], R, 16), "sum")
        assert np.array_equal(ks, wk) and np.array_equal(ss, wsum)
        with pytest.raises(sgx_lib._lib.IllegalStateException):
            dec_engine.set_compression(sid, "none")
    finally:
        dec_engine.unregister_shuffle(sid)


@pytest.mark.gpu
def test_gpu_compression_needs_kryo(engine, sgx_lib):
    engine.register_shuffle(951, 8)
    try:
        with pytest.raises(sgx_lib._lib.UnsupportedOperationException):
            engine.set_compression(951, "lz4")
        with pytest.raises(sgx_lib._lib.IllegalArgumentException):
            engine.set_compression(951, "snappy")
    finally:
        engine.unregister_shuffle(951)


@pytest.mark.gpu
def test_gpu_plugin_spark_shuffle_compress(sgx_lib, oracle_lib, tmp_path):
    """UcxShuffleManager with spark.shuffle.compress=true and the Kryo serializer: the writer's
    lengths and the committed data file are LZ4 frames; readSerialized() returns the Kryo
    stream of the partition range and read() its records (GPU decompression + decode)."""
    R, n = 128, 120_000
    mgr = sgx_lib.UcxShuffleManager(conf={"spark.shuffle.compress": "true",
                                          "spark.io.compression.lz4.blockSize": "16k"}, localDir=str(tmp_path))
    try:
        h = mgr.registerShuffle(7, sgx_lib.ShuffleDependency(sgx_lib.HashPartitioner(R), serializer="kryo"))
        recs = oracle_lib.gen_uniform16(n, 4242)
        recs[::3, :8] = (np.arange(0, n, 3, dtype=np.int64) % 321).view(np.uint8).reshape(-1, 8)
        w = mgr.getWriter(h, 0)
        w.write(recs)
        out, counts = oracle_lib.map_write(recs, R)
        kry = oracle_lib.kryo_serialize(out)
        ko = oracle_lib.kryo_partition_offsets(out, counts)
        want, wlens = oracle_lib.lz4_frame_partitions(kry, ko, 16 * 1024)
        assert np.array_equal(w.getPartitionLengths(), wlens)
        lengths = w.getPartitionLengths().copy()
        mgr.shuffleBlockResolver.writeIndexFileAndCommit(7, 0, lengths)
        assert open(mgr.shuffleBlockResolver.getDataFile(7, 0), "rb").read() == want.tobytes()
        rd = mgr.getReader(h, 10, 20)
        assert rd.readSerialized().tobytes() == kry[ko[10]:ko[20]].tobytes()
        o = oracle_lib.offsets(counts)
        assert rd.read().tobytes() == out[o[10]:o[20]].tobytes()
    finally:
        mgr.stop()


@pytest.mark.gpu
@pytest.mark.parametrize("R,fast,handle", [(1024, "true", "SerializedShuffleHandle"),
                                           (1024, "false", "SerializedShuffleHandle"),
                                           (200, "true", "BypassMergeSortShuffleHandle")])
def test_gpu_plugin_handle_selection_and_spills(sgx_lib, oracle_lib, tmp_path, R, fast, handle):
    """registerShuffle picks Spark's handle (SortShuffleManager.registerShuffle) and the writer
    the reference's getWriter runs for it (spark_3_0/UcxShuffleManager.scala:32-53); a map task
    written in spills publishes UnsafeShuffleWriter's fast-merge framing for a
    SerializedShuffleHandle and SortShuffleWriter's single stream per partition otherwise (slow
    merge, bypass handle); the data file and read() agree with the restatement."""
    mgr = sgx_lib.UcxShuffleManager(conf={"spark.shuffle.unsafe.fastMergeEnabled": fast}, localDir=str(tmp_path))
    try:
        h = mgr.registerShuffle(9, sgx_lib.ShuffleDependency(sgx_lib.HashPartitioner(R), serializer="kryo"))
        assert type(h).__name__ == handle
        assert h.writerClass == ("UnsafeShuffleWriter" if handle == "SerializedShuffleHandle" else "SortShuffleWriter")
        recs = oracle_lib.gen_uniform16(120_000, 0x9090)
        spills = [recs[:50_000], recs[50_000:50_001], recs[50_001:]]
        w = mgr.getWriter(h, 0)
        w.write(spills)
        if handle == "SerializedShuffleHandle" and fast == "true":
            want, wlens = oracle_lib.unsafe_writer_map_output(spills, R)
        else:
            out, counts = oracle_lib.map_write(recs, R)
            want, wlens = oracle_lib.lz4_frame_partitions(oracle_lib.kryo_serialize(out),
                                                          oracle_lib.kryo_partition_offsets(out, counts))
        assert np.array_equal(w.getPartitionLengths(), wlens)
        mgr.shuffleBlockResolver.writeIndexFileAndCommit(9, 0, w.getPartitionLengths().copy())
        assert open(mgr.shuffleBlockResolver.getDataFile(9, 0), "rb").read() == want.tobytes()
        out, counts = oracle_lib.map_write(recs, R)
        o = oracle_lib.offsets(counts)
        assert mgr.getReader(h, 3, R - 5).read().tobytes() == out[o[3]:o[R - 5]].tobytes()
        # map-side combine: never a SerializedShuffleHandle
        hc = mgr.registerShuffle(10, sgx_lib.ShuffleDependency(sgx_lib.HashPartitioner(R), serializer="kryo",
                                                               aggregator=sgx_lib.Aggregator("sum"),
                                                               mapSideCombine=True))
        assert type(hc).__name__ == "BaseShuffleHandle" and hc.writerClass == "SortShuffleWriter"
    finally:
        mgr.stop()


@pytest.mark.gpu
def test_gpu_rewrite_compressed_map_with_other_data(sgx_lib, oracle_lib):
    """A second attempt of the same map on an LZ4 shuffle (smaller, then larger than the
    first) publishes the frames of ITS Kryo stream -- never the earlier attempt's frames."""
    R = 64
    with sgx_lib.ShuffleEngine(device=0) as e:
        e.register_shuffle(1, R, serializer=sgx_lib.SER_KRYO)
        e.set_compression(1, "lz4", 4096)
        for k, n in enumerate((40_000, 7_000, 90_000)):
            recs = oracle_lib.gen_uniform16(n, 0x1234 + k)
            if k == 2:
                recs[:, 8:] = 0  # compressible values: LZ4 blocks, not RAW
            lens = e.write_map(1, 0, recs, n, 16, R)
            out, counts = oracle_lib.map_write(recs, R)
            kryo = oracle_lib.kryo_serialize(out)
            frames, flen = oracle_lib.lz4_frame_partitions(kryo, oracle_lib.kryo_partition_offsets(out, counts), 4096)
            assert np.array_equal(lens, flen), f"attempt {k}"
            assert np.array_equal(e.map_output_bytes(1, 0), frames), f"attempt {k}"
            got = e.read_records(1, [0], 0, R).reshape(-1, 16)
            assert np.array_equal(got, out), f"attempt {k}"


@pytest.mark.gpu
def test_gpu_serializer_cannot_leave_kryo_while_compressed(sgx_lib):
    with sgx_lib.ShuffleEngine(device=0) as e:
        e.register_shuffle(1, 8, serializer=sgx_lib.SER_KRYO)
        e.set_compression(1, "lz4", 32768)
        with pytest.raises(sgx_lib.IllegalStateException):
            e.set_serializer(1, sgx_lib.SER_FIXED)
        e.set_compression(1, "none")
        e.set_serializer(1, sgx_lib.SER_FIXED)  # allowed once compression is off


def _batch_shapes(oracle_lib, size):
    """Block shapes for the multi-sequence batch compressor (sgx_lz4.hip lz4_compress_batch):
    C1's Kryo stream (short matches every ~16 bytes: several sequences per 64-position batch),
    a low-entropy stream (matches that end inside the batch and hit again at `_next_match`),
    byte runs over three symbols (long matches past the batch, catch-ups), a period of 10,
    uniform bytes (no matches: the search's later, wider steps) and a stream of 8-byte
    repeats at batch-straddling offsets."""
    rng = np.random.default_rng(23)
    recs = oracle_lib.gen_uniform16(size // 8, 7, value_base=3 << 32)
    kryo = oracle_lib.kryo_serialize(recs).tobytes()
    low = b"".join(int(i % 4096).to_bytes(8, "little") + int(i).to_bytes(8, "little") for i in range(size // 16))
    rep = b"".join(bytes(rng.integers(0, 256, 8, dtype=np.uint8)) * int(rng.integers(1, 4)) + bytes(rng.integers(0, 256, int(rng.integers(1, 70)), dtype=np.uint8))
                   for _ in range(size // 40))
    return [kryo[:size], low[:size], bytes(rng.integers(0, 3, size, dtype=np.uint8)), (b"abcdefghij" * (size // 10 + 1))[:size],
            bytes(rng.integers(0, 256, size, dtype=np.uint8)), rep[:size]]


def test_batch_model_matches_oracle(oracle_lib):
    """The host model of the batch compressor's table state (tools/lz4_batch_model.py) against
    the oracle, on 4 KiB blocks of every shape (the GPU test below runs the kernel)."""
    import importlib.util

    spec = importlib.util.spec_from_file_location("lz4_batch_model", os.path.join(ROOT, "tools", "lz4_batch_model.py"))
    model = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(model)
    for blk in _batch_shapes(oracle_lib, 4096):
        assert model.compress(blk) == oracle_lib.lz4_compress_block(blk)


@pytest.mark.gpu
def test_gpu_batch_compressor_shapes(engine, oracle_lib):
    """Every batch-compressor shape as 32 KiB blocks (and ragged tails) through the GPU
    framing, byte-identical to the oracle."""
    cases = [c[:n] for c in _batch_shapes(oracle_lib, 65536) for n in (65536, 40001)]
    stream = b"".join(cases)
    offs = np.zeros(len(cases) + 1, dtype=np.int64)
    np.cumsum([len(c) for c in cases], out=offs[1:])
    buf = _to_device(engine, stream)
    try:
        framed, lens = engine.lz4_frame(buf.ptr, offs, 32768)
    finally:
        buf.free()
    want, wlens = oracle_lib.lz4_frame_partitions(np.frombuffer(stream, np.uint8), offs, 32768)
    assert np.array_equal(lens, wlens)
    assert framed.tobytes() == want.tobytes()
