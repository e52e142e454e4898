"""CPU oracle for the sparkucx_amd shuffle hot path.

TEST INFRASTRUCTURE ONLY: ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this package, and only as the checker (or, for the
baseline, as the timed CPU restatement).  The product package ``sparkucx_amd`` never
imports it and has no CPU fallback.

Two independent restatements of Spark 3.0.1's map-side shuffle semantics live here:
``spark_semantics.py`` (pure Python, small cases, fixture generation) and
``shuffle_oracle.c`` (C99, wrapped below via ctypes; fast and multi-threaded).
Parity is pinned by SURVEY.md §8(c)'s known-answer tests (the reference has no tests of
its own).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None

PART_HASH, PART_RANGE_I64, PART_RANGE_BYTES10 = 0, 1, 2


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        i32, i64, u64, vp = ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64, ctypes.c_void_p
        L.orc_java_long_hash.argtypes = [i64]
        L.orc_java_long_hash.restype = i32
        L.orc_non_negative_mod.argtypes = [i32, i32]
        L.orc_non_negative_mod.restype = i32
        L.orc_hash_partition.argtypes = [i64, i32]
        L.orc_hash_partition.restype = i32
        L.orc_range_partition_i64.argtypes = [i64, vp, i32, i32]
        L.orc_range_partition_i64.restype = i32
        L.orc_range_partition_bytes.argtypes = [vp, i32, vp, i32, i32]
        L.orc_range_partition_bytes.restype = i32
        L.orc_partition_ids.argtypes = [vp, i64, i32, i32, i32, vp, i32, i32, vp]
        L.orc_partition_ids.restype = None
        L.orc_stable_scatter.argtypes = [vp, i64, i32, vp, i32, vp, vp]
        L.orc_stable_scatter.restype = None
        L.orc_map_write.argtypes = [vp, i64, i32, i32, i32, vp, i32, i32, vp, vp, i32]
        L.orc_map_write.restype = ctypes.c_int
        L.orc_index_bytes.argtypes = [vp, i32, vp]
        L.orc_index_bytes.restype = None
        L.orc_check_index.argtypes = [vp, i64, i64, i32, vp]
        L.orc_check_index.restype = ctypes.c_int
        L.orc_splitmix64_at.argtypes = [u64, u64]
        L.orc_splitmix64_at.restype = u64
        L.orc_gen_uniform16.argtypes = [vp, i64, u64, i64]
        L.orc_gen_uniform16.restype = None
        L.orc_gen_terasort100.argtypes = [vp, i64, u64, i64]
        L.orc_gen_terasort100.restype = None
        L.orc_zipf_cdf.argtypes = [ctypes.c_double, i64, vp]
        L.orc_zipf_cdf.restype = None
        L.orc_gen_zipf16.argtypes = [vp, i64, u64, i64, vp, i64]
        L.orc_gen_zipf16.restype = None
        L.orc_lz4_compress_block.argtypes = [vp, ctypes.c_int, vp]
        L.orc_lz4_compress_block.restype = ctypes.c_int
        L.orc_xxh32.argtypes = [vp, i64, ctypes.c_uint32]
        L.orc_xxh32.restype = ctypes.c_uint32
        L.orc_lz4_frame_partitions.argtypes = [vp, vp, i32, ctypes.c_int, vp, vp]
        L.orc_lz4_frame_partitions.restype = i64
        _lib = L
    return _lib


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


# ---------------------------------------------------------------- generators ------
def gen_uniform16(n: int, seed: int, value_base: int = 0) -> np.ndarray:
    """n uniform 16-byte records as a (n, 16) uint8 array."""
    out = np.empty((n, 16), dtype=np.uint8)
    lib().orc_gen_uniform16(_ptr(out), n, seed & (2**64 - 1), value_base)
    return out


def gen_terasort100(n: int, seed: int, index_base: int = 0) -> np.ndarray:
    out = np.empty((n, 100), dtype=np.uint8)
    lib().orc_gen_terasort100(_ptr(out), n, seed & (2**64 - 1), index_base)
    return out


def zipf_cdf(s: float, K: int) -> np.ndarray:
    cdf = np.empty(K, dtype=np.float64)
    lib().orc_zipf_cdf(s, K, _ptr(cdf))
    return cdf


def gen_zipf16(n: int, seed: int, cdf: np.ndarray, value_base: int = 0) -> np.ndarray:
    out = np.empty((n, 16), dtype=np.uint8)
    lib().orc_gen_zipf16(_ptr(out), n, seed & (2**64 - 1), value_base, _ptr(cdf), len(cdf))
    return out


# ---------------------------------------------------------------- semantics -------
def _bounds_arg(kind: int, bounds):
    if bounds is None or kind == PART_HASH:
        return None, 0
    if kind == PART_RANGE_I64:
        b = np.ascontiguousarray(bounds, dtype=np.int64)
        return b, len(b)
    b = np.ascontiguousarray(bounds, dtype=np.uint8).reshape(-1, 10)
    return b, b.shape[0]


def partition_ids(records: np.ndarray, num_partitions: int, kind: int = PART_HASH,
                  bounds=None, ascending: bool = True) -> np.ndarray:
    records = np.ascontiguousarray(records)
    n, rb = records.shape
    b, nb = _bounds_arg(kind, bounds)
    pids = np.empty(n, dtype=np.int32)
    lib().orc_partition_ids(_ptr(records), n, rb, kind, num_partitions,
                            None if b is None else _ptr(b), nb, int(ascending), _ptr(pids))
    return pids


def map_write(records: np.ndarray, num_partitions: int, kind: int = PART_HASH, bounds=None,
              ascending: bool = True, nthreads: int = 1):
    """Map-side write: returns (partition-contiguous records, counts per partition)."""
    records = np.ascontiguousarray(records)
    n, rb = records.shape
    b, nb = _bounds_arg(kind, bounds)
    out = np.empty_like(records)
    counts = np.empty(num_partitions, dtype=np.int64)
    rc = lib().orc_map_write(_ptr(records), n, rb, kind, num_partitions,
                             None if b is None else _ptr(b), nb, int(ascending), _ptr(out),
                             _ptr(counts), nthreads)
    if rc != 0:
        raise MemoryError("orc_map_write failed")
    return out, counts


def index_bytes(lengths: np.ndarray) -> bytes:
    lengths = np.ascontiguousarray(lengths, dtype=np.int64)
    out = np.empty(8 * (len(lengths) + 1), dtype=np.uint8)
    lib().orc_index_bytes(_ptr(lengths), len(lengths), _ptr(out))
    return out.tobytes()


def offsets(counts: np.ndarray) -> np.ndarray:
    o = np.zeros(len(counts) + 1, dtype=np.int64)
    np.cumsum(counts, out=o[1:])
    return o


def canonical_reducer_sequences(map_outputs, num_partitions: int, record_bytes: int):
    """Per-reducer canonical sequences: for each reducer r, the concatenation over maps in
    ascending map order of that map's block r (SURVEY.md §8(a) parity note).
    ``map_outputs``: list of (data (n, rb) uint8, counts[R])."""
    seqs = []
    offs = [offsets(c) for _, c in map_outputs]
    for r in range(num_partitions):
        parts = [d[o[r]:o[r + 1]] for (d, _), o in zip(map_outputs, offs)]
        seqs.append(np.concatenate(parts) if parts else np.empty((0, record_bytes), np.uint8))
    return seqs


# ---------------------------------------------------------------- reduce side -----
# UcxShuffleReader.read after the fetch (spark_3_0/UcxShuffleReader.scala:137-191), on the
# canonical per-reducer sequences above.  Spark 3.0.1 semantics restated (spark-core, not
# vendored in the reference):
#  * keyOrdering: ExternalSorter(ordering = keyOrd).insertAll -> sorted iterator; the sort
#    is TimSort (java.util / Spark's Sorter), i.e. STABLE: equal keys keep arrival order.
#    Long keys compare signed; TeraSort's 10-byte keys compare unsigned lexicographically.
#  * aggregator, mapSideCombine = false: Aggregator.combineValuesByKey ->
#    ExternalAppendOnlyMap; groupByKey's combiner is a CompactBuffer appended in arrival
#    order; reduceByKey(_ + _) on Longs adds with two's-complement wrap-around.  Spark's
#    output order of groups is hash-map order (unspecified); the canonical form compared
#    here is ascending key order within each reducer.
def sort_key_order(records: np.ndarray) -> np.ndarray:
    """Stable permutation sorting fixed-width records by key (16 B: signed LE int64 at 0;
    100 B: 10-byte unsigned big-endian key at 0)."""
    records = np.ascontiguousarray(records)
    n, rb = records.shape
    if rb == 16:
        keys = records[:, :8].copy().view("<i8").reshape(n)
        return np.argsort(keys, kind="stable")
    if rb == 100:
        # lexsort: last key is primary; byte 0 most significant
        return np.lexsort(tuple(records[:, i] for i in range(9, -1, -1)))
    raise ValueError(f"record width {rb}")


def reduce_sorted(seqs) -> np.ndarray:
    """keyOrdering read: each reducer's canonical sequence sorted stably by key, reducer-major."""
    parts = [s[sort_key_order(s)] for s in seqs if len(s)]
    if not parts:
        w = seqs[0].shape[1] if seqs else 16
        return np.empty((0, w), dtype=np.uint8)
    return np.concatenate(parts)


def reduce_grouped(seqs, agg: str = "group"):
    """groupByKey ('group') -> (keys, group_starts, values); reduceByKey sum ('sum') ->
    (keys, sums).  Keys ascending per reducer, reducer-major; values in arrival order."""
    keys_l, starts_l, vals_l, sums_l = [], [], [], []
    base = 0
    for s in seqs:
        if not len(s):
            continue
        srt = s[sort_key_order(s)]
        k = srt[:, :8].copy().view("<i8").reshape(-1)
        v = srt[:, 8:16].copy().view("<i8").reshape(-1)
        first = np.ones(len(k), dtype=bool)
        first[1:] = k[1:] != k[:-1]
        st = np.nonzero(first)[0]
        keys_l.append(k[st])
        starts_l.append(st + base)
        vals_l.append(v)
        sums_l.append(np.add.reduceat(v.astype(np.uint64), st).astype(np.int64))  # wraps mod 2^64
        base += len(k)
    cat = lambda xs: np.concatenate(xs) if xs else np.empty(0, dtype=np.int64)  # noqa: E731
    if agg == "sum":
        return cat(keys_l), cat(sums_l)
    return cat(keys_l), cat(starts_l), cat(vals_l)


def map_combine_sum(records: np.ndarray, num_partitions: int, kind: int = PART_HASH, bounds=None,
                    ascending: bool = True):
    """Map-side combine of reduceByKey(_ + _) on (Long, Long) records (Spark 3.0.1: the writer
    built at UcxShuffleManager.scala:48-51 runs ExternalSorter.insertAll with the aggregator
    -- PartitionedAppendOnlyMap, createCombiner(v) = v, mergeValue(c, v) = c + v with Long
    wrap-around -- and writes one (key, combiner) pair per distinct key and partition).
    Spark iterates a partition's combiners in hash-map order (unspecified); the canonical
    order here is ascending key.  Returns (records (G, 16) partition-contiguous, counts[R]).
    Restated again in pure Python by spark_semantics.map_side_combine_sum."""
    records = np.ascontiguousarray(records)
    R = num_partitions
    if len(records) == 0:
        return np.empty((0, 16), np.uint8), np.zeros(R, np.int64)
    pids = partition_ids(records, R, kind, bounds, ascending).astype(np.int64)
    k = records[:, :8].copy().view("<i8").reshape(-1)
    v = records[:, 8:16].copy().view("<u8").reshape(-1)
    order = np.lexsort((k, pids))
    ks, ps, vs = k[order], pids[order], v[order]
    first = np.ones(len(ks), dtype=bool)
    first[1:] = (ks[1:] != ks[:-1]) | (ps[1:] != ps[:-1])
    st = np.nonzero(first)[0]
    out = np.empty((len(st), 16), np.uint8)
    out[:, :8] = ks[st].view(np.uint8).reshape(-1, 8)
    out[:, 8:] = np.add.reduceat(vs, st).view(np.uint8).reshape(-1, 8)  # uint64 adds wrap
    counts = np.bincount(ps[st], minlength=R).astype(np.int64)
    return out, counts


def kryo_record_lengths(records: np.ndarray) -> np.ndarray:
    """Bytes of each (Long, Long) record in Spark's Kryo stream (spark_semantics.kryo_*)."""
    kv = np.ascontiguousarray(records).view(np.uint64).reshape(-1, 2)
    z = (kv << np.uint64(1)) ^ (kv.view(np.int64) >> np.int64(63)).view(np.uint64)
    bits = np.zeros(z.shape, dtype=np.int64)
    for b in range(64):
        bits = np.where((z >> np.uint64(b)) != 0, b + 1, bits)
    vl = np.minimum(np.maximum((bits + 6) // 7, 1), 9)
    return (2 + vl[:, 0] + vl[:, 1]).astype(np.int64)


def kryo_serialize(records: np.ndarray) -> np.ndarray:
    """Vectorised Kryo framing of (n, 16) uint8 (Long, Long) records -> uint8 stream.  Same
    definition as spark_semantics.kryo_serialize_pairs (the tests pin one to the other)."""
    kv = np.ascontiguousarray(records).view(np.uint64).reshape(-1, 2)
    n = kv.shape[0]
    z = (kv << np.uint64(1)) ^ (kv.view(np.int64) >> np.int64(63)).view(np.uint64)
    mat = np.zeros((n, 20), dtype=np.uint8)
    use = np.zeros((n, 20), dtype=bool)
    col = 0
    for f in range(2):
        mat[:, col] = 0x09
        use[:, col] = True
        col += 1
        x = z[:, f].copy()
        done = np.zeros(n, dtype=bool)
        for i in range(9):
            last = (x < np.uint64(0x80)) | (i == 8)
            byte = np.where(last, x & np.uint64(0xFF), (x & np.uint64(0x7F)) | np.uint64(0x80)).astype(np.uint8)
            live = ~done
            mat[:, col + i] = np.where(live, byte, 0)
            use[:, col + i] = live
            done = done | last
            x = x >> np.uint64(7)
        # compact this field's 9 columns left so the next field starts right after it
        col += 9
    # row-major order of the used cells = the stream
    return mat[use]


def kryo_partition_offsets(records: np.ndarray, counts: np.ndarray) -> np.ndarray:
    """Byte offsets (R+1) of the Kryo-framed partitions of a partition-contiguous output."""
    lens = kryo_record_lengths(records)
    cum = np.zeros(len(lens) + 1, dtype=np.int64)
    np.cumsum(lens, out=cum[1:])
    return cum[offsets(counts)]


# ---------------------------------------------------------------- LZ4 framing -----
# spark.shuffle.compress=true with the lz4 codec: lz4_oracle.c (restatement of liblz4 1.9.x
# LZ4_compress_default, XXH32 and lz4-java's LZ4BlockOutputStream framing).
LZ4_BLOCK_SIZE = 32 * 1024  # spark.io.compression.lz4.blockSize default


def lz4_compress_block(block: bytes) -> bytes:
    src = np.frombuffer(bytes(block), dtype=np.uint8)
    dst = np.empty(len(src) + len(src) // 255 + 16, dtype=np.uint8)
    n = lib().orc_lz4_compress_block(_ptr(src) if len(src) else None, len(src), _ptr(dst))
    return dst[:n].tobytes()


def xxh32(data: bytes, seed: int) -> int:
    src = np.frombuffer(bytes(data), dtype=np.uint8)
    return int(lib().orc_xxh32(_ptr(src) if len(src) else None, len(src), seed & 0xFFFFFFFF))


def lz4_frame_partitions(stream: np.ndarray, offs: np.ndarray, block_size: int = LZ4_BLOCK_SIZE):
    """Each partition stream [offs[r], offs[r+1]) framed as Spark's LZ4BlockOutputStream writes
    it -> (framed bytes uint8, framed lengths int64[R])."""
    stream = np.ascontiguousarray(stream, dtype=np.uint8)
    offs = np.ascontiguousarray(offs, dtype=np.int64)
    R = len(offs) - 1
    lens = np.empty(R, dtype=np.int64)
    sp = _ptr(stream) if len(stream) else None
    total = lib().orc_lz4_frame_partitions(sp, _ptr(offs), R, block_size, None, _ptr(lens))
    out = np.empty(max(total, 1), dtype=np.uint8)
    lib().orc_lz4_frame_partitions(sp, _ptr(offs), R, block_size, _ptr(out), _ptr(lens))
    return out[:total], lens


def unsafe_writer_map_output(spills, num_partitions: int, kind: int = PART_HASH, bounds=None,
                             block_size: int = LZ4_BLOCK_SIZE):
    """UnsafeShuffleWriter (Spark 3.0.1; the reference runs it for a SerializedShuffleHandle,
    spark_3_0/UcxShuffleManager.scala:37-45) over a map whose (Long, Long) records arrive in
    `spills` (one (n, 16) uint8 array per spill), Kryo serializer, spark.shuffle.compress with
    lz4.  Per spill, ShuffleExternalSorter.writeSortedFile: records stably grouped by partition
    id (ShuffleInMemorySorter's radix sort on the partition), every non-empty partition segment
    written through its own compressed stream and closed (DiskBlockObjectWriter.commitAndGet:
    one LZ4BlockOutputStream per segment, ended by its end mark).  Then
    UnsafeShuffleWriter.mergeSpillsWithTransferTo (fast merge: lz4 supports concatenation of
    serialized streams): partition p of the data file = the spills' p segments back to back, in
    spill order.  Returns (data bytes uint8, lengths int64[R])."""
    R = num_partitions
    segs = []  # per spill: (framed bytes, framed offsets[R+1])
    for recs in spills:
        recs = np.ascontiguousarray(recs, dtype=np.uint8).reshape(-1, 16)
        out, counts = map_write(recs, R, kind, bounds)
        ser = kryo_serialize(out) if len(out) else np.zeros(0, np.uint8)
        framed, flens = lz4_frame_partitions(ser, kryo_partition_offsets(out, counts), block_size)
        fo = np.zeros(R + 1, dtype=np.int64)
        np.cumsum(flens, out=fo[1:])
        segs.append((framed, fo))
    parts, lengths = [], np.zeros(R, dtype=np.int64)
    for p in range(R):
        for framed, fo in segs:
            parts.append(framed[fo[p]:fo[p + 1]])
            lengths[p] += fo[p + 1] - fo[p]
    data = np.concatenate(parts) if parts else np.zeros(0, np.uint8)
    return data, lengths

