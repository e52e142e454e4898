"""Pure-Python restatement of the Spark 3.0.1 shuffle-write semantics on the hot path.

TEST INFRASTRUCTURE ONLY.  This module is an oracle: only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it,
and only as the checker.  The product (``sparkucx_amd``) never imports it.

PARITY STATUS: the reference (ofirfarjun7/sparkucx, Scala) ships no tests, no
fixtures and no golden vectors for this path, and its arithmetic lives in the
un-vendored dependency ``org.apache.spark:spark-core_2.12:3.0.1`` (pom.xml:80,90-95),
which cannot be built or run here (no JVM).  This restatement is therefore pinned
by the hand-verified known-answer tests of SURVEY.md §8(c) (Java semantics of
``Long.hashCode`` / ``%`` / ``Utils.nonNegativeMod``) and cross-checked against the
independent C restatement in ``oracle/shuffle_oracle.c``.  See DESIGN.md §Oracle.

Each function names the reference call site / external algorithm it restates.
Pure-Python loops: use only for small cases (fixtures, property checks).
"""
from __future__ import annotations

import struct
from typing import List, Optional, Sequence, Tuple

MASK64 = (1 << 64) - 1
MASK32 = (1 << 32) - 1

# ----------------------------------------------------------------------------
# Java integer semantics
# ----------------------------------------------------------------------------


def to_i32(x: int) -> int:
    """Wrap an integer to Java ``int`` (two's complement, 32 bit)."""
    x &= MASK32
    return x - (1 << 32) if x & 0x80000000 else x


def to_i64(x: int) -> int:
    """Wrap an integer to Java ``long`` (two's complement, 64 bit)."""
    x &= MASK64
    return x - (1 << 64) if x & (1 << 63) else x


def java_rem(a: int, b: int) -> int:
    """Java ``%`` on ints: truncating remainder, sign follows the dividend."""
    r = abs(a) % abs(b)
    return -r if a < 0 else r


def java_long_hash(k: int) -> int:
    """``java.lang.Long.hashCode(long value)`` = ``(int)(value ^ (value >>> 32))``.

    Spark's ``HashPartitioner.getPartition(key)`` calls ``key.hashCode`` on the boxed
    ``java.lang.Long`` (spark-core 3.0.1 ``Partitioner.scala``; invoked by the
    ``SortShuffleWriter`` built at ``spark_3_0/UcxShuffleManager.scala:50-51``).
    NOTE: this is NOT Scala's ``##`` (which maps longs that fit an int to that int,
    e.g. ``(-1L).## == -1`` whereas ``Long.hashCode(-1) == 0``).
    """
    u = k & MASK64
    return to_i32(u ^ (u >> 32))


def non_negative_mod(x: int, mod: int) -> int:
    """``org.apache.spark.util.Utils.nonNegativeMod(x, mod)`` (spark-core 3.0.1)::

        val rawMod = x % mod
        rawMod + (if (rawMod < 0) mod else 0)
    """
    raw = java_rem(x, mod)
    return raw + (mod if raw < 0 else 0)


def hash_partition(key: int, num_partitions: int) -> int:
    """``HashPartitioner.getPartition`` for a non-null ``java.lang.Long`` key.

    ``case null => 0; case _ => Utils.nonNegativeMod(key.hashCode, numPartitions)``.
    Primitive (Long, Long) records have no null keys.
    """
    return non_negative_mod(java_long_hash(key), num_partitions)


# ----------------------------------------------------------------------------
# RangePartitioner.getPartition (spark-core 3.0.1, Partitioner.scala)
# ----------------------------------------------------------------------------


def java_binary_search(a: Sequence, key, lt) -> int:
    """``java.util.Arrays.binarySearch`` (JDK 8 ``binarySearch0``), generic form.

    Returns the index of a match, else ``-(insertion point) - 1``.  Spark's
    ``CollectionsUtils.makeBinarySearch`` dispatches ``Long`` keys to
    ``Arrays.binarySearch(long[], long)`` and other keys to the Comparator form;
    both run this exact loop.
    """
    low, high = 0, len(a) - 1
    while low <= high:
        mid = (low + high) >> 1  # (low + high) >>> 1
        mv = a[mid]
        if lt(mv, key):
            low = mid + 1
        elif lt(key, mv):
            high = mid - 1
        else:
            return mid
    return -(low + 1)


def range_partition(key, bounds: Sequence, ascending: bool = True, lt=None) -> int:
    """``RangePartitioner.getPartition``::

        if (rangeBounds.length <= 128) {
          while (partition < rangeBounds.length && ordering.gt(k, rangeBounds(partition)))
            partition += 1
        } else {
          partition = binarySearch(rangeBounds, k)
          if (partition < 0) partition = -partition-1
          if (partition > rangeBounds.length) partition = rangeBounds.length
        }
        if (ascending) partition else rangeBounds.length - partition

    ``numPartitions = rangeBounds.length + 1``.
    """
    if lt is None:
        lt = lambda x, y: x < y  # noqa: E731
    nb = len(bounds)
    if nb <= 128:
        p = 0
        while p < nb and lt(bounds[p], key):  # ordering.gt(k, b) == lt(b, k)
            p += 1
    else:
        p = java_binary_search(bounds, key, lt)
        if p < 0:
            p = -p - 1
        if p > nb:
            p = nb
    return p if ascending else nb - p


def bytes_lt(a: bytes, b: bytes) -> bool:
    """Unsigned lexicographic order on byte keys (TeraSort's key comparator)."""
    return a < b  # Python bytes compare unsigned-lexicographically


# ----------------------------------------------------------------------------
# Map-side grouping, index layout, block lookup
# ----------------------------------------------------------------------------


def stable_group_by_partition(pids: Sequence[int], num_partitions: int) -> Tuple[List[int], List[int]]:
    """Stable group-by-partition of record indices.

    Restates the ordering contract of ``ExternalSorter``/``PartitionedPairBuffer``
    (TimSort with a partition comparator, stable) and ``ShuffleInMemorySorter``
    (LSD radix on the partition id, stable): runs in increasing partition order,
    map input order inside each run.  Returns ``(order, lengths_in_records)``.
    """
    buckets: List[List[int]] = [[] for _ in range(num_partitions)]
    for i, p in enumerate(pids):
        if not 0 <= p < num_partitions:
            raise ValueError(f"partition id {p} out of range")
        buckets[p].append(i)
    order = [i for b in buckets for i in b]
    return order, [len(b) for b in buckets]


def index_offsets(lengths: Sequence[int]) -> List[int]:
    """``IndexShuffleBlockResolver.writeIndexFileAndCommit`` offsets
    (``IndexShuffleBlockResolver.scala:184-192``): ``[0, L0, L0+L1, ..., sum]``."""
    out = [0]
    for length in lengths:
        out.append(to_i64(out[-1] + length))
    return out


def index_file_bytes(lengths: Sequence[int]) -> bytes:
    """The index file: ``numPartitions + 1`` big-endian longs (``DataOutputStream.writeLong``)."""
    return b"".join(struct.pack(">q", o) for o in index_offsets(lengths))


def check_index_and_data(index_bytes: bytes, data_length: int, blocks: int) -> Optional[List[int]]:
    """``IndexShuffleBlockResolver.checkIndexAndDataFile`` (``:110-149``).

    Returns the partition lengths if index and data match, else ``None``.
    """
    if len(index_bytes) != (blocks + 1) * 8:
        return None
    offs = [struct.unpack_from(">q", index_bytes, 8 * i)[0] for i in range(blocks + 1)]
    if offs[0] != 0:
        return None
    lengths = [offs[i + 1] - offs[i] for i in range(blocks)]
    return lengths if data_length == sum(lengths) else None


def block_range(index_bytes: bytes, start_reduce: int, end_reduce: int) -> Tuple[int, int]:
    """``IndexShuffleBlockResolver.getBlockData`` (``:219-262``): the (offset, length)
    of block ``(map, [start, end))`` read from the index at byte ``reduceId * 8``."""
    start = struct.unpack_from(">q", index_bytes, start_reduce * 8)[0]
    end = struct.unpack_from(">q", index_bytes, end_reduce * 8)[0]
    return start, end - start


def ucx_registered_blocks(lengths: Sequence[int]) -> List[Tuple[int, int, int]]:
    """``CommonUcxShuffleBlockResolver.writeIndexFileAndCommitCommon`` (``:37-61``):
    one ``(reduceId, fileOffset, size)`` per NON-EMPTY partition; offset is the
    running sum of the lengths (equal to the index offsets)."""
    out, off = [], 0
    for r, length in enumerate(lengths):
        if length > 0:
            out.append((r, off, length))
            off += length
    return out


def ucx_block_id_bytes(map_id: int, reduce_id: int) -> bytes:
    """``UcxShuffleBlockId.serialize`` (``UcxShuffleTransport.scala:55-72``): 8 bytes
    ``[mapId:i32][reduceId:i32]`` in ByteBuffer's default (big-endian) order;
    shuffleId is dropped (decodes as 0)."""
    return struct.pack(">ii", to_i32(map_id), to_i32(reduce_id))


# ----------------------------------------------------------------------------
# Synthetic inputs (the build's own definitions)
# ----------------------------------------------------------------------------

GOLDEN_GAMMA = 0x9E3779B97F4A7C15


def splitmix64_at(seed: int, i: int) -> int:
    """Counter-based splitmix64: the i-th output of the stream seeded by ``seed``."""
    z = (seed + (i + 1) * GOLDEN_GAMMA) & MASK64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK64
    return z ^ (z >> 31)


def gen_uniform_records(n: int, seed: int, value_base: int = 0) -> List[Tuple[int, int]]:
    """Uniform (Long, Long) records: key = splitmix64(seed, i) as signed i64,
    value = value_base + i."""
    return [(to_i64(splitmix64_at(seed, i)), value_base + i) for i in range(n)]


def pack_records16(records: Sequence[Tuple[int, int]]) -> bytes:
    """16-byte little-endian ``{i64 key, i64 value}`` record codec."""
    return b"".join(struct.pack("<qq", k, v) for k, v in records)


def map_side_shuffle(records: Sequence[Tuple[int, int]], num_partitions: int):
    """Full map-side write for the fixed 16 B codec with a HashPartitioner:
    returns ``(pids, data_bytes, lengths_in_bytes)``."""
    pids = [hash_partition(k, num_partitions) for k, _ in records]
    order, counts = stable_group_by_partition(pids, num_partitions)
    data = pack_records16([records[i] for i in order])
    return pids, data, [16 * c for c in counts]


def reducer_owner(reduce_id: int, num_partitions: int, world: int) -> int:
    """Contiguous reducer ownership used by the multi-GPU exchange: ``floor(r*P/R)``."""
    return (reduce_id * world) // num_partitions


# ------------------------------------------------------------------ RangePartitioner bounds
# Spark 3.0.1 RangePartitioner (spark-core, external): the rangeBounds initialiser,
# RangePartitioner.sketch, SamplingUtils.reservoirSampleAndCount, XORShiftRandom (+ its
# hashSeed over scala.util.hashing.MurmurHash3.bytesHash) and RangePartitioner.determineBounds,
# restated sequentially.  Parity of this row is UNPINNED: no Spark runs here and the reference
# holds no fixture for it.
M32 = 0xFFFFFFFF
M64 = 0xFFFFFFFFFFFFFFFF


def _rotl32(x, r):
    return ((x << r) | (x >> (32 - r))) & M32


def _mm3_mix_last(h, k):
    k = (k * 0xCC9E2D51) & M32
    k = _rotl32(k, 15)
    k = (k * 0x1B873593) & M32
    return h ^ k


def _mm3_mix(h, k):
    h = _mm3_mix_last(h, k)
    h = _rotl32(h, 13)
    return (h * 5 + 0xE6546B64) & M32


def murmur3_bytes_hash(data: bytes, seed: int) -> int:
    """scala.util.hashing.MurmurHash3.bytesHash (unsigned 32-bit result)."""
    h = seed & M32
    n = len(data)
    i = 0
    while n - i >= 4:
        k = data[i] | (data[i + 1] << 8) | (data[i + 2] << 16) | (data[i + 3] << 24)
        h = _mm3_mix(h, k)
        i += 4
    rem = n - i
    k = 0
    if rem == 3:
        k ^= data[i + 2] << 16
    if rem >= 2:
        k ^= data[i + 1] << 8
    if rem >= 1:
        k ^= data[i]
        h = _mm3_mix_last(h, k)
    h ^= n
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & M32
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & M32
    h ^= h >> 16
    return h


def xorshift_hash_seed(seed: int) -> int:
    b = (seed & M64).to_bytes(8, "big")  # ByteBuffer.putLong: big-endian
    lo = murmur3_bytes_hash(b, 0x3C074A61)  # MurmurHash3.arraySeed
    hi = murmur3_bytes_hash(b, lo)
    return (hi << 32) | lo


class XORShiftRandom:
    """org.apache.spark.util.random.XORShiftRandom: next(bits) + java.util.Random.nextDouble."""

    def __init__(self, seed: int):
        self.s = xorshift_hash_seed(seed)

    def next(self, bits: int) -> int:
        s = self.s
        s ^= (s << 21) & M64
        s ^= s >> 35
        s ^= (s << 4) & M64
        self.s = s
        return s & ((1 << bits) - 1)

    def next_double(self) -> float:
        return ((self.next(26) << 27) + self.next(27)) * (2.0 ** -53)


class JavaRandom:
    """java.util.Random (48-bit LCG): next(bits), nextInt(), nextLong()."""

    MULT, MASK = 0x5DEECE66D, (1 << 48) - 1

    def __init__(self, seed: int):
        self.s = (seed ^ self.MULT) & self.MASK

    def next(self, bits: int) -> int:
        self.s = (self.s * self.MULT + 0xB) & self.MASK
        return to_i32(self.s >> (48 - bits))  # (int)(seed >>> (48 - bits))

    def next_int(self) -> int:
        return self.next(32)

    def next_long(self) -> int:
        return to_i64((self.next(32) << 32) + self.next(32))


def bernoulli_sample(items: Sequence, fraction: float, seed: int) -> list:
    """BernoulliSampler(fraction) after setSeed(seed) (its rng is an XORShiftRandom): fraction
    <= 0.4 (RandomSampler.defaultMaxGapSamplingFraction) uses GapSampling(f, rng, 5e-11) -- one
    advance() when it is built (lazily, at the first sample()), then one per kept item, each
    dropping (log(max(u, eps)) / log1p(-f)).toInt items; otherwise one nextDouble per item,
    kept iff <= fraction."""
    import math

    rng = XORShiftRandom(seed)
    if fraction <= 0.0:
        return []
    if fraction >= 1.0:
        return list(items)
    if fraction <= 0.4:
        lnq = math.log1p(-fraction)

        def advance():
            g = math.log(max(rng.next_double(), 5e-11)) / lnq
            return 2147483647 if g >= 2147483647.0 else int(g)  # Scala Double.toInt saturates

        out, drop = [], advance()
        for it in items:
            if drop > 0:
                drop -= 1
            else:
                drop = advance()
                out.append(it)
        return out
    return [it for it in items if rng.next_double() <= fraction]


def byteswap32(v: int) -> int:
    hc = (v * 0x9E3775CD) & M32
    hc = int.from_bytes(hc.to_bytes(4, "little"), "big")
    return to_i32(hc * 0x9E3775CD)


def reservoir_sample_and_count(keys: Sequence, k: int, seed: int):
    """SamplingUtils.reservoirSampleAndCount."""
    res = list(keys[:k])
    if len(keys) < k:
        return res, len(keys)
    rnd = XORShiftRandom(seed)
    l = k
    for item in keys[k:]:
        l += 1
        r = int(rnd.next_double() * l)  # .toLong truncates; the product is non-negative
        if r < k:
            res[r] = item
    return res, l


def range_bounds(partitions_keys: Sequence[Sequence], num_partitions: int, rdd_id: int = 0,
                 sample_points_per_partition: int = 20, lt=None, parent_rdd_id: Optional[int] = None):
    """RangePartitioner.rangeBounds for input partitions given as key lists.  ``rdd_id`` is the
    id of rdd.map(_._1) (the RDD sketch runs on), ``parent_rdd_id`` the pair RDD's (default
    rdd_id - 1), which seeds the re-sampling of imbalanced partitions:
    new PartitionPruningRDD(rdd.map(_._1), imbalanced).sample(false, fraction,
    byteswap32(-rdd.id - 1)) -- PartitionwiseSampledRDD gives every kept partition, in order,
    the next nextLong() of java.util.Random(seed) for its BernoulliSampler."""
    import math

    if num_partitions <= 1 or not partitions_keys:
        return []
    parent = rdd_id - 1 if parent_rdd_id is None else parent_rdd_id
    sample_size = min(float(sample_points_per_partition) * num_partitions, 1e6)
    k = int(math.ceil(3.0 * sample_size / len(partitions_keys)))
    sketched = []
    for idx, keys in enumerate(partitions_keys):
        seed = byteswap32(to_i32(idx ^ (rdd_id << 16)))
        sample, n = reservoir_sample_and_count(list(keys), k, seed)
        sketched.append((idx, n, sample))
    num_items = sum(n for _, n, _ in sketched)
    if num_items == 0:
        return []
    fraction = min(sample_size / max(num_items, 1), 1.0)
    cand, imbalanced = [], []
    for idx, n, sample in sketched:
        if fraction * n > k:
            imbalanced.append(idx)
        elif sample:
            w = float(np_float32(n / len(sample)))
            cand.extend((key, w) for key in sample)
    if imbalanced:
        jr = JavaRandom(byteswap32(to_i32(-parent - 1)))
        w = float(np_float32(1.0 / fraction))
        for idx in imbalanced:
            cand.extend((key, w) for key in bernoulli_sample(list(partitions_keys[idx]), fraction, jr.next_long()))
    return determine_bounds(cand, min(num_partitions, len(cand)), lt)


def np_float32(x: float) -> float:
    import struct as _s

    return _s.unpack("<f", _s.pack("<f", x))[0]


def determine_bounds(candidates, partitions: int, lt=None):
    """RangePartitioner.determineBounds: stable sort by key, weights summed in sorted order."""
    import functools

    if lt is None:
        ordered = sorted(candidates, key=lambda kw: kw[0])
    else:
        ordered = sorted(candidates, key=functools.cmp_to_key(
            lambda a, b: -1 if lt(a[0], b[0]) else (1 if lt(b[0], a[0]) else 0)))
    gt = (lambda a, b: a > b) if lt is None else (lambda a, b: lt(b, a))
    sum_w = 0.0
    for _, w in ordered:
        sum_w += w
    step = sum_w / partitions
    cum, target = 0.0, step
    bounds, prev = [], None
    i = j = 0
    while i < len(ordered) and j < partitions - 1:
        key, w = ordered[i]
        cum += w
        if cum >= target:
            if prev is None or gt(key, prev):
                bounds.append(key)
                target += step
                j += 1
                prev = key
        i += 1
    return bounds


# ---------------------------------------------------------------------------------------
# Kryo framing of (Long, Long) records.  Spark's KryoSerializer
# (spark-core 3.0.1, kryo-shaded 4.0.2, both external): KryoSerializationStream.writeKey /
# writeValue -> kryo.writeClassAndObject(output, java.lang.Long).  Restated from Kryo's
# published sources:
#   * Kryo's constructor registers int, String, float, boolean, byte, char, short, long,
#     double, void as ids 0..9 (primitive wrappers share the primitive's registration), so
#     java.lang.Long is id 7 and DefaultClassResolver.writeClass writes varint(7 + 2) = 0x09;
#   * MapReferenceResolver.useReferences is false for wrapper classes: no reference byte;
#   * DefaultSerializers.LongSerializer.write = output.writeLong(v, false), which in Kryo 4
#     is writeVarLong(v, optimizePositive = false): zigzag, then 7 bits per byte, low group
#     first, 0x80 = more follows; the 9th byte (if any) carries bits 56..63 whole.
# With spark.shuffle.compress = false (and no encryption) SerializerManager.wrapStream is the
# identity, so a partition's bytes are its records' encodings back to back.
# Parity unpinned against a JVM (none here); pinned by hand-computed known answers.
# ---------------------------------------------------------------------------------------
KRYO_LONG_CLASS_BYTE = 0x09


def kryo_write_var_long(v: int, optimize_positive: bool = False) -> bytes:
    """Kryo 4 Output.writeVarLong."""
    z = v & 0xFFFFFFFFFFFFFFFF
    if not optimize_positive:
        z = ((z << 1) ^ (0xFFFFFFFFFFFFFFFF if v < 0 else 0)) & 0xFFFFFFFFFFFFFFFF
    out = bytearray()
    for _ in range(8):
        if z < 0x80:
            break
        out.append((z & 0x7F) | 0x80)
        z >>= 7
    out.append(z & 0xFF)
    return bytes(out)


def kryo_read_var_long(buf: bytes, pos: int, optimize_positive: bool = False) -> Tuple[int, int]:
    """Kryo 4 Input.readVarLong: returns (value, new position)."""
    z, shift = 0, 0
    for i in range(9):
        b = buf[pos]
        pos += 1
        if i == 8:
            z |= b << 56
            break
        z |= (b & 0x7F) << shift
        shift += 7
        if not b & 0x80:
            break
    if not optimize_positive:
        z = (z >> 1) ^ (-(z & 1) & 0xFFFFFFFFFFFFFFFF)
    return to_i64(z), pos


def kryo_serialize_pairs(records: Sequence[Tuple[int, int]]) -> bytes:
    """KryoSerializationStream of writeKey(k); writeValue(v) for each (Long, Long)."""
    out = bytearray()
    for k, v in records:
        out.append(KRYO_LONG_CLASS_BYTE)
        out += kryo_write_var_long(k)
        out.append(KRYO_LONG_CLASS_BYTE)
        out += kryo_write_var_long(v)
    return bytes(out)


def kryo_deserialize_pairs(buf: bytes) -> List[Tuple[int, int]]:
    """KryoDeserializationStream.asKeyValueIterator over (Long, Long): readClassAndObject x 2."""
    out, pos = [], 0
    while pos < len(buf):
        pair = []
        for _ in range(2):
            if buf[pos] != KRYO_LONG_CLASS_BYTE:
                raise ValueError(f"class byte {buf[pos]:#x} at {pos} is not java.lang.Long")
            x, pos = kryo_read_var_long(buf, pos + 1)
            pair.append(x)
        out.append((pair[0], pair[1]))
    return out


# ---------------------------------------------------------------------------------------
# Map-side combine (dep.mapSideCombine = true, reduceByKey's default).  Spark 3.0.1
# SortShuffleWriter -> ExternalSorter(aggregator = Some(agg)).insertAll: every record goes
# through PartitionedAppendOnlyMap.changeValue((getPartition(k), k), update) with
# update(hadValue, old) = hadValue ? mergeValue(old, v) : createCombiner(v); for
# reduceByKey(_ + _) on Longs createCombiner = identity, mergeValue = + (two's-complement
# wrap).  writePartitionedMapOutput then emits each partition's (k, combiner) pairs; the
# within-partition iteration order of the hash map is unspecified -- canonical: ascending key.
# ---------------------------------------------------------------------------------------
def map_side_combine_sum(records: Sequence[Tuple[int, int]], num_partitions: int):
    combiners = {}
    for k, v in records:
        key = (hash_partition(k, num_partitions), k)
        combiners[key] = to_i64(combiners[key] + v) if key in combiners else to_i64(v)
    return [(k, c) for (_, k), c in sorted(combiners.items())]
