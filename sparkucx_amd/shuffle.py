"""Host-side mirror of SparkUCX's plugin interface for the accelerated path.

Names, argument meaning and error behaviour follow the reference (Spark 3.0 profile,
/root/reference/src/main/scala/org/apache/spark/...):

  UcxShuffleManager            shuffle/compat/spark_3_0/UcxShuffleManager.scala:25-80
                               + shuffle/ucx/CommonUcxShuffleManager.scala:25-124
  GpuShuffleMapOutputWriter    shuffle/ucx/NvkvShuffleMapOutputWriter.scala:75-148
  UcxShuffleBlockResolver      IndexShuffleBlockResolver.scala:56-262 +
                               shuffle/ucx/CommonUcxShuffleBlockResolver.scala:37-71
  UcxShuffleReader             shuffle/compat/spark_3_0/UcxShuffleReader.scala:74-200
  GpuShuffleTransport          shuffle/ucx/ShuffleTransport.scala:110-167

The data path underneath is the HIP engine (libsgx.so); these classes hold no data and
compute nothing on the CPU.
"""
from __future__ import annotations

import enum
import os
import re
import struct
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence

import numpy as np

from . import _lib
from ._lib import IllegalArgumentException, IllegalStateException, UnsupportedOperationException
from .engine import DeviceBuffer, ShuffleEngine

# ---------------------------------------------------------------------------------------
# Partitioners / dependency / handle (Spark core types the plugin receives)
# ---------------------------------------------------------------------------------------


@dataclass(frozen=True)
class HashPartitioner:
    """org.apache.spark.HashPartitioner: nonNegativeMod(key.hashCode, numPartitions)."""

    numPartitions: int
    kind: int = _lib.PART_HASH

    def __post_init__(self):
        if self.numPartitions < 0:
            raise IllegalArgumentException(
                f"Number of partitions ({self.numPartitions}) cannot be negative.")


@dataclass(frozen=True)
class RangePartitioner:
    """org.apache.spark.RangePartitioner with its (already sampled) rangeBounds.
    ``rangeBounds``: int64 keys, or (n, 10) uint8 TeraSort keys (unsigned lexicographic)."""

    rangeBounds: np.ndarray
    ascending: bool = True

    @property
    def kind(self) -> int:
        b = np.asarray(self.rangeBounds)
        return _lib.PART_RANGE_BYTES10 if b.dtype == np.uint8 else _lib.PART_RANGE_I64

    @property
    def numPartitions(self) -> int:
        b = np.asarray(self.rangeBounds)
        n = b.shape[0] if b.ndim else 0
        return n + 1

    @classmethod
    def fromData(cls, engine, partitions: Sequence, nrecords: Sequence[int], recordBytes: int, numPartitions: int,
                 rddId: int = 0, ascending: bool = True, samplePointsPerPartitionHint: int = 20,
                 parentRddId: Optional[int] = None):
        """new RangePartitioner(partitions, rdd, ascending, samplePointsPerPartitionHint): the
        bounds come from RangePartitioner.sketch (GPU reservoir sampling with Spark's seeds),
        the re-sampling of imbalanced partitions and determineBounds.  ``partitions`` are the
        RDD's input partitions (record batches); ``rddId`` is the id of rdd.map(_._1) the
        sketch runs on, ``parentRddId`` the pair RDD's (default rddId - 1)."""
        b = engine.range_bounds(partitions, nrecords, recordBytes, numPartitions, rddId, samplePointsPerPartitionHint,
                                parentRddId)
        return cls(b, ascending)


@dataclass
class Aggregator:
    """Spark's Aggregator for the two combines the engine runs on (Long, Long) records:
    "group" = groupByKey (CompactBuffer append; Spark builds it with mapSideCombine = false),
    "sum" = reduceByKey(_ + _) on Long values (wrapping), with or without map-side combine."""
    kind: str = "group"

    def __post_init__(self):
        if self.kind not in ("group", "sum"):
            raise IllegalArgumentException(f"unsupported aggregator {self.kind!r} (group, sum)")


_SERIALIZERS = {"fixed": _lib.SER_FIXED, "kryo": _lib.SER_KRYO,
                "org.apache.spark.serializer.KryoSerializer": _lib.SER_KRYO}


@dataclass
class ShuffleDependency:
    partitioner: object
    recordBytes: int = 16  # fixed-width record codec: 16 B (Long, Long) or 100 B TeraSort
    aggregator: Optional[Aggregator] = None  # dep.aggregator
    keyOrdering: bool = False                # dep.keyOrdering: sort each reducer by key
    # dep.mapSideCombine (reduceByKey's default is true): the writer combines per key before
    # the shuffle (ExternalSorter.insertAll with the aggregator), the reader merges the
    # combiners (combineCombinersByKey, UcxShuffleReader.scala:158-161)
    mapSideCombine: bool = False
    # dep.serializer: "fixed" = the engine's fixed-width record codec; "kryo" =
    # org.apache.spark.serializer.KryoSerializer with spark.shuffle.compress=false (the data
    # file, index offsets and fetched blocks are Spark's own Kryo stream bytes)
    serializer: str = "fixed"

    def __post_init__(self):
        if self.mapSideCombine:
            # Spark's own check (ShuffleDependency: "Map-side combine without Aggregator
            # specified!")
            if self.aggregator is None:
                raise IllegalArgumentException("Map-side combine without Aggregator specified!")
            if self.aggregator.kind != "sum" or self.recordBytes != 16:
                raise UnsupportedOperationException(
                    "map-side combine runs on the GPU for reduceByKey(_ + _) on (Long, Long) records")
        if self.serializer not in _SERIALIZERS:
            raise IllegalArgumentException(f"unknown serializer {self.serializer!r} (fixed, kryo)")
        if self.serializer == "kryo" and self.recordBytes != 16:
            raise UnsupportedOperationException("Kryo framing is for (Long, Long) 16 B records")


@dataclass
class BaseShuffleHandle:
    shuffleId: int
    dependency: ShuffleDependency
    # the writer the reference's getWriter runs for this handle
    # (spark_3_0/UcxShuffleManager.scala:32-53): UnsafeShuffleWriter for a
    # SerializedShuffleHandle, SortShuffleWriter for every other handle (bypass included)
    writerClass = "SortShuffleWriter"


@dataclass
class BypassMergeSortShuffleHandle(BaseShuffleHandle):
    """SortShuffleWriter.shouldBypassMergeSort: no map-side combine and at most
    spark.shuffle.sort.bypassMergeThreshold (200) partitions.  The reference's getWriter still
    runs SortShuffleWriter for it."""


@dataclass
class SerializedShuffleHandle(BaseShuffleHandle):
    """SortShuffleManager.canUseSerializedShuffle: a serializer that supports relocation of
    serialized objects (Kryo), no map-side combine, at most 2^24 partitions."""
    writerClass = "UnsafeShuffleWriter"


@dataclass
class MapStatus:
    mapId: int
    partitionLengths: np.ndarray  # bytes per reduce partition


# ---------------------------------------------------------------------------------------
# Transport contract (ShuffleTransport.scala)
# ---------------------------------------------------------------------------------------


class OperationStatus(enum.Enum):
    SUCCESS = 0
    CANCELED = 1
    FAILURE = 2


@dataclass
class MemoryBlock:
    """ShuffleTransport.scala:15-20. The receiver owns it and must close() it."""

    address: int
    size: int
    isHostMemory: bool = True
    _owner: object = None
    _on_close: Optional[Callable[[], None]] = None

    def close(self):
        if self._on_close is not None:
            self._on_close()
            self._on_close = None


@dataclass(frozen=True)
class UcxShuffleBlockId:
    """UcxShuffleTransport.scala:55-72: serialized as [mapId:i32][reduceId:i32]; the
    shuffleId is not on the wire (it decodes as 0)."""

    shuffleId: int
    mapId: int
    reduceId: int
    serializedSize: int = 8

    def serialize(self) -> bytes:
        return struct.pack(">ii", _to_i32(self.mapId), _to_i32(self.reduceId))

    @staticmethod
    def deserialize(buf: bytes) -> "UcxShuffleBlockId":
        m, r = struct.unpack(">ii", buf[:8])
        return UcxShuffleBlockId(0, m, r)


def _to_i32(x: int) -> int:
    x &= 0xFFFFFFFF
    return x - (1 << 32) if x & 0x80000000 else x


@dataclass
class OperationResult:
    status: OperationStatus
    data: Optional[MemoryBlock] = None
    error: Optional[Exception] = None

    def getStatus(self):
        return self.status

    def getData(self):
        return self.data

    def getError(self):
        return self.error


@dataclass
class Request:
    completed: bool = False

    def isCompleted(self) -> bool:
        return self.completed


class MemoryPool:
    """memory/MemoryPool.scala:22-147 on the engine (sgx_pool_*): power-of-two size classes
    from minBufferSize (4 KiB) of pinned host memory (host=True, the default: DMA-able by the
    GPU) or HBM; ``get`` is the transport's BufferAllocator (ShuffleTransport.scala:113), the
    returned MemoryBlock's close() puts the buffer back."""

    def __init__(self, engine: ShuffleEngine):
        self.engine = engine

    def get(self, size: int, host: bool = True) -> MemoryBlock:
        import ctypes
        p, cap = ctypes.c_void_p(), ctypes.c_int64()
        _lib.check(_lib.lib().sgx_pool_get(self.engine.handle, int(size), _lib.MEM_HOST if host else _lib.MEM_DEVICE,
                                           ctypes.byref(p), ctypes.byref(cap)), "MemoryPool.get")
        addr = int(p.value)
        return MemoryBlock(addr, int(cap.value), host, self,
                           lambda: _lib.check(_lib.lib().sgx_pool_put(self.engine.handle, addr), "MemoryPool.put"))

    def preallocate(self, size: int, count: int, host: bool = True):
        _lib.check(_lib.lib().sgx_pool_preallocate(self.engine.handle, int(size), int(count),
                                                   _lib.MEM_HOST if host else _lib.MEM_DEVICE), "preallocate")

    def stats(self):
        import ctypes
        a, i = ctypes.c_int64(), ctypes.c_int64()
        _lib.check(_lib.lib().sgx_pool_stats(self.engine.handle, ctypes.byref(a), ctypes.byref(i)), "pool stats")
        return int(a.value), int(i.value)


class GpuShuffleTransport:
    """ShuffleTransport backed by the HIP engine: blocks are served from HBM (local map
    outputs or data received by the RCCL exchange) instead of UCX AM round trips."""

    def __init__(self, engine: ShuffleEngine):
        self.engine = engine
        self._pending: List[tuple] = []
        # UcxHostBounceBuffersPool (UcxShuffleTransport.scala:122-164): the default allocator
        self.hostBounceBufferMemoryPool = MemoryPool(engine)

    def init(self):
        return None

    def close(self):
        self._pending.clear()

    def register(self, blockId, block=None):
        return None  # map outputs register themselves when written

    def unregister(self, blockId):
        return None

    def unregisterShuffle(self, shuffleId: int):
        self.engine.unregister_shuffle(shuffleId)

    def fetchBlocksByBlockIds(self, executorId: int, blockIds: Sequence[UcxShuffleBlockId],
                              resultBufferAllocator: Callable[[int], MemoryBlock],
                              callbacks: Sequence[Callable[[OperationResult], None]]) -> List[Request]:
        """ShuffleTransport.scala:154-156.  Completion is delivered by progress() on the
        submitting thread, as in the reference (:158-165)."""
        if len(blockIds) != len(callbacks):
            raise IllegalArgumentException("blockIds and callbacks differ in length")
        reqs = []
        for bid, cb in zip(blockIds, callbacks):
            r = Request()
            reqs.append(r)
            self._pending.append((bid, resultBufferAllocator, cb, r))
        return reqs

    def progress(self):
        pending, self._pending = self._pending, []
        for bid, alloc, cb, req in pending:
            try:
                host, lens = self.engine.fetch_blocks(bid.shuffleId, [bid.mapId], [bid.reduceId])
                mb = alloc(int(lens[0]))
                if mb.size < int(lens[0]):
                    raise IllegalStateException("allocator returned a block smaller than requested")
                if lens[0]:
                    import ctypes
                    ctypes.memmove(mb.address, host.ctypes.data, int(lens[0]))
                req.completed = True
                cb(OperationResult(OperationStatus.SUCCESS, MemoryBlock(mb.address, int(lens[0]), True,
                                                                          mb, mb.close)))
            except _lib.ShuffleError as ex:
                req.completed = True
                cb(OperationResult(OperationStatus.FAILURE, None, ex))


class BlockFetchingListener:
    """org.apache.spark.network.shuffle.BlockFetchingListener."""

    def onBlockFetchSuccess(self, blockId: str, data) -> None:  # pragma: no cover - interface
        raise NotImplementedError

    def onBlockFetchFailure(self, blockId: str, exception: BaseException) -> None:  # pragma: no cover
        raise NotImplementedError


class UcxShuffleClient:
    """BlockStoreClient.fetchBlocks over the engine's HBM-resident blocks
    (spark_3_0/UcxShuffleClient.scala:17-91; Scala edition in jvm/.../GpuShuffleClient.scala).
    Same signature, same recursive split in halves (``splitAt(length / 2)``) while a request
    holds more than spark.shuffle.ucx.maxBlocksPerRequest ids (default 50, :53-58), same
    "shuffle_<s>_<m>_<r>" ids (:64).  One engine fetch (one gather launch)
    per request instead of one synchronous round trip per block (:17-47); a failed request
    reports onBlockFetchFailure for each of its blocks, which the reference never does
    (:36-40), so Spark's FetchFailed / stage retry runs."""

    def __init__(self, transport: "GpuShuffleTransport", conf: Optional[Dict[str, str]] = None):
        self.transport = transport
        self.maxBlocksPerRequest = int((conf or {}).get("spark.shuffle.ucx.maxBlocksPerRequest", 50))
        self.requests = 0  # engine fetches issued (tests check the split)
        self.request_sizes: List[int] = []  # block ids per engine fetch, in issue order

    def fetchBlocks(self, host: str, port: int, execId: str, blockIds: Sequence[str],
                    listener: BlockFetchingListener, downloadFileManager=None) -> None:
        blockIds = list(blockIds)
        if len(blockIds) > self.maxBlocksPerRequest:
            # the reference's split (UcxShuffleClient.scala:53-58): halve, recurse on both halves
            half = len(blockIds) // 2
            self.fetchBlocks(host, port, execId, blockIds[:half], listener, downloadFileManager)
            self.fetchBlocks(host, port, execId, blockIds[half:], listener, downloadFileManager)
            return
        if not blockIds:
            return
        try:
            parsed = [parse_block_id(b) for b in blockIds]
            sids = {s for s, _, _ in parsed}
            if len(sids) != 1:
                raise IllegalArgumentException("blocks of one request belong to one shuffle")
            self.requests += 1
            self.request_sizes.append(len(blockIds))
            data, lens = self.transport.engine.fetch_blocks(sids.pop(), [m for _, m, _ in parsed],
                                                            [r for _, _, r in parsed])
        except _lib.ShuffleError as ex:
            for b in blockIds:
                listener.onBlockFetchFailure(b, ex)
            return
        off = 0
        for b, n in zip(blockIds, lens):
            listener.onBlockFetchSuccess(b, data[off:off + int(n)])
            off += int(n)

    def close(self):
        return None


# ---------------------------------------------------------------------------------------
# Writer side
# ---------------------------------------------------------------------------------------


class ShufflePartitionWriter:
    def __init__(self, length: int):
        self._length = length

    def getNumBytesWritten(self) -> int:
        return self._length


class GpuShuffleMapOutputWriter:
    """ShuffleMapOutputWriter contract (NvkvShuffleMapOutputWriter.scala:75-148) over a
    map output already partitioned in HBM: partitions are visited in strictly increasing
    order (:108) and commitAllPartitions returns the per-partition lengths (:116-148)."""

    def __init__(self, shuffleId: int, mapId: int, lengths: np.ndarray):
        self.shuffleId, self.mapId = shuffleId, mapId
        self._lengths = lengths
        self._last = -1

    def getPartitionWriter(self, reducePartitionId: int) -> ShufflePartitionWriter:
        if reducePartitionId <= self._last:
            raise IllegalArgumentException("Partitions should be requested in increasing order.")
        if not 0 <= reducePartitionId < len(self._lengths):
            raise IllegalArgumentException(f"partition {reducePartitionId} out of range")
        self._last = reducePartitionId
        return ShufflePartitionWriter(int(self._lengths[reducePartitionId]))

    def commitAllPartitions(self) -> np.ndarray:
        return self._lengths.copy()

    def abort(self, error: BaseException):
        return None


class GpuShuffleWriter:
    """The ShuffleWriter getWriter returns (UcxShuffleManager.scala:32-53): one write() of a
    record batch runs partition id -> histogram -> scan -> stable scatter on the GPU."""

    def __init__(self, manager: "UcxShuffleManager", handle: BaseShuffleHandle, mapId: int):
        self.manager, self.handle, self.mapId = manager, handle, mapId
        self._status: Optional[MapStatus] = None

    def write(self, records, numRecords: Optional[int] = None):
        """records: one batch (numpy / torch / DeviceBuffer), or a list of batches -- the
        spills of the map task, appended in order (sgx_map_begin / _append / _commit)."""
        dep = self.handle.dependency
        rb = dep.recordBytes
        if isinstance(records, (list, tuple)):
            e, sid = self.manager.engine, self.handle.shuffleId
            e.map_begin(sid, self.mapId)
            for batch in records:
                e.map_append(sid, self.mapId, batch, self._count(batch, rb), rb)
            lengths = e.map_commit(sid, self.mapId, dep.partitioner.numPartitions)
            self.manager._map_written(sid, self.mapId)
            self._status = MapStatus(self.mapId, lengths)
            return
        if numRecords is None:
            if isinstance(records, np.ndarray):
                numRecords = records.nbytes // rb
            elif isinstance(records, DeviceBuffer):
                numRecords = records.nbytes // rb
            else:
                numRecords = records.numel() * records.element_size() // rb
        R = dep.partitioner.numPartitions
        lengths = self.manager.engine.write_map(self.handle.shuffleId, self.mapId, records, numRecords, rb, R)
        self.manager._map_written(self.handle.shuffleId, self.mapId)
        self._status = MapStatus(self.mapId, lengths)

    @staticmethod
    def _count(batch, rb: int) -> int:
        if isinstance(batch, (np.ndarray, DeviceBuffer)):
            return batch.nbytes // rb
        return batch.numel() * batch.element_size() // rb

    def mapOutputWriter(self) -> GpuShuffleMapOutputWriter:
        if self._status is None:
            raise IllegalStateException("write() was not called")
        return GpuShuffleMapOutputWriter(self.handle.shuffleId, self.mapId, self._status.partitionLengths)

    def getPartitionLengths(self) -> np.ndarray:
        if self._status is None:
            raise IllegalStateException("write() was not called")
        return self._status.partitionLengths

    def stop(self, success: bool) -> Optional[MapStatus]:
        return self._status if success else None


# ---------------------------------------------------------------------------------------
# Index + data layout (IndexShuffleBlockResolver)
# ---------------------------------------------------------------------------------------

_BLOCK_RE = re.compile(r"^shuffle_(\d+)_(-?\d+)_(\d+)$")


def parse_block_id(name: str):
    """'shuffle_<s>_<m>_<r>' (UcxShuffleClient.scala:64 via BlockId.apply)."""
    m = _BLOCK_RE.match(name)
    if not m:
        raise IllegalArgumentException(f"unexpected shuffle block id format: {name}")
    return int(m.group(1)), int(m.group(2)), int(m.group(3))


class UcxShuffleBlockResolver:
    """Index/data files in Spark's layout, written from HBM. NOOP_REDUCE_ID = 0 (:271)."""

    NOOP_REDUCE_ID = 0

    def __init__(self, manager: "UcxShuffleManager", root: str):
        self.manager = manager
        self.root = root
        os.makedirs(root, exist_ok=True)

    def getDataFile(self, shuffleId: int, mapId: int) -> str:
        return os.path.join(self.root, f"shuffle_{shuffleId}_{mapId}_{self.NOOP_REDUCE_ID}.data")

    def getIndexFile(self, shuffleId: int, mapId: int) -> str:
        return os.path.join(self.root, f"shuffle_{shuffleId}_{mapId}_{self.NOOP_REDUCE_ID}.index")

    def writeIndexFileAndCommit(self, shuffleId: int, mapId: int, lengths: np.ndarray) -> None:
        """IndexShuffleBlockResolver.scala:161-217; ``lengths`` is updated in place to the
        committed attempt's lengths (an existing valid attempt wins)."""
        got = self.manager.engine.write_index(shuffleId, mapId, self.getIndexFile(shuffleId, mapId),
                                              self.getDataFile(shuffleId, mapId), len(lengths))
        lengths[:] = got

    def checkIndexAndDataFile(self, index: str, data: str, blocks: int) -> Optional[np.ndarray]:
        out = np.empty(blocks, dtype=np.int64)
        rc = _lib.lib().sgx_check_index_and_data(index.encode(), data.encode(), blocks, out.ctypes.data)
        return out if rc == 0 else None

    def getBlockData(self, blockId) -> bytes:
        """IndexShuffleBlockResolver.scala:219-262 (ShuffleBlockId or (s, m, start, end))."""
        if isinstance(blockId, str):
            s, m, r = parse_block_id(blockId)
            start, end = r, r + 1
        elif len(blockId) == 3:
            s, m, start = blockId
            end = start + 1
        elif len(blockId) == 4:
            s, m, start, end = blockId
        else:
            raise IllegalArgumentException(f"unexpected shuffle block id format: {blockId}")
        import ctypes
        off, ln = ctypes.c_int64(), ctypes.c_int64()
        _lib.check(_lib.lib().sgx_index_block_range(self.getIndexFile(s, m).encode(), start, end,
                                                    ctypes.byref(off), ctypes.byref(ln)), "getBlockData")
        with open(self.getDataFile(s, m), "rb") as f:
            f.seek(off.value)
            return f.read(ln.value)

    def removeDataByMap(self, shuffleId: int, mapId: int):
        for p in (self.getDataFile(shuffleId, mapId), self.getIndexFile(shuffleId, mapId)):
            if os.path.exists(p):
                os.unlink(p)


# ---------------------------------------------------------------------------------------
# Reader
# ---------------------------------------------------------------------------------------


class TaskKilledException(_lib.ShuffleError):
    """org.apache.spark.TaskKilledException: the task was cancelled."""


class TaskContext:
    """The part of Spark's TaskContext a shuffle read uses: cancellation (``markInterrupted``
    by the executor, ``killTaskIfInterrupted`` by the task) and the task's read metrics
    (``taskMetrics().mergeShuffleReadMetrics()`` folds a reader's temporary metrics in)."""

    def __init__(self):
        self._reason: Optional[str] = None
        self.shuffleReadMetrics = ShuffleReadMetricsReporter()
        self._temps: List["ShuffleReadMetricsReporter"] = []

    def markInterrupted(self, reason: str = "killed") -> None:
        self._reason = reason

    def isInterrupted(self) -> bool:
        return self._reason is not None

    def killTaskIfInterrupted(self) -> None:
        if self._reason is not None:
            raise TaskKilledException(self._reason)

    def createTempShuffleReadMetrics(self) -> "ShuffleReadMetricsReporter":
        m = ShuffleReadMetricsReporter()
        self._temps.append(m)
        return m

    def mergeShuffleReadMetrics(self) -> None:
        t = ShuffleReadMetricsReporter()
        for m in self._temps:
            for k, v in vars(m).items():
                setattr(t, k, getattr(t, k) + v)
        self.shuffleReadMetrics = t


class ShuffleReadMetricsReporter:
    """Spark 3.0's ShuffleReadMetricsReporter (what getReader's ``metrics`` is): the counters the
    reference's reader feeds (spark_3_0/UcxShuffleReader.scala:118-123 fetch wait, :148-153
    records read) plus the block / byte counts Spark's fetcher iterator reports."""

    def __init__(self):
        self.remoteBlocksFetched = 0
        self.localBlocksFetched = 0
        self.remoteBytesRead = 0
        self.localBytesRead = 0
        self.fetchWaitTime = 0  # ms
        self.recordsRead = 0

    def incRemoteBlocksFetched(self, v: int) -> None:
        self.remoteBlocksFetched += int(v)

    def incLocalBlocksFetched(self, v: int) -> None:
        self.localBlocksFetched += int(v)

    def incRemoteBytesRead(self, v: int) -> None:
        self.remoteBytesRead += int(v)

    def incLocalBytesRead(self, v: int) -> None:
        self.localBytesRead += int(v)

    def incFetchWaitTime(self, ms: int) -> None:
        self.fetchWaitTime += int(ms)

    def incRecordsRead(self, v: int) -> None:
        self.recordsRead += int(v)


class InterruptibleIterator:
    """org.apache.spark.InterruptibleIterator: checks the task's cancellation before every
    element (the reference wraps its read in one, spark_3_0/UcxShuffleReader.scala:155-156,
    193-199)."""

    def __init__(self, context: TaskContext, delegate):
        self.context = context
        self.delegate = iter(delegate)

    def __iter__(self):
        return self

    def __next__(self):
        self.context.killTaskIfInterrupted()
        return next(self.delegate)


class UcxShuffleReader:
    """Reads reduce partitions [startPartition, endPartition) (UcxShuffleReader.scala:74-200).
    Blocks are fetched per (map, reduce) from HBM; the result is returned in the canonical
    order: reduce partition ascending, then map (source) ascending, map input order inside
    each block (SURVEY.md §8(a) parity note)."""

    def __init__(self, manager: "UcxShuffleManager", handle: BaseShuffleHandle, startPartition: int,
                 endPartition: int, mapIds: Optional[Sequence[int]] = None, context: Optional[TaskContext] = None,
                 readMetrics: Optional[ShuffleReadMetricsReporter] = None):
        R = handle.dependency.partitioner.numPartitions
        if not 0 <= startPartition <= endPartition <= R:
            raise IllegalArgumentException(f"bad partition range [{startPartition}, {endPartition})")
        self.manager, self.handle = manager, handle
        self.start, self.end = startPartition, endPartition
        self.mapIds = list(mapIds) if mapIds is not None else None
        self.context = context or TaskContext()
        self.readMetrics = readMetrics if readMetrics is not None else self.context.createTempShuffleReadMetrics()

    def _count_blocks(self) -> None:
        """Local blocks and bytes of the range (every block this engine holds for it)."""
        maps = self._maps()
        rids = [r for r in range(self.start, self.end) for _ in maps]
        lens = self.manager.engine.block_lengths(self.handle.shuffleId, maps * (self.end - self.start), rids)
        self.readMetrics.incLocalBlocksFetched(int(np.count_nonzero(lens)))
        self.readMetrics.incLocalBytesRead(int(lens.sum()))

    def read_blocks(self):
        maps = self.mapIds if self.mapIds is not None else self.manager.known_maps(self.handle.shuffleId)
        mids, rids = [], []
        for r in range(self.start, self.end):
            for m in sorted(maps):
                mids.append(m)
                rids.append(r)
        data, lens = self.manager.engine.fetch_blocks(self.handle.shuffleId, mids, rids)
        return data, lens, mids, rids

    def readSerialized(self) -> np.ndarray:
        """The partition range's serialized bytes as Spark's reader sees them after
        SerializerManager.wrapStream (UcxShuffleReader.scala:137-145): fetched blocks, LZ4
        frames decompressed on the GPU when the shuffle is compressed."""
        data, _, _, _ = self.read_blocks()
        if self.manager.compressed(self.handle.shuffleId):
            return self.manager.engine.lz4_unframe(data)
        return data

    def _maps(self):
        return sorted(self.mapIds if self.mapIds is not None else self.manager.known_maps(self.handle.shuffleId))

    def read(self):
        """UcxShuffleReader.read (:74-200) on the GPU.
        * no aggregator, no keyOrdering: every record of the partition range in the canonical
          order, as an (n, recordBytes) uint8 array;
        * keyOrdering (sortByKey, TeraSort): the same records, each reducer sorted stably by
          key (ExternalSorter with an ordering, :166-181);
        * aggregator "group" (groupByKey, combineValuesByKey :155-164): (keys, group_starts,
          values) -- keys ascending per reducer, values in arrival order;
        * aggregator "sum" (reduceByKey(_ + _)): (keys, sums).
        Metrics as the reference's reader reports them: the range's blocks and bytes, and
        ``incRecordsRead`` with the shuffled records read (for an aggregator: the records it
        consumed, not its groups); a task killed before the read raises TaskKilledException
        (``iterator()`` checks per record)."""
        dep = self.handle.dependency
        sid = self.handle.shuffleId
        self.context.killTaskIfInterrupted()
        self._count_blocks()
        if dep.aggregator is not None:
            if dep.recordBytes != 16:
                raise UnsupportedOperationException("aggregation needs (Long, Long) 16 B records")
            agg = _lib.AGG_SUM if dep.aggregator.kind == "sum" else _lib.AGG_GROUP
            out = self.manager.engine.read_grouped(sid, self._maps(), self.start, self.end, agg)
            # the shuffled records the aggregator consumed, not its groups (the reference counts
            # ahead of combineValuesByKey / combineCombinersByKey, UcxShuffleReader.scala:148-162)
            nrec = self.manager.engine.last_read_records()
        elif dep.keyOrdering:
            out = self.manager.engine.read_sorted(sid, self._maps(), self.start, self.end).reshape(-1, dep.recordBytes)
            nrec = len(out)
        elif _SERIALIZERS[dep.serializer] != _lib.SER_FIXED:  # the Kryo stream, decoded on the GPU
            out = self.manager.engine.read_records(sid, self._maps(), self.start, self.end).reshape(-1, 16)
            nrec = len(out)
        else:
            data, _, _, _ = self.read_blocks()
            out = data.reshape(-1, dep.recordBytes)
            nrec = len(out)
        self.readMetrics.incRecordsRead(nrec)
        self.context.mergeShuffleReadMetrics()
        return out

    def iterator(self) -> InterruptibleIterator:
        """read() as Spark's task consumes it: (key, value) pairs of (Long, Long) records (or
        (key, sum) / (key, values) after an aggregator), one at a time, in an
        InterruptibleIterator that stops at the next record once the task is killed, with
        ``incRecordsRead`` per record (spark_3_0/UcxShuffleReader.scala:148-156); behind an
        aggregator, every record it consumed, counted when its first group is handed over."""
        dep = self.handle.dependency
        self.context.killTaskIfInterrupted()
        self._count_blocks()
        if dep.aggregator is not None:
            if dep.recordBytes != 16:
                raise UnsupportedOperationException("aggregation needs (Long, Long) 16 B records")
            agg = _lib.AGG_SUM if dep.aggregator.kind == "sum" else _lib.AGG_GROUP
            res = self.manager.engine.read_grouped(self.handle.shuffleId, self._maps(), self.start, self.end, agg)
            # the aggregator consumed every shuffled record before its first group comes out
            consumed = self.manager.engine.last_read_records()
            if agg == _lib.AGG_SUM:
                pairs = zip(res[0].tolist(), res[1].tolist())
            else:
                keys, starts, vals = res
                ends = list(starts[1:].tolist()) + [len(vals)]
                pairs = ((k, vals[s:e].tolist()) for k, s, e in zip(keys.tolist(), starts.tolist(), ends))
        else:
            out = self.read_raw()
            kv = out.view("<i8").reshape(-1, dep.recordBytes // 8)[:, :2] if dep.recordBytes == 16 else None
            pairs = ((int(a), int(b)) for a, b in kv) if kv is not None else (bytes(r) for r in out)

        def counted():
            if dep.aggregator is not None:
                self.readMetrics.incRecordsRead(consumed)
            for p in pairs:
                if dep.aggregator is None:
                    self.readMetrics.incRecordsRead(1)
                yield p
            self.context.mergeShuffleReadMetrics()

        return InterruptibleIterator(self.context, counted())

    def read_raw(self) -> np.ndarray:
        """The range's records (sorted when the dependency has a key ordering), no metrics."""
        dep = self.handle.dependency
        sid = self.handle.shuffleId
        if dep.keyOrdering:
            return self.manager.engine.read_sorted(sid, self._maps(), self.start, self.end).reshape(-1, dep.recordBytes)
        if _SERIALIZERS[dep.serializer] != _lib.SER_FIXED:
            return self.manager.engine.read_records(sid, self._maps(), self.start, self.end).reshape(-1, 16)
        data, _, _, _ = self.read_blocks()
        return data.reshape(-1, dep.recordBytes)


# ---------------------------------------------------------------------------------------
# The manager
# ---------------------------------------------------------------------------------------
_BYTE_UNITS = {"b": 1, "k": 1 << 10, "kb": 1 << 10, "m": 1 << 20, "mb": 1 << 20, "g": 1 << 30, "gb": 1 << 30,
               "t": 1 << 40, "tb": 1 << 40, "p": 1 << 50, "pb": 1 << 50}
_BYTE_RE = re.compile(r"^\s*([0-9]+)\s*([a-z]*)\s*$")


def byte_string(value: str) -> int:
    """JavaUtils.byteStringAs(value, ByteUnit.BYTE) -- how Spark reads a bytes conf such as
    spark.io.compression.lz4.blockSize: a bare number is bytes, suffixes b/k/kb/m/mb/g/gb/t/tb/
    p/pb (case-insensitive) scale by 1024."""
    m = _BYTE_RE.match(str(value).lower())
    if not m or m.group(2) not in ("",) + tuple(_BYTE_UNITS):
        raise NumberFormatException(f"Size must be specified as bytes (b), kibibytes (k), mebibytes (m), "
                                    f"gibibytes (g), tebibytes (t), or pebibytes(p). E.g. 50b, 100k, or 250m. "
                                    f"Failed to parse byte string: {value}")
    return int(m.group(1)) * (_BYTE_UNITS[m.group(2)] if m.group(2) else 1)


class NumberFormatException(IllegalArgumentException):
    """java.lang.NumberFormatException (an IllegalArgumentException) of byteStringAs."""




class UcxShuffleManager:
    """spark.shuffle.manager=org.apache.spark.shuffle.UcxShuffleManager, MI355X edition."""

    def __init__(self, conf: Optional[Dict[str, str]] = None, isDriver: bool = False, device: int = 0,
                 localDir: Optional[str] = None):
        self.conf = dict(conf or {})
        self.isDriver = isDriver
        self.engine = ShuffleEngine(device=device,
                                    num_chunks=int(self.conf.get("spark.shuffle.ucx.gpu.numChunks", 0)))
        self.ucxTransport = GpuShuffleTransport(self.engine)
        self.shuffleClient = UcxShuffleClient(self.ucxTransport, self.conf)
        root = localDir or self.conf.get("spark.local.dir") or os.path.join(os.getcwd(), "sgx-shuffle")
        self.shuffleBlockResolver = UcxShuffleBlockResolver(self, root)
        self._handles: Dict[int, BaseShuffleHandle] = {}
        self._maps: Dict[int, set] = {}
        self._compressed: set = set()

    def compressed(self, shuffleId: int) -> bool:
        return shuffleId in self._compressed

    def getTransport(self) -> GpuShuffleTransport:
        return self.ucxTransport

    def registerShuffle(self, shuffleId: int, dependency: ShuffleDependency) -> BaseShuffleHandle:
        p = dependency.partitioner
        bounds = getattr(p, "rangeBounds", None)
        self.engine.register_shuffle(shuffleId, p.numPartitions, p.kind, bounds,
                                     getattr(p, "ascending", True), dependency.recordBytes,
                                     _SERIALIZERS[dependency.serializer])
        if dependency.mapSideCombine:
            self.engine.set_map_side_combine(shuffleId, _lib.AGG_SUM)
        h = self._handle_for(shuffleId, dependency)
        # spark.shuffle.compress (Spark 3.0.1's default: true) with spark.io.compression.codec
        # lz4 (the default): applied to Kryo shuffles, whose bytes are Spark's own; the fixed
        # 16 B / 100 B record codec is the engine's own format and stays raw
        if (self.conf.get("spark.shuffle.compress", "true").lower() == "true"
                and _SERIALIZERS[dependency.serializer] == _lib.SER_KRYO):
            codec = self.conf.get("spark.io.compression.codec", "lz4").lower()
            if codec not in ("lz4", "org.apache.spark.io.lz4compressioncodec"):
                raise UnsupportedOperationException(f"compression codec {codec!r}: only lz4 is on the GPU path")
            block = byte_string(self.conf.get("spark.io.compression.lz4.blockSize", "32k"))
            if block > 32 * 1024:
                raise UnsupportedOperationException(
                    f"spark.io.compression.lz4.blockSize {block} B: the GPU codec takes blocks up to 32 KiB")
            self.engine.set_compression(shuffleId, "lz4", block)
            self._compressed.add(shuffleId)
        # UnsafeShuffleWriter merges its spills fast (spark.shuffle.unsafe.fastMergeEnabled,
        # lz4 supports concatenation): each spill's partition segment stays its own stream;
        # the slow merge re-compresses one stream per partition, as SortShuffleWriter writes
        if (isinstance(h, SerializedShuffleHandle)
                and self.conf.get("spark.shuffle.unsafe.fastMergeEnabled", "true").lower() == "true"):
            self.engine.set_map_writer(shuffleId, "unsafe")
        self._handles[shuffleId] = h
        self._maps[shuffleId] = set()
        return h

    def _handle_for(self, shuffleId: int, dep: ShuffleDependency) -> BaseShuffleHandle:
        """SortShuffleManager.registerShuffle (Spark 3.0.1; inherited by the reference,
        shuffle/ucx/CommonUcxShuffleManager.scala:25): bypass if SortShuffleWriter
        .shouldBypassMergeSort, else serialized if SortShuffleManager.canUseSerializedShuffle,
        else the base handle.  The engine's fixed record codec is not a Spark serializer: its
        dependencies get the base handle."""
        R = dep.partitioner.numPartitions
        if not dep.mapSideCombine and R <= int(self.conf.get("spark.shuffle.sort.bypassMergeThreshold", "200")):
            return BypassMergeSortShuffleHandle(shuffleId, dep)
        relocatable = _SERIALIZERS[dep.serializer] == _lib.SER_KRYO  # KryoSerializer (autoReset on)
        if relocatable and not dep.mapSideCombine and R <= (1 << 24):
            return SerializedShuffleHandle(shuffleId, dep)
        return BaseShuffleHandle(shuffleId, dep)

    def getWriter(self, handle: BaseShuffleHandle, mapId: int, context=None, metrics=None) -> GpuShuffleWriter:
        if handle.shuffleId not in self._handles:
            raise IllegalStateException(f"shuffle {handle.shuffleId} is not registered")
        return GpuShuffleWriter(self, handle, mapId)

    def getReader(self, handle: BaseShuffleHandle, startPartition: int, endPartition: int, context=None,
                  metrics=None, mapIds: Optional[Sequence[int]] = None) -> UcxShuffleReader:
        return UcxShuffleReader(self, handle, startPartition, endPartition, mapIds, context, metrics)

    def exchange(self, handle: BaseShuffleHandle, mapId: int):
        """Push a local map output to the reducers' owners over RCCL (collective)."""
        self.engine.exchange(handle.shuffleId, mapId)

    def unregisterShuffle(self, shuffleId: int) -> bool:
        if shuffleId not in self._handles:
            return False
        self.ucxTransport.unregisterShuffle(shuffleId)
        del self._handles[shuffleId]
        self._maps.pop(shuffleId, None)
        self._compressed.discard(shuffleId)
        return True

    def stop(self):
        for s in list(self._handles):
            self.unregisterShuffle(s)
        self.ucxTransport.close()
        self.engine.close()

    # bookkeeping for readers without a MapOutputTracker
    def _map_written(self, shuffleId: int, mapId: int):
        self._maps.setdefault(shuffleId, set()).add(mapId)

    def known_maps(self, shuffleId: int) -> List[int]:
        return sorted(self._maps.get(shuffleId, ()))
