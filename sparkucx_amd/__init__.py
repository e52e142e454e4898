"""sparkucx_amd — MI355X-native shuffle engine behind SparkUCX's UcxShuffleManager API.

The data path (partition ids, histogram, decoupled-look-back scan, stable scatter,
RCCL all-to-all exchange, regroup) runs in the in-tree HIP library ``libsgx.so``
(include/sgx.h).  This package is the host-side mirror of the plugin interface; it has no
CPU fallback and raises if the library is missing.
"""
from ._lib import (  # noqa: F401
    AGG_GROUP, AGG_SUM, FLAG_ASSUME_LDS_DISORDER, FLAG_DEBUG_SYNC, FLAG_LZ4_LANE_DECODE, FLAG_NO_BUCKET_SORT, FLAG_NO_SPLIT_SCATTER, FLAG_NO_WIDE_STAGED, FLAG_NO_WRITE_COMBINING,
    FLAG_SORT_ALL_DIGITS, FLAG_NO_PADDED_MAP, FLAG_PAD_ANY_SIZE, FLAG_NO_SEG_WINDOW, FLAG_NO_DEFERRED_APPEND, FLAG_NO_P2P_EXCHANGE, FLAG_NO_OVERLAP_WRITES, FLAG_TEST_P2P_UNAVAILABLE, HIST_ATOMIC, LAYOUT_CONTIGUOUS, LAYOUT_PADDED, LAYOUT_SERIALIZED_PADDED,
    HIST_BALLOT, MEM_DEVICE, MEM_DEVICE_RETAINED, MEM_HOST, PART_HASH, PART_RANGE_BYTES10, PART_RANGE_I64, PLACE_BYTES, PLACE_EVEN,
    RANK_MATCH, RANK_ORDERED,
    SER_FIXED, SER_KRYO, STAGES, WRITER_SORT, WRITER_UNSAFE,
    BlockNotFoundException, DeviceError, IllegalArgumentException, IllegalStateException,
    ShuffleError, ShuffleIOException, TransportError, UnsupportedOperationException, lib,
)
from .engine import (  # noqa: F401
    DeviceBuffer, ShuffleEngine, balanced_ranges, bootstrap_join, bootstrap_serve, even_ranges, get_unique_id,
    plan_exchange, plan_exchange_maps, reducer_owner,
)
from .shuffle import (  # noqa: F401
    Aggregator, BaseShuffleHandle, BlockFetchingListener, BypassMergeSortShuffleHandle, SerializedShuffleHandle, GpuShuffleMapOutputWriter, GpuShuffleTransport, GpuShuffleWriter,
    HashPartitioner, InterruptibleIterator, MapStatus, MemoryBlock, MemoryPool, OperationResult, OperationStatus,
    RangePartitioner, ShuffleDependency, ShuffleReadMetricsReporter, TaskContext, TaskKilledException, UcxShuffleBlockId, UcxShuffleBlockResolver, UcxShuffleManager,
    UcxShuffleClient, UcxShuffleReader, byte_string, parse_block_id,
)

__all__ = [n for n in dir() if not n.startswith("_")]
