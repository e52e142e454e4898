"""Thin object wrapper over the C ABI (one ShuffleEngine per GPU = per executor).

Buffers accepted wherever records go in or blocks come out:
  * ``numpy.ndarray`` (host memory)            -> SGX_MEM_HOST
  * ``DeviceBuffer`` (allocated by the engine) -> SGX_MEM_DEVICE
  * any object with ``data_ptr()`` and ``is_cuda`` (a torch tensor on ``cuda:N``)
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Optional, Sequence, Tuple

import numpy as np

from . import _lib
from ._lib import MEM_DEVICE, MEM_HOST, check, lib

LZ4_BLOCK_SIZE = 32 * 1024  # spark.io.compression.lz4.blockSize default (Spark 3.0.1)


class DeviceBuffer:
    """HBM allocation owned by the engine's device (freed by ``free()`` or GC)."""

    def __init__(self, engine: "ShuffleEngine", nbytes: int):
        self.engine = engine
        self.nbytes = int(nbytes)
        p = ctypes.c_void_p()
        check(lib().sgx_device_alloc(engine.handle, self.nbytes, ctypes.byref(p)), "sgx_device_alloc")
        self.ptr = int(p.value)

    def free(self):
        if self.ptr and self.engine.handle:
            check(lib().sgx_device_free(self.engine.handle, self.ptr), "sgx_device_free")
        self.ptr = 0

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass

    def to_numpy(self, nbytes: Optional[int] = None, offset: int = 0) -> np.ndarray:
        n = self.nbytes - offset if nbytes is None else int(nbytes)
        out = np.empty(n, dtype=np.uint8)
        if n:
            check(lib().sgx_memcpy(self.engine.handle, out.ctypes.data, self.ptr + offset, n), "sgx_memcpy")
        return out

    def copy_from(self, arr: np.ndarray, offset: int = 0):
        arr = np.ascontiguousarray(arr)
        if arr.nbytes + offset > self.nbytes:
            raise _lib.IllegalArgumentException("copy_from overflows the device buffer")
        if arr.nbytes:
            check(lib().sgx_memcpy(self.engine.handle, self.ptr + offset, arr.ctypes.data, arr.nbytes), "sgx_memcpy")


def buffer_arg(buf) -> Tuple[int, int, int]:
    """(pointer, nbytes, mem_kind) of a records/destination buffer."""
    if isinstance(buf, DeviceBuffer):
        return buf.ptr, buf.nbytes, MEM_DEVICE
    if isinstance(buf, np.ndarray):
        if not buf.flags["C_CONTIGUOUS"]:
            raise _lib.IllegalArgumentException("host buffers must be C-contiguous")
        return buf.ctypes.data, buf.nbytes, MEM_HOST
    if hasattr(buf, "data_ptr") and getattr(buf, "is_cuda", False):
        if not buf.is_contiguous():
            raise _lib.IllegalArgumentException("device tensors must be contiguous")
        return int(buf.data_ptr()), int(buf.numel() * buf.element_size()), MEM_DEVICE
    raise _lib.IllegalArgumentException(f"unsupported buffer type {type(buf)!r}")


@dataclass
class StageStats:
    ms: dict
    count: dict


class ShuffleEngine:
    """One engine per GPU: owns the HIP streams, work buffers, map outputs in HBM and the
    RCCL communicator (the role CommonUcxShuffleManager.startUcxTransport plays,
    shuffle/ucx/CommonUcxShuffleManager.scala:67-100)."""

    def __init__(self, device: int = 0, num_chunks: int = 0, scatter_waves: int = 0, scatter_items: int = 0,
                 hist_mode: int = _lib.HIST_ATOMIC, rank_mode: int = _lib.RANK_ORDERED, flags: int = 0,
                 comm_timeout_ms: int = 0):
        """sgx_config (include/sgx.h): kernel choices that change speed, never bytes."""
        cfg = (ctypes.c_int32 * 8)(device, num_chunks, scatter_waves, scatter_items, hist_mode, rank_mode, flags,
                                   comm_timeout_ms)
        h = ctypes.c_void_p()
        check(lib().sgx_create(ctypes.cast(cfg, ctypes.c_void_p), ctypes.byref(h)), "sgx_create")
        self.handle = h.value
        self.device = device
        self._host_comm = None

    @property
    def lds_order_ok(self) -> bool:
        """sgx_lds_order_ok: the engine-start check of the lane-ordered LDS atomics the default
        ranking rests on passed on this device (False: every scatter is ballot-ranked)."""
        return lib().sgx_lds_order_ok(self.handle) == 1

    def close(self):
        if self.handle:
            lib().sgx_destroy(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- shuffle registry -------------------------------------------------------------
    def register_shuffle(self, shuffle_id: int, num_partitions: int, kind: int = _lib.PART_HASH,
                         bounds=None, ascending: bool = True, record_bytes: int = 16,
                         serializer: int = _lib.SER_FIXED):
        ptr, nb = None, 0
        keep = None
        if bounds is not None and kind != _lib.PART_HASH:
            if kind == _lib.PART_RANGE_I64:
                keep = np.ascontiguousarray(bounds, dtype=np.int64)
                nb = keep.shape[0]
            else:
                keep = np.ascontiguousarray(bounds, dtype=np.uint8).reshape(-1, 10)
                nb = keep.shape[0]
            ptr = keep.ctypes.data if nb else None
        check(lib().sgx_register_shuffle(self.handle, shuffle_id, num_partitions, kind, ptr, nb,
                                         int(bool(ascending)), record_bytes), "registerShuffle")
        if serializer != _lib.SER_FIXED:
            self.set_serializer(shuffle_id, serializer)

    def set_serializer(self, shuffle_id: int, serializer: int):
        """dep.serializer: SER_FIXED (fixed-width records) or SER_KRYO (Spark's Kryo stream)."""
        check(lib().sgx_set_serializer(self.handle, shuffle_id, serializer), "setSerializer")

    def set_compression(self, shuffle_id: int, codec: str = "lz4", block_size: int = LZ4_BLOCK_SIZE):
        """spark.shuffle.compress / spark.io.compression.codec: "lz4" publishes every map output's
        partition streams LZ4-framed (needs the Kryo serializer); "none" turns it off."""
        codes = {"none": 0, "lz4": 1}
        if codec not in codes:
            raise _lib.IllegalArgumentException(f"unknown codec {codec!r} (none, lz4)")
        check(lib().sgx_set_compression(self.handle, shuffle_id, codes[codec], block_size), "setCompression")

    def set_map_side_combine(self, shuffle_id: int, agg: int = _lib.AGG_SUM):
        """dep.mapSideCombine with a sum aggregator (reduceByKey): map outputs hold one
        {key, sum} combiner per distinct key and partition."""
        check(lib().sgx_set_map_side_combine(self.handle, shuffle_id, agg), "setMapSideCombine")

    def set_map_writer(self, shuffle_id: int, writer: str = "unsafe"):
        """The map writer Spark runs for the shuffle's handle: "sort" (SortShuffleWriter, the
        default: a multi-spill map's partition is one compressed stream) or "unsafe"
        (UnsafeShuffleWriter's fast merge: one LZ4 stream per spill segment, concatenated)."""
        codes = {"sort": _lib.WRITER_SORT, "unsafe": _lib.WRITER_UNSAFE}
        if writer not in codes:
            raise _lib.IllegalArgumentException(f"unknown map writer {writer!r} (sort, unsafe)")
        check(lib().sgx_set_map_writer(self.handle, shuffle_id, codes[writer]), "setMapWriter")

    def set_reducer_placement(self, shuffle_id: int, placement: str = "bytes"):
        """Reducer placement of the shuffle's exchange rounds: "even" (floor(r*P/R), the
        default) or "bytes" (contiguous ranges balancing each rank's received bytes)."""
        codes = {"even": _lib.PLACE_EVEN, "bytes": _lib.PLACE_BYTES}
        if placement not in codes:
            raise _lib.IllegalArgumentException(f"unknown placement {placement!r} (even, bytes)")
        check(lib().sgx_set_reducer_placement(self.handle, shuffle_id, codes[placement]), "setReducerPlacement")

    def shuffle_reducers(self, shuffle_id: int) -> Tuple[int, int]:
        """[r0, r1): the reducers this rank holds for the shuffle (fixed by its first exchange)."""
        r0, r1 = ctypes.c_int32(0), ctypes.c_int32(0)
        check(lib().sgx_shuffle_reducers(self.handle, shuffle_id, ctypes.byref(r0), ctypes.byref(r1)),
              "shuffleReducers")
        return r0.value, r1.value

    def round_reducers(self, shuffle_id: int, map_id: int) -> Tuple[int, int]:
        """[r0, r1): the reducers this rank holds for the exchange round that carried map_id."""
        r0, r1 = ctypes.c_int32(0), ctypes.c_int32(0)
        check(lib().sgx_round_reducers(self.handle, shuffle_id, map_id, ctypes.byref(r0), ctypes.byref(r1)),
              "roundReducers")
        return r0.value, r1.value

    def release_thread(self):
        """Free the calling thread's HIP stream and scratch (recreated on its next call)."""
        check(lib().sgx_release_thread(self.handle), "release_thread")

    def unregister_shuffle(self, shuffle_id: int):
        check(lib().sgx_unregister_shuffle(self.handle, shuffle_id), "unregisterShuffle")

    # -- map side -----------------------------------------------------------------------
    def write_map(self, shuffle_id: int, map_id: int, records, nrecords: int, record_bytes: int,
                  num_partitions: Optional[int] = None) -> Optional[np.ndarray]:
        """Partition + scatter one map batch on the GPU. Returns per-partition byte lengths
        when ``num_partitions`` is given (synchronous), else None (asynchronous)."""
        ptr, nbytes, kind = buffer_arg(records)
        if nrecords * record_bytes > nbytes:
            raise _lib.IllegalArgumentException(
                f"{nrecords} records of {record_bytes} B exceed the {nbytes} B buffer")
        out = None
        out_ptr = None
        if num_partitions is not None:
            out = np.empty(num_partitions, dtype=np.int64)
            out_ptr = out.ctypes.data
        check(lib().sgx_write_map(self.handle, shuffle_id, map_id, ptr, nrecords, record_bytes, kind,
                                  out_ptr), "write_map")
        return out

    def map_begin(self, shuffle_id: int, map_id: int):
        """Open a streaming map output (batches appended with map_append, merged by map_commit)."""
        check(lib().sgx_map_begin(self.handle, shuffle_id, map_id), "map_begin")

    def map_append(self, shuffle_id: int, map_id: int, records, nrecords: int, record_bytes: int,
                   offset: int = 0, retained: bool = False):
        """Append one batch: ``nrecords`` records from byte ``offset`` of ``records``.  A device
        batch with ``retained`` stays where it is (SGX_MEM_DEVICE_RETAINED): the caller keeps it
        unchanged until the map's lengths are known -- map_commit with ``num_partitions`` has
        returned, or map_lengths / sync after an asynchronous commit -- since the commit's
        kernels read it in place; otherwise the engine copies it before returning."""
        ptr, nbytes, kind = buffer_arg(records)
        if offset < 0 or offset + nrecords * record_bytes > nbytes:
            raise _lib.IllegalArgumentException(
                f"{nrecords} records of {record_bytes} B at offset {offset} exceed the {nbytes} B buffer")
        if retained:
            if kind != MEM_DEVICE:
                raise _lib.IllegalArgumentException("only device batches can be retained")
            kind = _lib.MEM_DEVICE_RETAINED
        check(lib().sgx_map_append(self.handle, shuffle_id, map_id, ptr + offset, nrecords, record_bytes, kind),
              "map_append")

    def map_commit(self, shuffle_id: int, map_id: int, num_partitions: Optional[int] = None) -> Optional[np.ndarray]:
        out = None
        if num_partitions is not None:
            out = np.empty(num_partitions, dtype=np.int64)
        check(lib().sgx_map_commit(self.handle, shuffle_id, map_id, out.ctypes.data if out is not None else None),
              "map_commit")
        return out

    def map_lengths(self, shuffle_id: int, map_id: int, num_partitions: int) -> np.ndarray:
        out = np.empty(num_partitions, dtype=np.int64)
        check(lib().sgx_map_lengths(self.handle, shuffle_id, map_id, out.ctypes.data), "map_lengths")
        return out

    def map_data(self, shuffle_id: int, map_id: int) -> Tuple[int, int]:
        p = ctypes.c_void_p()
        n = ctypes.c_int64()
        check(lib().sgx_map_data(self.handle, shuffle_id, map_id, ctypes.byref(p), ctypes.byref(n)), "map_data")
        return int(p.value or 0), int(n.value)

    def map_layout(self, shuffle_id: int, map_id: int) -> int:
        """LAYOUT_PADDED if the map was written in one pass into padded sub-bins, else
        LAYOUT_CONTIGUOUS (two-pass write, or the padded write's overflow fallback);
        LAYOUT_SERIALIZED_PADDED: a Kryo map whose records were written padded (its published
        Kryo stream is contiguous)."""
        v = ctypes.c_int32()
        check(lib().sgx_map_layout(self.handle, shuffle_id, map_id, ctypes.byref(v)), "map_layout")
        return int(v.value)

    def map_output_bytes(self, shuffle_id: int, map_id: int) -> np.ndarray:
        ptr, n = self.map_data(shuffle_id, map_id)
        out = np.empty(n, dtype=np.uint8)
        if n:
            check(lib().sgx_memcpy(self.handle, out.ctypes.data, ptr, n), "sgx_memcpy")
        return out

    def lz4_frame(self, stream_ptr: int, part_offsets, block_size: int = LZ4_BLOCK_SIZE):
        """spark.shuffle.compress=true (lz4): frame the partition streams
        [part_offsets[r], part_offsets[r+1]) of the device bytes at ``stream_ptr`` as lz4-java's
        LZ4BlockOutputStream writes them, on the GPU.  Returns (framed bytes on the host,
        framed lengths int64[R])."""
        offs = np.ascontiguousarray(part_offsets, dtype=np.int64)
        R = len(offs) - 1
        lens = np.empty(R, dtype=np.int64)
        # one compression pass into a bound-sized buffer: a frame is at most its 21-byte header
        # plus the block (RAW when LZ4 does not shrink it), plus a 21-byte end mark per stream
        plen = np.diff(offs)
        nblk = (plen + block_size - 1) // block_size
        bound = int((nblk * (21 + block_size) + np.where(plen > 0, 21, 0)).sum())
        buf = self.alloc(max(bound, 1))
        try:
            check(lib().sgx_lz4_frame_partitions(self.handle, stream_ptr or None, offs.ctypes.data, R, block_size,
                                                  buf.ptr, bound, lens.ctypes.data), "lz4 frame")
            return buf.to_numpy(int(lens.sum())), lens
        finally:
            buf.free()

    def lz4_unframe(self, framed, stream_lens=None) -> np.ndarray:
        """LZ4BlockInputStream on the GPU: ``framed`` (host bytes/ndarray or DeviceBuffer) holds
        LZ4-framed partition streams back to back; returns their decompressed bytes (host).
        ``stream_lens``: the streams' byte lengths when known (parallel per-stream walks)."""
        sl = None if stream_lens is None else np.ascontiguousarray(stream_lens, dtype=np.int64)

        def call(ptr, n, dst, cap, total):
            if sl is None:
                return lib().sgx_lz4_unframe(self.handle, ptr, n, dst, cap, total)
            return lib().sgx_lz4_unframe_streams(self.handle, ptr, sl.ctypes.data, len(sl), dst, cap, total)

        own = None
        if isinstance(framed, DeviceBuffer):
            ptr, n = framed.ptr, framed.nbytes
        else:
            arr = np.frombuffer(bytes(framed), np.uint8) if not isinstance(framed, np.ndarray) else framed
            n = int(arr.nbytes)
            own = self.alloc(max(n, 1))
            if n:
                own.copy_from(np.ascontiguousarray(arr).view(np.uint8).reshape(-1))
            ptr = own.ptr
        try:
            total = ctypes.c_int64()
            check(call(ptr, n, None, 0, ctypes.byref(total)), "lz4 unframe (measure)")
            out = self.alloc(max(total.value, 1))
            try:
                check(call(ptr, n, out.ptr, total.value, ctypes.byref(total)), "lz4 unframe")
                return out.to_numpy(total.value)
            finally:
                out.free()
        finally:
            if own is not None:
                own.free()

    def lz4_frame_map(self, shuffle_id: int, map_id: int, num_partitions: int,
                      block_size: int = LZ4_BLOCK_SIZE):
        """The map output's published partition streams (fixed codec or Kryo) LZ4-framed."""
        lens = self.map_lengths(shuffle_id, map_id, num_partitions)
        ptr, _ = self.map_data(shuffle_id, map_id)
        offs = np.zeros(num_partitions + 1, dtype=np.int64)
        np.cumsum(lens, out=offs[1:])
        return self.lz4_frame(ptr, offs, block_size)

    def write_index(self, shuffle_id: int, map_id: int, index_path: str, data_path: str,
                    num_partitions: int) -> np.ndarray:
        out = np.empty(num_partitions, dtype=np.int64)
        check(lib().sgx_write_index(self.handle, shuffle_id, map_id, index_path.encode(),
                                    data_path.encode(), out.ctypes.data), "writeIndexFileAndCommit")
        return out

    # -- exchange / fetch -----------------------------------------------------------------
    def comm_init(self, nranks: int, rank: int, unique_id: bytes):
        if len(unique_id) != 128:
            raise _lib.IllegalArgumentException("unique id must be 128 bytes")
        buf = ctypes.create_string_buffer(bytes(unique_id), 128)
        check(lib().sgx_comm_init(self.handle, nranks, rank, ctypes.cast(buf, ctypes.c_void_p)), "comm_init")

    def comm_init_host(self, nranks: int, rank: int, collectives=None):
        """Exchange over the host collective backend: ``collectives`` has allgather(bytes) and
        alltoallv(bytes, send_counts, recv_counts) (default: torch.distributed's group)."""
        from .hostcomm import HostCommBinding, TorchDistributedCollectives

        binding = HostCommBinding(collectives if collectives is not None else TorchDistributedCollectives())
        check(lib().sgx_comm_init_host(self.handle, nranks, rank, ctypes.byref(binding.struct)), "comm_init_host")
        self._host_comm = binding  # the callbacks must outlive the engine's use of them

    def exchange(self, shuffle_id: int, map_ids: Optional[Sequence[int]] = None):
        """The shuffle's exchange (collective, every rank calls it): with ``map_ids`` None, every
        committed map output of the shuffle this rank holds that no earlier exchange carried
        (sgx_exchange); otherwise exactly those local maps (sgx_exchange_maps, may be empty)."""
        if map_ids is None:
            check(lib().sgx_exchange(self.handle, shuffle_id), "exchange")
            return
        m = np.ascontiguousarray([int(x) for x in map_ids], dtype=np.int64)
        check(lib().sgx_exchange_maps(self.handle, shuffle_id, m.ctypes.data if len(m) else None, len(m)),
              "exchange")

    def exchange_fail(self, num_partitions: int, code: int = _lib.SGX_ERR_STATE):
        """Join an exchange round this rank cannot take part in, marked failed (sgx_exchange_fail):
        every rank's exchange of the round fails together.  Always raises."""
        check(lib().sgx_exchange_fail(self.handle, num_partitions, code), "exchange_fail")

    def fetch_blocks(self, shuffle_id: int, map_ids: Sequence[int], reduce_ids: Sequence[int], dst=None,
                     dst_cap: Optional[int] = None):
        """Copy blocks back to back into ``dst`` (host ndarray, DeviceBuffer or device tensor).
        With ``dst`` None, a host buffer is sized by a first (length-only) pass.
        Returns (dst, lengths)."""
        m = np.ascontiguousarray(map_ids, dtype=np.int64)
        r = np.ascontiguousarray(reduce_ids, dtype=np.int32)
        lens = np.empty(len(m), dtype=np.int64)
        if dst is None:
            rc = lib().sgx_fetch_blocks(self.handle, shuffle_id, m.ctypes.data, r.ctypes.data, len(m), None, 0,
                                        MEM_HOST, lens.ctypes.data)
            if rc not in (0, _lib.SGX_ERR_INVALID):
                check(rc, "fetchBlocks")
            dst = np.empty(int(lens.sum()), dtype=np.uint8)
        ptr, cap, kind = buffer_arg(dst)
        if dst_cap is not None:
            cap = dst_cap
        check(lib().sgx_fetch_blocks(self.handle, shuffle_id, m.ctypes.data, r.ctypes.data, len(m),
                                     ptr if cap else None, cap, kind, lens.ctypes.data), "fetchBlocks")
        return dst, lens

    def block_lengths(self, shuffle_id: int, map_ids: Sequence[int], reduce_ids: Sequence[int]) -> np.ndarray:
        """Byte length of every block (map_ids[j], reduce_ids[j]) (sgx_fetch_blocks' size query:
        no destination, nothing copied)."""
        m = np.ascontiguousarray(map_ids, dtype=np.int64)
        r = np.ascontiguousarray(reduce_ids, dtype=np.int32)
        lens = np.zeros(len(m), dtype=np.int64)
        if len(m):
            rc = lib().sgx_fetch_blocks(self.handle, shuffle_id, m.ctypes.data, r.ctypes.data, len(m), None, 0,
                                        MEM_HOST, lens.ctypes.data)
            if rc not in (0, _lib.SGX_ERR_INVALID):
                check(rc, "fetchBlocks")
        return lens

    def import_blocks(self, shuffle_id: int, map_ids: Sequence[int], start_partition: int, end_partition: int,
                      data, lengths) -> int:
        """Hand blocks fetched from another executor to this engine (sgx_import_blocks): the
        blocks (map_ids[j], r), r in [start, end), reducer-major then map, back to back in
        ``data`` (host ndarray, DeviceBuffer or device tensor), ``lengths`` in the same order.
        The reads then run over them on this GPU.  Returns the import id (release_import)."""
        m = np.ascontiguousarray([int(x) for x in map_ids], dtype=np.int64)
        lens = np.ascontiguousarray(lengths, dtype=np.int64)
        if len(lens) != len(m) * (end_partition - start_partition):
            raise _lib.IllegalArgumentException("one length per (reducer, map) block")
        ptr, nbytes, kind = buffer_arg(data)
        if int(lens.sum()) > nbytes:
            raise _lib.IllegalArgumentException("lengths exceed the data buffer")
        out = ctypes.c_int64(0)
        check(lib().sgx_import_blocks(self.handle, shuffle_id, m.ctypes.data if len(m) else None, len(m),
                                      start_partition, end_partition, ptr if nbytes else None, kind,
                                      lens.ctypes.data if len(lens) else None, ctypes.byref(out)), "import_blocks")
        return int(out.value)

    def release_import(self, shuffle_id: int, import_id: int):
        check(lib().sgx_release_import(self.handle, shuffle_id, import_id), "release_import")

    def read_sorted(self, shuffle_id: int, map_ids: Sequence[int], start_partition: int, end_partition: int,
                    dst=None) -> np.ndarray:
        """UcxShuffleReader.read with dep.keyOrdering (sortByKey / TeraSort reduce side): the
        canonical blocks of reducers [start, end) x map_ids, each reducer's records sorted
        stably by key, back to back (host ndarray of bytes unless ``dst`` is given)."""
        m = np.ascontiguousarray(map_ids, dtype=np.int64)
        nbytes = ctypes.c_int64(0)
        check(lib().sgx_read_sorted(self.handle, shuffle_id, m.ctypes.data, len(m), start_partition, end_partition,
                                    None, 0, MEM_HOST, ctypes.byref(nbytes)), "readSorted")
        if dst is None:
            dst = np.empty(nbytes.value, dtype=np.uint8)
        ptr, cap, kind = buffer_arg(dst)
        check(lib().sgx_read_sorted(self.handle, shuffle_id, m.ctypes.data, len(m), start_partition, end_partition,
                                    ptr if cap else None, cap, kind, ctypes.byref(nbytes)), "readSorted")
        return dst

    def read_records(self, shuffle_id: int, map_ids: Sequence[int], start_partition: int, end_partition: int,
                     dst=None) -> np.ndarray:
        """UcxShuffleReader.read without aggregator or key ordering: the records of reducers
        [start, end) x map_ids in the canonical order (a Kryo shuffle's stream decoded on the
        GPU), back to back (host ndarray of bytes unless ``dst`` is given)."""
        m = np.ascontiguousarray(map_ids, dtype=np.int64)
        nbytes = ctypes.c_int64(0)
        check(lib().sgx_read_records(self.handle, shuffle_id, m.ctypes.data, len(m), start_partition, end_partition,
                                     None, 0, MEM_HOST, ctypes.byref(nbytes)), "readRecords")
        if dst is None:
            dst = np.empty(nbytes.value, dtype=np.uint8)
        ptr, cap, kind = buffer_arg(dst)
        check(lib().sgx_read_records(self.handle, shuffle_id, m.ctypes.data, len(m), start_partition, end_partition,
                                     ptr if cap else None, cap, kind, ctypes.byref(nbytes)), "readRecords")
        return dst

    def read_grouped(self, shuffle_id: int, map_ids: Sequence[int], start_partition: int, end_partition: int,
                     agg: int = _lib.AGG_GROUP, device: bool = False, out=None):
        """UcxShuffleReader.read with an aggregator on (Long, Long) records.  AGG_GROUP ->
        (keys, group_starts, values); AGG_SUM -> (keys, sums).  Keys ascending per reducer,
        values in canonical arrival order.  Host int64 arrays, or DeviceBuffers of int64 left
        in HBM with ``device=True`` (the caller frees them).  ``out``: host int64 arrays
        (keys, group_starts or None, values) to fill instead of fresh ones -- as the JVM reader
        reuses its direct buffers -- at least as long as the result; the returned arrays are
        views of them.  The size query computes the result and the filling call reuses it (one
        fetch + sort + group per read)."""
        m = np.ascontiguousarray(map_ids, dtype=np.int64)
        ng, nv = ctypes.c_int64(0), ctypes.c_int64(0)
        check(lib().sgx_read_grouped(self.handle, shuffle_id, m.ctypes.data, len(m), start_partition, end_partition,
                                     agg, None, None, None, 0, 0, MEM_HOST, ctypes.byref(ng), ctypes.byref(nv)),
              "readGrouped")
        G, V = ng.value, nv.value
        group = agg == _lib.AGG_GROUP
        if device:
            keys, vals = self.alloc(max(G, 1) * 8), self.alloc(max(V, 1) * 8)
            starts = self.alloc(max(G, 1) * 8) if group else None
            ptrs, kind = (keys.ptr, starts.ptr if group else None, vals.ptr), MEM_DEVICE
        elif out is not None:
            keys, vals = out[0][:G], out[2][:V]
            starts = out[1][:G] if group else None
            for a in (keys, starts, vals):
                if a is not None and (a.dtype != np.int64 or not a.flags["C_CONTIGUOUS"]):
                    raise ValueError("out arrays must be C-contiguous int64")
            if len(keys) < G or len(vals) < V or (group and len(starts) < G):
                raise ValueError("out arrays are shorter than the result")
            ptrs, kind = (keys.ctypes.data, starts.ctypes.data if group else None, vals.ctypes.data), MEM_HOST
        else:
            keys, vals = np.empty(G, dtype=np.int64), np.empty(V, dtype=np.int64)
            starts = np.empty(G, dtype=np.int64) if group else None
            ptrs, kind = (keys.ctypes.data, starts.ctypes.data if group else None, vals.ctypes.data), MEM_HOST
        try:
            check(lib().sgx_read_grouped(self.handle, shuffle_id, m.ctypes.data, len(m), start_partition,
                                         end_partition, agg, ptrs[0], ptrs[1], ptrs[2], G, V, kind,
                                         ctypes.byref(ng), ctypes.byref(nv)), "readGrouped")
        except Exception:
            if device:
                for b in (keys, starts, vals):
                    if b is not None:
                        b.free()
            raise
        if group:
            return keys, starts, vals
        return keys, vals

    def set_overlap_writes(self, on: bool):
        """sgx_set_overlap_writes: consecutive padded writes of a thread on two alternating
        streams (the default) or on one (kernel-alone timings)."""
        check(lib().sgx_set_overlap_writes(self.handle, 1 if on else 0), "set_overlap_writes")

    def last_read_records(self) -> int:
        """Records (before any aggregation) the calling thread's last read_records / read_sorted
        / read_grouped consumed -- what the reference's reader counts with incRecordsRead
        (spark_3_0/UcxShuffleReader.scala:148-162)."""
        n = ctypes.c_int64(0)
        check(lib().sgx_last_read_records(self.handle, ctypes.byref(n)), "lastReadRecords")
        return int(n.value)

    def range_bounds(self, batches: Sequence, nrecords: Sequence[int], record_bytes: int, num_partitions: int,
                     rdd_id: int = 0, sample_points_per_partition: int = 20,
                     parent_rdd_id: Optional[int] = None) -> np.ndarray:
        """RangePartitioner.rangeBounds from the data (sketch on the GPU, Spark's re-sampling of
        imbalanced partitions, determineBounds): int64[nb] for 16 B records, uint8[nb, 10] for
        100 B TeraSort records.  ``batches`` are the RDD's input partitions (all host ndarrays
        or all device buffers); ``rdd_id`` is the id of ``rdd.map(_._1)`` (the sketch's RDD),
        ``parent_rdd_id`` that of the pair RDD (default rdd_id - 1: Spark creates the key RDD
        inside the partitioner's constructor, right after nothing else in the usual case)."""
        parent = rdd_id - 1 if parent_rdd_id is None else parent_rdd_id
        args = [buffer_arg(b) for b in batches]
        kinds = {k for _, _, k in args}
        if len(kinds) > 1:
            raise _lib.IllegalArgumentException("mixed host / device batches")
        ptrs = (ctypes.c_void_p * max(1, len(args)))(*[p for p, _, _ in args])
        ns = np.ascontiguousarray(nrecords, dtype=np.int64)
        kb = 8 if record_bytes == 16 else 10
        out = np.empty(max(1, num_partitions - 1) * kb, dtype=np.uint8)
        nb = ctypes.c_int32(0)
        check(lib().sgx_range_bounds(self.handle, ptrs, ns.ctypes.data, len(args), record_bytes,
                                     kinds.pop() if kinds else MEM_HOST, num_partitions, rdd_id, parent,
                                     sample_points_per_partition, out.ctypes.data, ctypes.byref(nb)), "rangeBounds")
        out = out[:nb.value * kb]
        return out.view("<i8").copy() if kb == 8 else out.reshape(-1, 10).copy()

    def progress(self) -> bool:
        return bool(check(lib().sgx_progress(self.handle), "progress"))

    def sync(self):
        check(lib().sgx_sync(self.handle), "sync")

    def copy_items(self, src: DeviceBuffer, dst: DeviceBuffer, items: np.ndarray, align: int = 16):
        it = np.ascontiguousarray(items, dtype=np.int64).reshape(-1, 3)
        check(lib().sgx_copy_items(self.handle, src.ptr, dst.ptr, it.ctypes.data, it.shape[0], align),
              "copy_items")

    # -- measurement ----------------------------------------------------------------------
    def exchange_bytes(self) -> dict:
        """Bytes the exchange rounds moved since stats_reset: to other ranks, kept, rounds."""
        out = (ctypes.c_int64 * 3)()
        check(lib().sgx_exchange_bytes(self.handle, out), "exchangeBytes")
        return {"sent": int(out[0]), "kept": int(out[1]), "rounds": int(out[2])}

    def stats_reset(self):
        check(lib().sgx_stats_reset(self.handle), "stats_reset")

    def stats(self) -> StageStats:
        ms = np.zeros(len(_lib.STAGES), dtype=np.float64)
        cnt = np.zeros(len(_lib.STAGES), dtype=np.int64)
        check(lib().sgx_stats_get(self.handle, ms.ctypes.data, cnt.ctypes.data), "stats_get")
        return StageStats(dict(zip(_lib.STAGES, ms.tolist())), dict(zip(_lib.STAGES, cnt.tolist())))

    # -- synthetic inputs ------------------------------------------------------------------
    def alloc(self, nbytes: int) -> DeviceBuffer:
        return DeviceBuffer(self, nbytes)

    def gen_uniform16(self, buf: DeviceBuffer, n: int, seed: int, value_base: int = 0):
        check(lib().sgx_gen_uniform16(self.handle, buf.ptr, n, seed & (2**64 - 1), value_base), "gen_uniform16")

    def gen_zipf16(self, buf: DeviceBuffer, n: int, seed: int, cdf: np.ndarray, value_base: int = 0):
        cdf = np.ascontiguousarray(cdf, dtype=np.float64)
        check(lib().sgx_gen_zipf16(self.handle, buf.ptr, n, seed & (2**64 - 1), value_base, cdf.ctypes.data,
                                   len(cdf)), "gen_zipf16")

    def gen_terasort100(self, buf: DeviceBuffer, n: int, seed: int, index_base: int = 0):
        check(lib().sgx_gen_terasort100(self.handle, buf.ptr, n, seed & (2**64 - 1), index_base),
              "gen_terasort100")


def bootstrap_serve(port: int, nranks: int, unique_id: bytes, timeout_ms: int = 60_000):
    """Driver side of the id exchange (replaces ExecutorAdded / IntroduceAllExecutors):
    blocks until ranks 1..nranks-1 fetched ``unique_id`` (128 bytes)."""
    buf = (ctypes.c_uint8 * 128).from_buffer_copy(bytes(unique_id).ljust(128, b"\0")[:128])
    check(lib().sgx_bootstrap_serve(port, nranks, ctypes.cast(buf, ctypes.c_void_p), timeout_ms), "bootstrapServe")


def bootstrap_join(host: str, port: int, rank: int, timeout_ms: int = 60_000) -> Tuple[bytes, int]:
    """Executor side: fetch (unique_id, nranks) from the serving rank."""
    buf = (ctypes.c_uint8 * 128)()
    nr = ctypes.c_int32(0)
    check(lib().sgx_bootstrap_join(host.encode(), port, rank, timeout_ms, ctypes.cast(buf, ctypes.c_void_p),
                                   ctypes.byref(nr)), "bootstrapJoin")
    return bytes(buf), nr.value


def get_unique_id() -> bytes:
    buf = ctypes.create_string_buffer(128)
    check(lib().sgx_get_unique_id(ctypes.cast(buf, ctypes.c_void_p)), "get_unique_id")
    return buf.raw


def plan_exchange(lengths_all: np.ndarray, rank: int, item_bytes: int = 0, bounds=None):
    """Pure-host exchange plan (no GPU): returns (send_counts, send_displs, recv_counts,
    recv_displs, items[n,3]).  bounds: the P + 1 reducer-range bounds (default: the even
    placement, floor(r*P/R))."""
    L = np.ascontiguousarray(lengths_all, dtype=np.int64)
    P, R = L.shape
    b = even_ranges(P, R) if bounds is None else np.ascontiguousarray(bounds, dtype=np.int32)
    sc, sd, rc, rd = (np.zeros(P, np.int64) for _ in range(4))
    n = ctypes.c_int64(0)

    def call(items, cnt):
        check(lib().sgx_plan_exchange_ranges(L.ctypes.data, P, R, rank, b.ctypes.data, item_bytes, sc.ctypes.data,
                                             sd.ctypes.data, rc.ctypes.data, rd.ctypes.data, items, ctypes.byref(cnt)),
              "plan_exchange")

    call(None, n)
    items = np.zeros((max(n.value, 1), 3), np.int64)
    call(items.ctypes.data, ctypes.c_int64(n.value))
    return sc, sd, rc, rd, items[: n.value]


def plan_exchange_maps(lengths_all: np.ndarray, maps_per_rank, rank: int, bounds=None):
    """Pure-host plan of the per-shuffle exchange (sgx_plan_exchange_maps): ``lengths_all``
    [M][R] of every rank's maps, source-rank-major, ``maps_per_rank`` [P].  Returns
    (send_counts, send_displs, recv_counts, recv_displs, block_off[M][nmine])."""
    L = np.ascontiguousarray(lengths_all, dtype=np.int64)
    cnt = np.ascontiguousarray(maps_per_rank, dtype=np.int64)
    P = len(cnt)
    R = L.shape[1]  # lengths_all is [M][R], M may be 0
    b = even_ranges(P, R) if bounds is None else np.ascontiguousarray(bounds, dtype=np.int32)
    nmine = int(b[rank + 1] - b[rank])
    sc, sd, rc, rd = (np.zeros(P, np.int64) for _ in range(4))
    bo = np.zeros((max(len(L), 1), max(nmine, 1)), np.int64)
    check(lib().sgx_plan_exchange_maps(L.ctypes.data if L.size else None, cnt.ctypes.data, P, R, rank, b.ctypes.data,
                                       sc.ctypes.data, sd.ctypes.data, rc.ctypes.data, rd.ctypes.data, bo.ctypes.data),
          "plan_exchange_maps")
    return sc, sd, rc, rd, bo[: len(L), :nmine]


def even_ranges(P: int, R: int) -> np.ndarray:
    """Bounds [P + 1] of the even placement: rank j holds [b[j], b[j + 1])."""
    b = np.zeros(P + 1, np.int32)
    check(lib().sgx_even_ranges(P, R, b.ctypes.data), "even_ranges")
    return b


def balanced_ranges(lengths_all: np.ndarray) -> np.ndarray:
    """Bounds [P + 1] of the byte-balanced placement over [P][R] lengths (sgx_balanced_ranges)."""
    L = np.ascontiguousarray(lengths_all, dtype=np.int64)
    P, R = L.shape
    b = np.zeros(P + 1, np.int32)
    check(lib().sgx_balanced_ranges(L.ctypes.data, P, R, b.ctypes.data), "balanced_ranges")
    return b


def reducer_owner(reduce_id: int, num_partitions: int, nranks: int) -> int:
    return int(lib().sgx_reducer_owner(reduce_id, num_partitions, nranks))
