"""Three engine capabilities the reference's writer has and a one-shot, one-thread engine
would not:

* concurrent map tasks: an executor runs one map task per core, and the reference routes
  each calling thread to its own worker (ucx/UcxShuffleTransport.scala:277-296).  Here every
  calling thread gets its own HIP stream and scratch; 8 threads write 8 maps on ONE engine
  (and read while others write), bit-exact against the oracle.
* streaming map outputs: the reference's writer receives unbounded partition streams, merged
  across spills in spill order (ucx/NvkvShuffleMapOutputWriter.scala:106-113,228-246):
  sgx_map_begin / _append / _commit must equal sgx_write_map of the concatenation.
* map-side combine (reduceByKey's default, mapSideCombine = true; read back with
  combineCombinersByKey, spark_3_0/UcxShuffleReader.scala:158-161).
"""
import threading

import numpy as np
import pytest

from oracle import spark_semantics as ss


# ---------------------------------------------------------------- CPU: the oracle itself
def test_combine_oracle_matches_pure_python_restatement(oracle_lib):
    rng = np.random.default_rng(7)
    for R, n, distinct in [(1, 50, 5), (7, 400, 30), (200, 3000, 900), (16, 2000, 2000)]:
        keys = rng.integers(-(1 << 62), 1 << 62, size=distinct)[rng.integers(0, distinct, size=n)]
        keys[: min(3, n)] = [-1, 1 << 32, -(1 << 63)][: min(3, n)]
        vals = rng.integers(-(1 << 63), (1 << 63) - 1, size=n, dtype=np.int64)
        recs = np.empty((n, 16), np.uint8)
        recs[:, :8] = keys.astype(np.int64).view(np.uint8).reshape(-1, 8)
        recs[:, 8:] = vals.view(np.uint8).reshape(-1, 8)
        out, counts = oracle_lib.map_combine_sum(recs, R)
        want = ss.map_side_combine_sum(list(zip(keys.tolist(), vals.tolist())), R)
        got = list(zip(out[:, :8].copy().view("<i8").ravel().tolist(), out[:, 8:].copy().view("<i8").ravel().tolist()))
        assert got == want
        assert counts.sum() == len(want)
        pids = [ss.hash_partition(k, R) for k, _ in want]
        assert np.array_equal(np.bincount(pids, minlength=R), counts)


# ---------------------------------------------------------------- GPU
def _check_map(engine, oracle_lib, sid, mid, recs, R):
    want_out, want_counts = oracle_lib.map_write(recs, R)
    lengths = engine.map_lengths(sid, mid, R)
    assert np.array_equal(lengths, want_counts * 16)
    assert np.array_equal(engine.map_output_bytes(sid, mid).reshape(-1, 16), want_out)


@pytest.mark.gpu
def test_eight_threads_write_eight_maps_on_one_engine(sgx_lib, oracle_lib):
    R, T = 1024, 8
    recs = [oracle_lib.gen_uniform16(400_000 + 977 * t, 0x7000 + t, value_base=t << 40) for t in range(T)]
    with sgx_lib.ShuffleEngine(device=0) as e:
        e.register_shuffle(1, R)
        errors = []
        barrier = threading.Barrier(T)

        def task(t):
            try:
                barrier.wait()
                for rep in range(3):  # re-attempts of the same map reuse its slot
                    dev = e.alloc(recs[t].nbytes)
                    dev.copy_from(recs[t])
                    e.write_map(1, t, dev, len(recs[t]), 16, R if rep == 2 else None)
                    dev.free()
                e.release_thread()
            except Exception as ex:  # noqa: BLE001
                errors.append(ex)

        threads = [threading.Thread(target=task, args=(t,)) for t in range(T)]
        for th in threads:
            th.start()
        for th in threads:
            th.join(timeout=120)
        assert not errors, errors
        e.sync()
        for t in range(T):
            _check_map(e, oracle_lib, 1, t, recs[t], R)


@pytest.mark.gpu
def test_concurrent_readers_and_writers(sgx_lib, oracle_lib):
    """Threads fetch and read sorted blocks of finished maps while other threads write new
    maps of the same shuffle (Kryo framing on, so the writers run several kernels)."""
    R = 200
    base = [oracle_lib.gen_uniform16(150_000 + 31 * m, 0x8100 + m, value_base=m << 40) for m in range(4)]
    more = [oracle_lib.gen_uniform16(120_000 + 17 * m, 0x8200 + m, value_base=(m + 4) << 40) for m in range(4)]
    with sgx_lib.ShuffleEngine(device=0) as e:
        e.register_shuffle(2, R, serializer=sgx_lib.SER_KRYO)
        for m, r in enumerate(base):
            e.write_map(2, m, r, len(r), 16, R)
        outs = [oracle_lib.map_write(r, R) for r in base]
        seqs = oracle_lib.canonical_reducer_sequences(outs, R, 16)
        errors = []

        def reader(i):
            try:
                for _ in range(3):
                    r0 = (37 * i) % (R - 10)
                    got = e.read_records(2, [0, 1, 2, 3], r0, r0 + 10).reshape(-1, 16)
                    assert np.array_equal(got, np.concatenate(seqs[r0:r0 + 10]))
                    got = e.read_sorted(2, [0, 1, 2, 3], r0, r0 + 10).reshape(-1, 16)
                    assert np.array_equal(got, oracle_lib.reduce_sorted(seqs[r0:r0 + 10]))
            except Exception as ex:  # noqa: BLE001
                errors.append(ex)

        def writer(m):
            try:
                e.write_map(2, 4 + m, more[m], len(more[m]), 16, R)
            except Exception as ex:  # noqa: BLE001
                errors.append(ex)

        threads = [threading.Thread(target=reader, args=(i,)) for i in range(4)]
        threads += [threading.Thread(target=writer, args=(m,)) for m in range(4)]
        for th in threads:
            th.start()
        for th in threads:
            th.join(timeout=180)
        assert not errors, errors
        for m in range(4):
            out, counts = oracle_lib.map_write(more[m], R)
            want = np.diff(oracle_lib.kryo_partition_offsets(out, counts))
            assert np.array_equal(e.map_lengths(2, 4 + m, R), want)
            assert np.array_equal(e.map_output_bytes(2, 4 + m), oracle_lib.kryo_serialize(out))


@pytest.mark.gpu
@pytest.mark.parametrize("codec", ["fixed", "kryo", "kryo+lz4"])
@pytest.mark.parametrize("R", [1, 200, 1024, 4096])
def test_streaming_map_equals_one_batch(sgx_lib, oracle_lib, codec, R):
    sizes = [0, 1, 70_001, 8192, 250_000, 3]
    recs = oracle_lib.gen_uniform16(sum(sizes), 0x5500 + R)
    with sgx_lib.ShuffleEngine(device=0) as e:
        for sid in (1, 2):
            e.register_shuffle(sid, R, serializer=sgx_lib.SER_FIXED if codec == "fixed" else sgx_lib.SER_KRYO)
            if codec == "kryo+lz4":
                e.set_compression(sid, "lz4", 32768)
        one = e.write_map(1, 0, recs, len(recs), 16, R)
        e.map_begin(2, 0)
        pos = 0
        for k, sz in enumerate(sizes):
            part = recs[pos:pos + sz]
            if k % 2:  # device and host batches
                dev = e.alloc(max(part.nbytes, 16))
                dev.copy_from(part)
                e.map_append(2, 0, dev, sz, 16)
                dev.free()
            else:
                e.map_append(2, 0, np.ascontiguousarray(part), sz, 16)
            pos += sz
        many = e.map_commit(2, 0, R)
        assert np.array_equal(one, many)
        assert np.array_equal(e.map_output_bytes(1, 0), e.map_output_bytes(2, 0))
        if codec == "fixed":
            _check_map(e, oracle_lib, 2, 0, recs, R)
        # an open map cannot be read; a committed one can be rewritten in one batch
        e.map_begin(2, 1)
        with pytest.raises(sgx_lib.IllegalStateException):
            e.fetch_blocks(2, [1], [0])
        e.map_commit(2, 1, R)
        with pytest.raises(sgx_lib.IllegalStateException):
            e.map_append(2, 1, recs[:5], 5, 16)


@pytest.mark.gpu
@pytest.mark.parametrize("R", [1, 3, 200, 1024])
@pytest.mark.parametrize("block", [32768, 64])
def test_unsafe_writer_fast_merge_framing(sgx_lib, oracle_lib, R, block):
    """UnsafeShuffleWriter (SerializedShuffleHandle, spark_3_0/UcxShuffleManager.scala:37-45)
    on a compressed Kryo shuffle: every spill's partition segment is its own LZ4 stream and a
    partition concatenates them in spill order (mergeSpillsWithTransferTo's fast merge).
    Lengths, published bytes and fetched blocks equal the restatement; one spill equals the
    SortShuffleWriter output; the readers decode the concatenated streams."""
    sizes = [70_001, 0, 1, 8192, 30_000, 3] if block == 32768 else [700, 0, 1, 90, 300, 3]
    recs = oracle_lib.gen_uniform16(sum(sizes), 0x6600 + R)
    spills, pos = [], 0
    for sz in sizes:
        spills.append(recs[pos:pos + sz])
        pos += sz
    want, want_len = oracle_lib.unsafe_writer_map_output(spills, R, block_size=block)
    with sgx_lib.ShuffleEngine(device=0) as e:
        for sid, writer in ((1, "unsafe"), (2, "sort"), (3, "unsafe")):
            e.register_shuffle(sid, R, serializer=sgx_lib.SER_KRYO)
            e.set_compression(sid, "lz4", block)
            e.set_map_writer(sid, writer)
        for sid in (1, 2):
            e.map_begin(sid, 0)
            for k, part in enumerate(spills):
                e.map_append(sid, 0, np.ascontiguousarray(part), len(part), 16)
            lengths = e.map_commit(sid, 0, R)
            if sid == 1:
                assert np.array_equal(lengths, want_len)
                assert np.array_equal(e.map_output_bytes(1, 0), want)
        # several spills: the two writers' bytes differ, their records do not
        assert not np.array_equal(e.map_output_bytes(1, 0), e.map_output_bytes(2, 0))
        seqs = oracle_lib.canonical_reducer_sequences([oracle_lib.map_write(recs, R)], R, 16)
        for r0, r1 in ((0, R), (R // 2, R)):
            got = e.read_records(1, [0], r0, r1).reshape(-1, 16)
            assert np.array_equal(got, np.concatenate(seqs[r0:r1]))
            assert np.array_equal(e.read_sorted(1, [0], r0, r1).reshape(-1, 16), oracle_lib.reduce_sorted(seqs[r0:r1]))
        # every block is the partition's concatenated streams
        off = np.concatenate([[0], np.cumsum(want_len)])
        for r in {0, R // 2, R - 1}:
            host, lens = e.fetch_blocks(1, [0], [r])
            assert np.array_equal(host[:lens[0]], want[off[r]:off[r + 1]])
        # one spill: UnsafeShuffleWriter writes what SortShuffleWriter writes
        e.write_map(3, 0, recs, len(recs), 16, R)
        one_len = e.map_lengths(3, 0, R)
        e.map_begin(3, 1)
        e.map_append(3, 1, recs, len(recs), 16)
        assert np.array_equal(e.map_commit(3, 1, R), one_len)
        assert np.array_equal(e.map_output_bytes(3, 1), e.map_output_bytes(3, 0))
        # Spark never gives a combining dependency a SerializedShuffleHandle
        e.register_shuffle(4, R, serializer=sgx_lib.SER_KRYO)
        e.set_map_side_combine(4)
        with pytest.raises(sgx_lib.IllegalStateException):
            e.set_map_writer(4, "unsafe")
        with pytest.raises(sgx_lib.IllegalStateException):
            e.set_map_side_combine(1)  # shuffle 1 already has map outputs


@pytest.mark.gpu
@pytest.mark.parametrize("codec", ["fixed", "kryo", "kryo+lz4"])
@pytest.mark.parametrize("R,n,distinct", [(1, 10_000, 50), (200, 300_000, 20_000), (1024, 500_000, 3_000_000),
                                          (4096, 200_000, 700)])
def test_map_side_combine_sum(sgx_lib, oracle_lib, codec, R, n, distinct):
    """reduceByKey with mapSideCombine = true: each map output holds one {key, sum} record per
    (partition, distinct key), keys ascending (oracle.map_combine_sum); the reduce side sums
    the combiners (combineCombinersByKey) to the same result as summing the raw records."""
    rng = np.random.default_rng(n + R)
    maps = []
    for m in range(3):
        keys = rng.integers(-(1 << 62), 1 << 62, size=distinct)[rng.integers(0, distinct, size=n + m)]
        recs = np.empty((n + m, 16), np.uint8)
        recs[:, :8] = keys.astype(np.int64).view(np.uint8).reshape(-1, 8)
        recs[:, 8:] = rng.integers(-(1 << 63), (1 << 63) - 1, size=n + m, dtype=np.int64).view(np.uint8).reshape(-1, 8)
        maps.append(recs)
    mgr = sgx_lib.UcxShuffleManager(conf={"spark.shuffle.compress": "true" if codec == "kryo+lz4" else "false"})
    try:
        dep = sgx_lib.ShuffleDependency(sgx_lib.HashPartitioner(R), 16, aggregator=sgx_lib.Aggregator("sum"),
                                        mapSideCombine=True, serializer="fixed" if codec == "fixed" else "kryo")
        h = mgr.registerShuffle(9, dep)
        combined = []
        for m, recs in enumerate(maps):
            w = mgr.getWriter(h, m)
            w.write(recs)
            out, counts = oracle_lib.map_combine_sum(recs, R)
            combined.append((out, counts))
            if codec == "fixed":
                assert np.array_equal(w.getPartitionLengths(), counts * 16)
                assert np.array_equal(mgr.engine.map_output_bytes(9, m).reshape(-1, 16), out)
            else:
                kryo = oracle_lib.kryo_serialize(out)
                koff = oracle_lib.kryo_partition_offsets(out, counts)
                if codec == "kryo":
                    assert np.array_equal(w.getPartitionLengths(), np.diff(koff))
                    assert np.array_equal(mgr.engine.map_output_bytes(9, m), kryo)
                else:
                    frames, flen = oracle_lib.lz4_frame_partitions(kryo, koff)
                    assert np.array_equal(w.getPartitionLengths(), flen)
                    assert np.array_equal(mgr.engine.map_output_bytes(9, m), frames)
        keys, sums = mgr.getReader(h, 0, R).read()
        raw = oracle_lib.canonical_reducer_sequences([oracle_lib.map_write(r, R) for r in maps], R, 16)
        wk, ws = oracle_lib.reduce_grouped(raw, "sum")
        assert np.array_equal(keys, wk) and np.array_equal(sums, ws)
    finally:
        mgr.stop()


@pytest.mark.gpu
def test_map_side_combine_errors(sgx_lib):
    with pytest.raises(sgx_lib.IllegalArgumentException):
        sgx_lib.ShuffleDependency(sgx_lib.HashPartitioner(4), mapSideCombine=True)
    with pytest.raises(sgx_lib.UnsupportedOperationException):
        sgx_lib.ShuffleDependency(sgx_lib.HashPartitioner(4), aggregator=sgx_lib.Aggregator("group"),
                                  mapSideCombine=True)
    with sgx_lib.ShuffleEngine(device=0) as e:
        e.register_shuffle(1, 8)
        e.set_map_side_combine(1)
        e.write_map(1, 0, np.zeros((10, 16), np.uint8), 10, 16, 8)
        with pytest.raises(sgx_lib.IllegalStateException):
            e.set_map_side_combine(1)
        with pytest.raises(sgx_lib.UnsupportedOperationException):
            e.read_grouped(1, [0], 0, 8, sgx_lib.AGG_GROUP)
