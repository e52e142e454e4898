"""Reads of blocks fetched from another executor (sgx_import_blocks): a reduce task Spark
placed off its reducers' owner takes the raw blocks the owner serves (GpuFetchRemote,
sgx_fetch_blocks) and runs the read on its own GPU -- the reference's "any block from
anywhere" (spark_3_0/UcxShuffleReader.scala:74-103) at GPU speed, instead of Spark's CPU
reader.  Two engines in one process stand for the owner and the reader executor."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("codec", ["fixed", "kryo", "kryo+lz4"])
@pytest.mark.parametrize("where", ["host", "device"])
def test_reads_over_imported_blocks_match_oracle(sgx_lib, oracle_lib, codec, where):
    R, sid = 128, 7
    maps = [11, 12, 13]
    recs = {m: oracle_lib.gen_uniform16(40_000 + 101 * m, 0xF0 + m, value_base=m << 32) for m in maps}
    for m in maps:  # repeated keys, so grouping has work
        recs[m][:, :8] = (recs[m][:, :8].view("<i8") % 9_000).view(np.uint8)
    ser = sgx_lib.SER_FIXED if codec == "fixed" else sgx_lib.SER_KRYO
    with sgx_lib.ShuffleEngine(device=0) as owner, sgx_lib.ShuffleEngine(device=0) as reader:
        for e in (owner, reader):
            e.register_shuffle(sid, R, serializer=ser)
            if codec == "kryo+lz4":
                e.set_compression(sid, "lz4", 4096)
        for m in maps:
            owner.write_map(sid, m, recs[m], len(recs[m]), 16)
        outs = [oracle_lib.map_write(recs[m], R) for m in maps]
        seqs = oracle_lib.canonical_reducer_sequences(outs, R, 16)
        r0, r1 = 20, 77
        # the owner serves the blocks (reducer-major, map-minor), as GpuFetchRemote does
        mids = [m for r in range(r0, r1) for m in maps]
        rids = [r for r in range(r0, r1) for _ in maps]
        data, lens = owner.fetch_blocks(sid, mids, rids)
        if where == "device":
            buf = reader.alloc(max(data.nbytes, 16))
            buf.copy_from(data)
            data = buf
        imp = reader.import_blocks(sid, maps, r0, r1, data, lens)
        got = reader.read_records(sid, maps, r0, r1).reshape(-1, 16)
        assert np.array_equal(got, np.concatenate(seqs[r0:r1]))
        got = reader.read_sorted(sid, maps, r0, r1).reshape(-1, 16)
        assert np.array_equal(got, oracle_lib.reduce_sorted(seqs[r0:r1]))
        k, st, v = reader.read_grouped(sid, maps, r0, r1, sgx_lib.AGG_GROUP)
        wk, wst, wv = oracle_lib.reduce_grouped(seqs[r0:r1], "group")
        assert np.array_equal(k, wk) and np.array_equal(st, wst) and np.array_equal(v, wv)
        k, s = reader.read_grouped(sid, maps, r0, r1, sgx_lib.AGG_SUM)
        wk, ws = oracle_lib.reduce_grouped(seqs[r0:r1], "sum")
        assert np.array_equal(k, wk) and np.array_equal(s, ws)
        # a sub-range and the raw blocks come from the import as well
        got, l2 = reader.fetch_blocks(sid, [12, 11], [30, 30])
        o = [oracle_lib.offsets(c) for _, c in outs]
        if codec == "fixed":
            want = np.concatenate([outs[1][0][o[1][30]:o[1][31]], outs[0][0][o[0][30]:o[0][31]]]).reshape(-1)
            assert np.array_equal(got, want)
        # outside the import nothing is there; after release nothing is
        with pytest.raises(sgx_lib.BlockNotFoundException):
            reader.fetch_blocks(sid, [11], [r1])
        reader.release_import(sid, imp)
        with pytest.raises(sgx_lib.BlockNotFoundException):
            reader.fetch_blocks(sid, [11], [r0])
        with pytest.raises(sgx_lib.BlockNotFoundException):
            reader.release_import(sid, imp)
        if where == "device":
            data.free()


def test_import_argument_checks(sgx_lib):
    with sgx_lib.ShuffleEngine(device=0) as e:
        e.register_shuffle(1, 8)
        with pytest.raises(sgx_lib.IllegalArgumentException):
            e.import_blocks(1, [1, 1], 0, 1, np.zeros(32, np.uint8), [16, 16])  # a map twice
        with pytest.raises(sgx_lib.IllegalArgumentException):
            e.import_blocks(1, [1], 0, 2, np.zeros(32, np.uint8), [16, 8])  # not whole records
        with pytest.raises(sgx_lib.IllegalArgumentException):
            e.import_blocks(1, [1], 4, 9, np.zeros(80, np.uint8), [16] * 5)  # past R
        with pytest.raises(sgx_lib.IllegalStateException):
            e.import_blocks(2, [1], 0, 1, np.zeros(16, np.uint8), [16])  # unknown shuffle
        i = e.import_blocks(1, [5], 0, 8, np.zeros(0, np.uint8), [0] * 8)  # all empty
        data, lens = e.fetch_blocks(1, [5] * 8, list(range(8)))
        assert data.size == 0 and not lens.any()
        e.release_import(1, i)
