"""The reader's task metrics and cancellation (the Python mirror of GpuShuffleReader; the
reference's reader: spark_3_0/UcxShuffleReader.scala:118-123 fetch wait, :148-153 records read
merged on completion, :155-156 / :193-199 InterruptibleIterator).

CPU tests drive UcxShuffleReader against a stand-in engine that serves synthetic blocks; the
GPU test reads real map outputs and checks the counters against the oracle's blocks."""
import numpy as np
import pytest


class _Engine:
    """Block (m, r) = (r + 1) % 4 records {key = m * 1000 + r, value = i} (some blocks empty)."""

    def __init__(self):
        self.calls = []

    def _block(self, m, r):
        n = (r + 1) % 4
        out = np.zeros((n, 2), "<i8")
        out[:, 0] = m * 1000 + r
        out[:, 1] = np.arange(n)
        return out.view(np.uint8).reshape(-1)

    def block_lengths(self, sid, mids, rids):
        self.calls.append("lengths")
        return np.array([len(self._block(m, r)) for m, r in zip(mids, rids)], dtype=np.int64)

    def read_grouped(self, sid, maps, r0, r1, agg):
        """The aggregation of the same blocks: one group per distinct key, summed values."""
        self.calls.append("grouped")
        recs = np.concatenate([self._block(m, r) for r in range(r0, r1) for m in maps]).view("<i8").reshape(-1, 2)
        self._consumed = len(recs)
        keys, inv = np.unique(recs[:, 0], return_inverse=True)
        return keys, np.bincount(inv, weights=recs[:, 1]).astype(np.int64)

    def last_read_records(self):
        return self._consumed

    def fetch_blocks(self, sid, mids, rids):
        self.calls.append("fetch")
        parts = [self._block(m, r) for m, r in zip(mids, rids)]
        lens = np.array([len(p) for p in parts], dtype=np.int64)
        return (np.concatenate(parts) if parts else np.zeros(0, np.uint8)), lens


class _Manager:
    def __init__(self, maps):
        self.engine = _Engine()
        self._maps = maps

    def known_maps(self, sid):
        return sorted(self._maps)

    def compressed(self, sid):
        return False


def _reader(maps, r0, r1, context=None, metrics=None, aggregator=None):
    import sparkucx_amd as sgx

    dep = sgx.ShuffleDependency(sgx.HashPartitioner(8), 16, aggregator=aggregator)
    h = sgx.BaseShuffleHandle(3, dep)
    return sgx.UcxShuffleReader(_Manager(maps), h, r0, r1, None, context, metrics)


def test_read_reports_blocks_bytes_and_records():
    import sparkucx_amd as sgx

    ctx = sgx.TaskContext()
    rd = _reader([5, 9], 0, 8, ctx)
    out = rd.read()
    # blocks: r % 4 != 3 -> records (r + 1) % 4; r = 0..7 -> 1,2,3,0,1,2,3,0 per map
    per_map = [(r + 1) % 4 for r in range(8)]
    assert len(out) == 2 * sum(per_map)
    m = rd.readMetrics
    assert m.localBlocksFetched == 2 * sum(1 for c in per_map if c)
    assert m.localBytesRead == 16 * len(out)
    assert m.recordsRead == len(out)
    assert m.remoteBlocksFetched == 0 and m.remoteBytesRead == 0
    # merged into the task's metrics on completion (mergeShuffleReadMetrics)
    assert ctx.shuffleReadMetrics.recordsRead == len(out)
    assert ctx.shuffleReadMetrics.localBytesRead == m.localBytesRead


def test_aggregated_read_counts_the_shuffled_records():
    """Behind an aggregator the reference counts every shuffled record it consumed, not the
    groups it emits (spark_3_0/UcxShuffleReader.scala:148-162)."""
    import sparkucx_amd as sgx

    want = 2 * sum((r + 1) % 4 for r in range(8))
    rd = _reader([5, 9], 0, 8, sgx.TaskContext(), aggregator=sgx.Aggregator("sum"))
    keys, sums = rd.read()
    assert len(keys) < want
    assert rd.readMetrics.recordsRead == want
    ctx = sgx.TaskContext()
    it = _reader([5, 9], 0, 8, ctx, aggregator=sgx.Aggregator("sum")).iterator()
    groups = list(it)
    assert len(groups) == len(keys)
    assert ctx.shuffleReadMetrics.recordsRead == want


def test_iterator_counts_per_record_and_merges_at_the_end():
    import sparkucx_amd as sgx

    ctx = sgx.TaskContext()
    rd = _reader([1], 0, 4, ctx)
    it = rd.iterator()
    assert isinstance(it, sgx.InterruptibleIterator)
    first = next(it)
    assert first == (1000, 0)
    assert rd.readMetrics.recordsRead == 1
    assert ctx.shuffleReadMetrics.recordsRead == 0  # not merged before completion
    rest = list(it)
    assert 1 + len(rest) == sum((r + 1) % 4 for r in range(4))
    assert rd.readMetrics.recordsRead == 1 + len(rest)
    assert ctx.shuffleReadMetrics.recordsRead == 1 + len(rest)


def test_killed_task_stops_at_the_next_record():
    import sparkucx_amd as sgx

    ctx = sgx.TaskContext()
    rd = _reader([1, 2], 0, 8, ctx)
    it = rd.iterator()
    next(it)
    next(it)
    ctx.markInterrupted("stage cancelled")
    with pytest.raises(sgx.TaskKilledException, match="stage cancelled"):
        next(it)
    assert rd.readMetrics.recordsRead == 2


def test_killed_before_the_read_reads_nothing():
    import sparkucx_amd as sgx

    ctx = sgx.TaskContext()
    ctx.markInterrupted("killed")
    rd = _reader([1], 0, 8, ctx)
    with pytest.raises(sgx.TaskKilledException):
        rd.read()
    assert rd.manager.engine.calls == []
    assert rd.readMetrics.recordsRead == 0


def test_explicit_metrics_reporter_is_the_one_fed():
    import sparkucx_amd as sgx

    m = sgx.ShuffleReadMetricsReporter()
    rd = _reader([4], 2, 6, sgx.TaskContext(), m)
    out = rd.read()
    assert rd.readMetrics is m and m.recordsRead == len(out) and m.localBytesRead == 16 * len(out)


@pytest.mark.gpu
def test_read_metrics_on_the_gpu(sgx_lib, oracle_lib, tmp_path):
    import oracle
    import sparkucx_amd as sgx

    R = 64
    mgr = sgx.UcxShuffleManager(device=0, localDir=str(tmp_path))
    try:
        h = mgr.registerShuffle(0, sgx.ShuffleDependency(sgx.HashPartitioner(R), 16))
        outs = []
        for mid in (3, 7, 11):
            recs = oracle.gen_uniform16(5000 + 113 * mid, 0xAB + mid, value_base=mid << 32)
            w = mgr.getWriter(h, mid)
            w.write(recs)
            outs.append(oracle.map_write(recs, R))
        seqs = oracle.canonical_reducer_sequences(outs, R, 16)
        ctx = sgx.TaskContext()
        rd = mgr.getReader(h, 10, 30, ctx)
        got = rd.read()
        want = np.concatenate(seqs[10:30])
        assert np.array_equal(got, want)
        counts = [o[1] for o in outs]
        assert rd.readMetrics.localBlocksFetched == sum(int(np.count_nonzero(c[10:30])) for c in counts)
        assert rd.readMetrics.localBytesRead == 16 * len(want)
        assert ctx.shuffleReadMetrics.recordsRead == len(want)
        # groupByKey / reduceByKey over the same blocks: the shuffled records, not the groups
        for kind in ("group", "sum"):
            hg = mgr.registerShuffle(1 if kind == "group" else 2, sgx.ShuffleDependency(
                sgx.HashPartitioner(R), 16, aggregator=sgx.Aggregator(kind)))
            for mid, recs in zip((3, 7, 11), [oracle.gen_uniform16(5000 + 113 * m, 0xAB + m, value_base=m << 32)
                                              for m in (3, 7, 11)]):
                mgr.getWriter(hg, mid).write(recs)
            ctxg = sgx.TaskContext()
            res = mgr.getReader(hg, 10, 30, ctxg).read()
            assert len(res[0]) <= len(want)
            assert ctxg.shuffleReadMetrics.recordsRead == len(want)
        # per record, with cancellation
        ctx2 = sgx.TaskContext()
        it = mgr.getReader(h, 0, R, ctx2).iterator()
        k0 = next(it)
        first = np.concatenate(seqs).view("<i8").reshape(-1, 2)[0]
        assert k0 == (int(first[0]), int(first[1]))
        ctx2.markInterrupted("cancelled")
        with pytest.raises(sgx.TaskKilledException):
            next(it)
    finally:
        mgr.stop()
