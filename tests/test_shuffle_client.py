"""CPU tests of the fetchBlocks request split (no GPU: the engine is a stand-in that serves
synthetic blocks).  The reference's UcxShuffleClient.fetchBlocks halves a request while it
holds more than maxBlocksPerRequest ids (spark_3_0/UcxShuffleClient.scala:53-58:
``blockIds.splitAt(blockIds.length / 2)`` then both halves recursively), so 130 ids under the
default 50 go out as 32 / 33 / 32 / 33."""
import numpy as np
import pytest


class _Engine:
    """Serves block (s, m, r) as (m * 1000 + r) % 251 repeated r % 7 + 1 times."""

    def __init__(self):
        self.calls = []

    def fetch_blocks(self, sid, mids, rids):
        self.calls.append(len(mids))
        parts = [np.full(r % 7 + 1, (m * 1000 + r) % 251, np.uint8) for m, r in zip(mids, rids)]
        lens = np.array([len(p) for p in parts], dtype=np.int64)
        return (np.concatenate(parts) if parts else np.zeros(0, np.uint8)), lens


class _Transport:
    def __init__(self):
        self.engine = _Engine()


def reference_split(ids, limit):
    """splitAt(length / 2) recursion of UcxShuffleClient.fetchBlocks: the request sizes."""
    if len(ids) > limit:
        h = len(ids) // 2
        return reference_split(ids[:h], limit) + reference_split(ids[h:], limit)
    return [len(ids)] if ids else []


@pytest.mark.parametrize("n,limit", [(130, 50), (50, 50), (51, 50), (1, 50), (0, 50), (1000, 7), (257, 1)])
def test_fetch_blocks_recursive_halving(n, limit):
    from sparkucx_amd.shuffle import BlockFetchingListener, UcxShuffleClient

    client = UcxShuffleClient(_Transport(), {"spark.shuffle.ucx.maxBlocksPerRequest": str(limit)})
    ids = [f"shuffle_4_{i % 3}_{i}" for i in range(n)]

    class L(BlockFetchingListener):
        def __init__(self):
            self.ok = {}

        def onBlockFetchSuccess(self, blockId, data):
            self.ok[blockId] = bytes(data)

    lst = L()
    client.fetchBlocks("h", 1, "1", ids, lst)
    assert client.request_sizes == reference_split(ids, limit)
    assert all(s <= limit for s in client.request_sizes)
    if (n, limit) == (130, 50):
        assert client.request_sizes == [32, 33, 32, 33]
    assert len(lst.ok) == n
    for i, b in enumerate(ids):
        m, r = i % 3, i
        assert lst.ok[b] == bytes([(m * 1000 + r) % 251]) * (r % 7 + 1)
