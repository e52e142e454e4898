"""Generate the committed golden fixtures under tests/golden/.

The reference (Scala, spark-core 3.0.1 not vendored, no JVM here) cannot be run, and it
ships no tests or fixtures for this path.  These vectors therefore
come from the pure-Python restatement ``oracle/spark_semantics.py`` and are pinned by the
hand-verified known-answer tests of SURVEY.md §8(c), which are written into kats.json
verbatim and re-checked here before anything is emitted.

Run:  python tests/golden/make_golden.py      (deterministic; rewrites the files)
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import spark_semantics as S  # noqa: E402

SEED = 0x5EEDC0DE

# SURVEY.md §8(c) known-answer tests (Java semantics), verbatim.
LONG_HASH_KATS = [
    (0, 0), (1, 1), (-1, 0), (2**32, 1), (-2, 1), (2**63 - 1, -2**31), (-2**63, -2**31),
    (123456789012345, -2045923535),
]
PID_KATS = [  # (key, R, pid)
    (123456789012345, 1024, 817), (2**63 - 1, 1024, 0), (-1, 1024, 0),
    (-123456789012345, 1000, 464), (-1024, 200, 23), (2**31, 200, 152), (-2**31 - 1, 200, 152),
]
NNMOD_KATS = [(-7, 3, 2)]

EDGE_KEYS = [0, 1, -1, 2, -2, 2**31 - 1, 2**31, -2**31, -2**31 - 1, 2**32, 2**32 - 1, -2**32,
             2**63 - 1, -2**63, -2**63 + 1, 0x7FFFFFFF80000000, 0x00000000FFFFFFFF,
             -0x7FFFFFFF, 0x1234567890ABCDEF, -0x1234567890ABCDEF, 123456789012345,
             -123456789012345, 0x80000000, -0x80000001]
EDGE_RS = [1, 2, 3, 7, 200, 1000, 1024, 4096, 65536, 16777216, 2**31 - 1]


def check_kats():
    for k, h in LONG_HASH_KATS:
        assert S.java_long_hash(k) == h, (k, h)
    for k, r, p in PID_KATS:
        assert S.hash_partition(k, r) == p, (k, r, p)
    for x, m, v in NNMOD_KATS:
        assert S.non_negative_mod(x, m) == v


def records_array(recs):
    return np.frombuffer(S.pack_records16(recs), dtype=np.uint8).reshape(-1, 16)


def hash_case(name, recs, R):
    pids, data, lens = S.map_side_shuffle(recs, R)
    np.savez_compressed(
        os.path.join(HERE, f"{name}.npz"),
        records=records_array(recs), num_partitions=np.int32(R), pids=np.array(pids, np.int32),
        out=np.frombuffer(data, np.uint8).reshape(-1, 16) if data else np.zeros((0, 16), np.uint8),
        lengths=np.array(lens, np.int64),
        index=np.frombuffer(S.index_file_bytes(lens), np.uint8))


def range_case(name, keys, bounds, ascending, recs_bytes=None, lt=None):
    """keys: list of python ints (i64) or bytes (10 B)."""
    nb = len(bounds)
    R = nb + 1
    pids = [S.range_partition(k, bounds, ascending, lt) for k in keys]
    if recs_bytes is None:
        recs = [(k, i) for i, k in enumerate(keys)]
        arr = records_array(recs)
        b = np.array(bounds, np.int64)
    else:
        arr = recs_bytes
        b = np.frombuffer(b"".join(bounds), np.uint8).reshape(-1, 10)
    order, counts = S.stable_group_by_partition(pids, R)
    out = arr[np.array(order, dtype=np.int64)] if order else arr[:0]
    rb = arr.shape[1]
    np.savez_compressed(
        os.path.join(HERE, f"{name}.npz"), records=arr, bounds=b, ascending=np.int32(ascending),
        num_partitions=np.int32(R), pids=np.array(pids, np.int32), out=out,
        lengths=np.array([c * rb for c in counts], np.int64))


def terasort_records(n, seed):
    out = bytearray()
    for i in range(n):
        a = S.splitmix64_at(seed, 2 * i).to_bytes(8, "little")
        b = S.splitmix64_at(seed, 2 * i + 1).to_bytes(8, "little")
        out += a + b[:2] + i.to_bytes(8, "little") + bytes(((i + j) & 0xFF) for j in range(18, 100))
    return np.frombuffer(bytes(out), np.uint8).reshape(n, 100)


def main():
    check_kats()
    kats = {
        "long_hash": LONG_HASH_KATS, "hash_pid": PID_KATS, "non_negative_mod": NNMOD_KATS,
        "edge_pids": [[k, r, S.hash_partition(k, r)] for k in EDGE_KEYS for r in EDGE_RS],
        "splitmix64": [[SEED, i, S.splitmix64_at(SEED, i)] for i in range(8)],
        "block_id_bytes": [[m, r, S.ucx_block_id_bytes(m, r).hex()] for m, r in
                           [(0, 0), (1, 2), (-1, 7), (2**31 - 1, 1023)]],
    }
    with open(os.path.join(HERE, "kats.json"), "w") as f:
        json.dump(kats, f, indent=1)

    # Hash partitioner, uniform keys, the three BASELINE reducer counts + ragged sizes.
    for R, n in [(200, 4096), (1024, 5000), (4096, 6000), (1, 100), (3, 1)]:
        hash_case(f"hash_uniform_R{R}_n{n}", S.gen_uniform_records(n, SEED), R)
    hash_case("hash_empty_R1024", [], 1024)
    # Edge keys in map order, repeated (collisions on purpose).
    edge = [(k, i) for i, k in enumerate(EDGE_KEYS * 3)]
    hash_case("hash_edge_R200", edge, 200)
    # Zipf(1.1) skew over a small rank universe (keys = ranks), R = 4096.
    import random
    rnd = random.Random(7)
    ranks = list(range(1, 2**12 + 1))
    w = [r ** -1.1 for r in ranks]
    zkeys = rnd.choices(ranks, weights=w, k=6000)
    hash_case("hash_zipf_R4096", [(k, i) for i, k in enumerate(zkeys)], 4096)

    # RangePartitioner, i64 keys: linear path (<=128 bounds) and binary path, both orders,
    # keys that hit bounds exactly, and a duplicate-bounds array (pins the exact loop).
    rnd = random.Random(11)
    keys = [S.to_i64(S.splitmix64_at(SEED + 1, i)) for i in range(3000)]
    for nb in (50, 1023):
        bounds = sorted(rnd.sample(keys, nb))
        probe = keys + bounds + [b + 1 for b in bounds[:20]] + [b - 1 for b in bounds[:20]]
        for asc in (1, 0):
            range_case(f"range_i64_nb{nb}_asc{asc}", probe, bounds, asc)
    dup = sorted(rnd.choices(keys[:300], k=300))
    range_case("range_i64_dupbounds_nb300", keys[:2000] + dup, dup, 1)
    range_case("range_i64_dupbounds_nb100", keys[:2000] + dup[:100], dup[:100], 1)

    # TeraSort 100 B records, 10 B unsigned keys, sampled bounds (R = 1024 and R = 64).
    ts = terasort_records(3000, SEED)
    tkeys = [bytes(ts[i, :10]) for i in range(ts.shape[0])]
    for nb in (1023, 63):
        sample = sorted(rnd.sample(tkeys, 20 * (nb + 1) if 20 * (nb + 1) < len(tkeys) else len(tkeys)))
        step = len(sample) / (nb + 1)
        bounds = [sample[int(step * (i + 1))] for i in range(nb)]
        range_case(f"range_bytes10_nb{nb}", tkeys, bounds, 1, recs_bytes=ts, lt=S.bytes_lt)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
