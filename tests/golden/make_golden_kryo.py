"""Golden fixtures for the Kryo-framed map output.

Spark's KryoSerializer cannot run here (no JVM; spark-core 3.0.1 / kryo-shaded 4.0.2 are
external and absent), so these vectors come from the pure-Python restatement
``oracle/spark_semantics.py`` (kryo_serialize_pairs, map_side_shuffle), pinned by the
hand-computed varlong known answers in kats_kryo.json, which are re-checked here first.

Run:  python tests/golden/make_golden_kryo.py      (deterministic; rewrites the files)
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

# Kryo 4 Output.writeVarLong(v, optimizePositive=false) -- zigzag, 7-bit groups low first,
# the 9th byte whole -- worked by hand; and one record's full frame.
VARLONG_KATS = [
    (0, "00"), (1, "02"), (-1, "01"), (63, "7e"), (-64, "7f"), (64, "8001"), (-65, "8101"),
    (8191, "fe7f"), (8192, "808001"), (2**55 - 1, "feffffffffffff7f"), (2**55, "8080808080808080" + "01"),
    (2**63 - 1, "fe" + "ff" * 8), (-2**63, "ff" * 9),
]
RECORD_KATS = [((1, -1), "09020901"), ((0, 64), "0900098001"), ((-2**63, 0), "09" + "ff" * 9 + "0900")]


def check_kats():
    for v, h in VARLONG_KATS:
        assert S.kryo_write_var_long(v).hex() == h, (v, S.kryo_write_var_long(v).hex(), h)
        assert S.kryo_read_var_long(bytes.fromhex(h), 0) == (v, len(h) // 2)
    for (k, v), h in RECORD_KATS:
        assert S.kryo_serialize_pairs([(k, v)]).hex() == h
        assert S.kryo_deserialize_pairs(bytes.fromhex(h)) == [(k, v)]


def edge_records(n: int, seed: int):
    """Keys/values whose zigzag varlongs take every length 1..9, both signs."""
    recs = S.gen_uniform_records(n, seed)
    out = []
    for i, (k, v) in enumerate(recs):
        sh = i % 64
        kk = S.to_i64(k >> sh) if i % 3 else k
        vv = S.to_i64((v * 0x9E3779B97F4A7C15) >> (i % 64)) * (-1 if i % 2 else 1)
        out.append((kk, S.to_i64(vv)))
    out += [(2**63 - 1, -2**63), (-2**63, 2**63 - 1), (0, 0), (-1, 1), (63, -64), (64, -65)]
    return out


def emit(name, recs, R):
    pids, data16, lengths16 = S.map_side_shuffle(recs, R)
    counts = [L // 16 for L in lengths16]
    order, _ = S.stable_group_by_partition(pids, R)
    ordered = [recs[i] for i in order]
    stream, lengths, pos = bytearray(), [], 0
    for p in range(R):
        part = ordered[pos:pos + counts[p]]
        pos += counts[p]
        b = S.kryo_serialize_pairs(part)
        lengths.append(len(b))
        stream += b
    np.savez_compressed(os.path.join(HERE, name), num_partitions=np.int64(R),
                        records=np.frombuffer(S.pack_records16(recs), dtype=np.uint8).reshape(-1, 16),
                        kryo_lengths=np.array(lengths, dtype=np.int64),
                        kryo_stream=np.frombuffer(bytes(stream), dtype=np.uint8),
                        index=np.frombuffer(S.index_file_bytes(lengths), dtype=np.uint8))


def main():
    check_kats()
    with open(os.path.join(HERE, "kats_kryo.json"), "w") as f:
        json.dump({"varlong": [[v, h] for v, h in VARLONG_KATS],
                   "record": [[list(kv), h] for kv, h in RECORD_KATS]}, f, indent=1)
    emit("kryo_uniform_R200_n3000.npz", S.gen_uniform_records(3000, SEED), 200)
    emit("kryo_edge_R1024_n4100.npz", edge_records(4100, SEED + 1), 1024)
    emit("kryo_edge_R3_n17.npz", edge_records(17, SEED + 2), 3)


if __name__ == "__main__":
    main()
