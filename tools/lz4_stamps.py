#!/usr/bin/env python3
"""Phase shares of the LZ4 batch compressor (sgx_lz4.hip lz4_compress_batch), from a stamp build:
    bash tools/build_variant.sh lz4st - -DSGX_LZ4_STAMPS
    python tools/ab_run.py tools/ab/libsgx_lz4st.so lz4_stamps [--records N] [--case c1|lowentropy|uniform]
Frames a Kryo map output (C1's stream: values 2^27 + i, or the low-entropy / uniform streams of
tools/prof_lz4.py) and prints one JSON line: s_memtime cycles per block in each phase and
their shares.  The build's own run time is not a measurement (the stamps' waits change it)."""
import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PHASES = ["probe_wait", "hash_table_read", "same_hash_ballots", "candidate_bytes_wait", "search_in_batch",
          "hit_catchup_count", "emit", "test_in_batch", "test_past_batch", "batch_end"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=1 << 24)
    ap.add_argument("--partitions", type=int, default=1024)
    ap.add_argument("--case", default="c1", choices=["c1", "lowentropy", "uniform"])
    a = ap.parse_args()
    import numpy as np

    import oracle
    import sparkucx_amd as sgx
    import sparkucx_amd._lib as L

    e = sgx.ShuffleEngine(0)
    so = ctypes.CDLL(L.LIB_PATH)
    fn = so.sgx_diag_lz4_stamps
    fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    n, R = a.records, a.partitions
    recs = oracle.gen_uniform16(n, 0x5EEDC0DE)
    if a.case == "c1":  # bench.py's values at C1 size: record indices around 2^27 (varints of 4 bytes)
        recs[:, 8:] = (np.arange(n, dtype=np.int64) + (1 << 27)).view(np.uint8).reshape(-1, 8)
    elif a.case == "lowentropy":
        recs[:, :8] = (np.arange(n, dtype=np.int64) % 4096).view(np.uint8).reshape(-1, 8)
    e.register_shuffle(1, R)
    e.set_serializer(1, 1)
    e.write_map(1, 0, recs, n, 16)
    out = (ctypes.c_ulonglong * 16)()
    e.lz4_frame_map(1, 0, R)  # warm-up
    e.sync()
    assert fn(out, 1) == 0
    e.lz4_frame_map(1, 0, R)
    e.sync()
    assert fn(out, 1) == 0
    v = list(out)
    blocks = max(1, v[15])
    tot = sum(v[:10])
    res = {"case": a.case, "records": n, "blocks": v[15],
           "cycles_per_block": {p: round(v[i] / blocks, 1) for i, p in enumerate(PHASES)},
           "share": {p: round(v[i] / max(1, tot), 4) for i, p in enumerate(PHASES)}}
    print(json.dumps(res))
    e.close()


if __name__ == "__main__":
    main()
