#!/usr/bin/env python3
"""Phase shares of the write-combining K4's tile loop, from a stamp build:
    bash tools/build_variant.sh stamps - -DSGX_WC_STAMPS
    python tools/ab_run.py tools/ab/libsgx_stamps.so wc_stamps [--partitions 1024]
Prints one JSON line: s_memtime cycles per tile per wave in each phase and their shares.
The build's own run time is not a measurement (the stamps' waits forbid overlaps)."""
import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PHASES = ["wait_loads", "rank", "merge", "stage_zero_loads_B4", "unused", "loop", "stage_reads", "stage_deferred_writes",
          "stage_new_writes", "drain_lds_reads", "drain_stores", "unused2"]
# k_scatter_wide2 (TeraSort 100 B records, --record-bytes 100)
PHASES_WIDE2 = ["loop_top", "land_stage_writes_barrier", "issue_next_loads", "partition_ids", "rank_barrier",
                "merge", "sorted_index", "drain_lds_reads", "drain_stores", "final_barrier", "unused", "unused2"]
# k_scatter_wide_wc (the padded TeraSort K4, --record-bytes 100 --wide-wc)
PHASES_WIDE_WC = ["loop_top", "carry_writeback", "land_barrier", "issue_next_loads", "partition_ids_rank_barrier",
                  "merge_rows_read", "sorted_index_barrier", "drain", "owner_next_carries", "final_barrier",
                  "merge_scan_barrier", "merge_totals_read", "merge_rows_units_written", "merge_barrier"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=1 << 28)
    ap.add_argument("--partitions", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--dist", default="uniform")
    ap.add_argument("--record-bytes", type=int, default=16, choices=[16, 100])
    ap.add_argument("--wide-wc", action="store_true", help="100 B records on the padded write (k_scatter_wide_wc)")
    a = ap.parse_args()
    import numpy as np

    import sparkucx_amd as sgx
    import sparkucx_amd._lib as L

    e = sgx.ShuffleEngine(0, 0)
    so = ctypes.CDLL(L.LIB_PATH)
    fn = so.sgx_diag_wc_stamps
    fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    rb = a.record_bytes
    n = a.records if rb == 16 else a.records * 16 // 100
    buf = e.alloc(n * rb)
    if rb == 100:
        e.gen_terasort100(buf, n, 0x5EEDC0DE)
        hi = (np.arange(1, a.partitions, dtype=np.uint64) * (np.uint64(1 << 63) // np.uint64(a.partitions)) * 2)
        bounds = np.zeros((a.partitions - 1, 10), np.uint8)
        for j in range(8):
            bounds[:, j] = (hi >> np.uint64(56 - 8 * j)) & np.uint64(0xFF)
        e.register_shuffle(1, a.partitions, kind=sgx.PART_RANGE_BYTES10, bounds=bounds, record_bytes=100)
    elif a.dist == "uniform":
        e.gen_uniform16(buf, a.records, 0x5EEDC0DE)
    else:
        r = np.arange(1, (1 << 24) + 1, dtype=np.float64)
        cdf = np.cumsum(r ** -1.1)
        cdf /= cdf[-1]
        e.gen_zipf16(buf, a.records, 0x5EEDC0DE, cdf)
    if rb == 16:
        e.register_shuffle(1, a.partitions)
    out = (ctypes.c_ulonglong * 16)()
    e.write_map(1, 0, buf, n, rb)  # warm-up
    e.sync()
    assert fn(out, 1) == 0
    for i in range(a.iters):
        e.write_map(1, 1 + i, buf, n, rb)
    e.sync()
    assert fn(out, 1) == 0
    v = list(out)
    waves_tiles = v[14]  # every wave adds its workgroup's tile count
    nph = 14 if a.wide_wc else 12
    tot = sum(v[:nph])
    names = PHASES_WIDE_WC if a.wide_wc else PHASES_WIDE2 if rb == 100 else PHASES
    names = names[:nph]
    res = {"partitions": a.partitions, "dist": a.dist if rb == 16 else "terasort", "workgroups": v[15] // 8, "tile_waves": v[14],
           "cycles_per_tile_wave": {p: round(v[i] / max(1, waves_tiles), 1) for i, p in enumerate(names)},
           "share": {p: round(v[i] / max(1, tot), 4) for i, p in enumerate(names)}}
    print(json.dumps(res))
    e.close()


if __name__ == "__main__":
    main()
