"""The product's exchange with several ranks (ucx/UcxWorkerWrapper.scala:96-186
is what it replaces, spark_3_0/UcxShuffleReader.scala:74-103 / UcxShuffleClient.scala:17-47 the
"any block from anywhere" contract it has to honour).

Each process is one executor with its own engine.  Like Spark's map tasks, the maps land on
executors unevenly -- some ranks hold none, some several -- and every rank then calls
``sgx_exchange(e, shuffle_id)`` once per round: an all-gather of every rank's map count and
lengths, then one grouped all-to-all of the partition-contiguous map outputs into the
[source rank][its maps][my reducers] receive layout.  Afterwards each rank fetches its
reducers' blocks of EVERY map of EVERY rank and every round (canonical order: reducer-major,
map ids ascending) and reads them back decoded, sorted and summed -- all compared with the
oracle.  The reducer ranges are fixed by the shuffle's first round, so a second round's
blocks land where the first round's did.

* ``host`` backend (sgx_comm_init_host over a gloo group): ranks SHARE cuda:0 (RCCL refuses
  two ranks on one device); runs on the one-GPU box.
* ``rccl`` backend (sgx_comm_init, ncclAllGather + grouped ncclSend/ncclRecv over xGMI): one
  GPU per rank; skipped unless the box has enough GPUs (the driver's 8-GPU node runs it).

Config C4 (TeraSort 100 B records, 10-byte keys, RangePartitioner) runs the same exchange:
every rank's sorted read is its reducers' canonical sequences sorted, and the rank-order
concatenation of all ranks' sorted reads is the globally sorted input.
"""
import datetime
import os
import socket
import traceback

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

_ZIPF = {}


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def map_id(t, j, k):
    """Map k of rank j in round t: unique across ranks and rounds."""
    return t * 4096 + j * 64 + k


def batch(oracle, t, j, k, n, keys="uniform", rb=16):
    """The records of map (t, j, k): ragged sizes, their own seeds."""
    nn = n + 101 * j + 7 * k + 13 * t
    seed = 0xA0 + 4096 * t + 64 * j + k
    base = (j << 40) | (k << 34) | (t << 30)
    if rb == 100:
        return oracle.gen_terasort100(nn, seed, index_base=base)
    if keys == "zipf":  # config C3's key distribution: Zipf(1.1) ranks over 2^20 keys
        if "cdf" not in _ZIPF:
            _ZIPF["cdf"] = oracle.zipf_cdf(1.1, 1 << 20)
        return oracle.gen_zipf16(nn, seed, _ZIPF["cdf"], value_base=base)
    return oracle.gen_uniform16(nn, seed, value_base=base)


def terasort_bounds(oracle, R):
    """R - 1 RangePartitioner bounds over 10-byte keys, from a sample every rank draws alike."""
    sample = oracle.gen_terasort100(20 * R, 0xC4)[:, :10]
    sample = sample[np.lexsort(sample.T[::-1])]
    return np.ascontiguousarray(sample[[int(len(sample) / R * (i + 1)) for i in range(R - 1)]])


def all_maps(world, counts_by_round, upto):
    """[(t, j, k)] of every map written in rounds 0..upto, in map id order."""
    out = [(t, j, k) for t in range(upto + 1) for j in range(world) for k in range(counts_by_round[t][j])]
    return sorted(out, key=lambda x: map_id(*x))


def worker(rank, world, port, backend, codec, R, n, result_dir, placement, keys, counts_by_round, rb, flags=0):
    import torch.distributed as dist

    fallback = isinstance(flags, (list, tuple))  # per-rank flags: one rank refuses the peer gather
    flags = flags[rank] if fallback else flags
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=120))
    msg = "ok"
    try:
        import oracle
        import sparkucx_amd as sgx

        e = sgx.ShuffleEngine(device=rank if backend == "rccl" else 0, comm_timeout_ms=60_000, flags=flags)
        if backend == "rccl":
            uid = [sgx.get_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            e.comm_init(world, rank, uid[0])
        else:
            e.comm_init_host(world, rank)
        sid = 1
        kind, bounds = oracle.PART_HASH, None
        if rb == 100:
            kind, bounds = oracle.PART_RANGE_BYTES10, terasort_bounds(oracle, R)
            e.register_shuffle(sid, R, sgx.PART_RANGE_BYTES10, bounds, True, 100)
        else:
            e.register_shuffle(sid, R, serializer=sgx.SER_FIXED if codec == "fixed" else sgx.SER_KRYO)
        if codec == "kryo+lz4":
            e.set_compression(sid, "lz4", 4096)
        if placement == "bytes":
            e.set_reducer_placement(sid, "bytes")
        outs = {}  # (t, j, k) -> oracle map output
        published = 0  # bytes of my maps: what the exchange rounds must move, no more
        for t, counts in enumerate(counts_by_round):
            for k in range(counts[rank]):
                recs = batch(oracle, t, rank, k, n, keys, rb)
                lens_k = e.write_map(sid, map_id(t, rank, k), recs, len(recs), rb, R)
                published += int(lens_k.sum())
                if flags & sgx.FLAG_PAD_ANY_SIZE and codec == "fixed" and not flags & sgx.FLAG_NO_P2P_EXCHANGE:
                    # after a fallback (round 0's exchange) every later map is written two-pass
                    padded = e.map_layout(sid, map_id(t, rank, k)) == sgx.LAYOUT_PADDED
                    if padded != (not fallback or t == 0):
                        raise AssertionError(f"round {t}: map layout padded={padded} under a communicator")
            e.exchange(sid)  # every rank, whatever it holds (maybe nothing)
            e.sync()
            for key in all_maps(world, counts_by_round, t):
                if key not in outs:
                    outs[key] = oracle.map_write(batch(oracle, *key, n, keys, rb), R, kind, bounds)
            order = all_maps(world, counts_by_round, t)
            maps = [map_id(*x) for x in order]
            seqs = oracle.canonical_reducer_sequences([outs[x] for x in order], R, rb)
            r0, r1 = e.shuffle_reducers(sid)
            # the ranges are the shuffle's: every rank agrees and they tile [0, R)
            ranges = [None] * world
            dist.all_gather_object(ranges, (r0, r1))
            if ranges[0][0] != 0 or ranges[-1][1] != R or any(ranges[i][1] != ranges[i + 1][0]
                                                              for i in range(world - 1)):
                msg = f"round {t}: reducer ranges {ranges} do not tile [0, {R})"
                break
            if placement == "even":
                want_r = sgx.even_ranges(world, R)
            elif codec == "fixed":  # byte-balanced over the FIRST round's lengths, summed per rank
                first = [(j, k) for j in range(world) for k in range(counts_by_round[0][j])]
                per_rank = np.zeros((world, R), np.int64)
                for (j, k) in first:
                    per_rank[j] += outs[(0, j, k)][1] * rb
                want_r = sgx.balanced_ranges(per_rank) if first else sgx.even_ranges(world, R)
            else:
                want_r = None
            if want_r is not None and (r0, r1) != (int(want_r[rank]), int(want_r[rank + 1])):
                msg = f"round {t}: placement [{r0}, {r1}) differs from {list(want_r)}"
                break
            if t > 0 and e.round_reducers(sid, maps[0]) != (r0, r1):
                msg = f"round {t}: an earlier round's range differs from the shuffle's"
                break
            mine = list(range(r0, r1))
            if rb == 100 and t == len(counts_by_round) - 1:
                got = e.read_sorted(sid, maps, r0, r1).reshape(-1, rb) if mine else np.zeros((0, rb), np.uint8)
                np.save(os.path.join(result_dir, f"sorted{rank}.npy"), got)
            if not mine or not maps:
                continue
            # raw blocks of my reducers, reducer-major / map-minor: the published bytes
            mids = [m for r in mine for m in maps]
            rids = [r for r in mine for _ in maps]
            data, lens = e.fetch_blocks(sid, mids, rids)
            if codec == "fixed":
                want = np.concatenate([seqs[r] for r in mine]).reshape(-1)
            else:
                blocks = []
                for r in mine:
                    for x in order:
                        out, counts_ = outs[x]
                        o = oracle.offsets(counts_)
                        s = oracle.kryo_serialize(out[o[r]:o[r + 1]])
                        if codec == "kryo+lz4":
                            s, _ = oracle.lz4_frame_partitions(s, np.array([0, len(s)], np.int64), 4096)
                        blocks.append(np.asarray(s, np.uint8).reshape(-1))
                want = np.concatenate(blocks) if blocks else np.zeros(0, np.uint8)
            if not np.array_equal(data, want):
                msg = f"round {t}: fetched blocks differ ({data.size} vs {want.size} bytes)"
                break
            got = e.read_records(sid, maps, r0, r1).reshape(-1, rb)
            if not np.array_equal(got, np.concatenate([seqs[r] for r in mine])):
                msg = f"round {t}: decoded records differ"
                break
            got = e.read_sorted(sid, maps, r0, r1).reshape(-1, rb)
            if not np.array_equal(got, oracle.reduce_sorted(seqs[r0:r1])):
                msg = f"round {t}: sorted read differs"
                break
            if rb == 16:
                gk, gs = e.read_grouped(sid, maps, r0, r1, sgx.AGG_SUM)
                wk, ws = oracle.reduce_grouped(seqs[r0:r1], "sum")
                if not (np.array_equal(gk, wk) and np.array_equal(gs, ws)):
                    msg = f"round {t}: reduceByKey sums differ"
                    break
        st = e.stats()
        if msg == "ok" and st.count["alltoall"] < len(counts_by_round):
            msg = f"only {st.count['alltoall']} exchange rounds recorded"
        xb = e.exchange_bytes()
        if msg == "ok" and xb["sent"] + xb["kept"] != published:
            msg = f"the exchange moved {xb['sent']} + {xb['kept']} bytes for {published} published"
        e.close()
    except Exception:  # noqa: BLE001 - reported through the result file
        msg = traceback.format_exc()
    finally:
        with open(os.path.join(result_dir, f"rank{rank}"), "w") as f:
            f.write(msg)
        dist.destroy_process_group()


def run_world(tmp_path, world, backend, codec, R, n, placement="even", keys="uniform", counts_by_round=None,
              rb=16, flags=0):
    import torch.multiprocessing as mp

    counts_by_round = counts_by_round or [[1] * world] * 3
    mp.start_processes(worker, args=(world, free_port(), backend, codec, R, n, str(tmp_path), placement, keys,
                                     counts_by_round, rb, flags),
                       nprocs=world, start_method="spawn", join=True)
    msgs = {r: (tmp_path / f"rank{r}").read_text() for r in range(world)}
    bad = {r: m for r, m in msgs.items() if m != "ok"}
    assert not bad, "\n".join(f"rank {r}: {m}" for r, m in bad.items())


@pytest.mark.parametrize("codec,R,n", [("fixed", 1024, 60_000), ("kryo", 200, 30_000), ("kryo+lz4", 200, 30_000)])
def test_exchange_per_shuffle_uneven_maps(sgx_lib, oracle_lib, tmp_path, codec, R, n):
    """Spark's task model: 3 executors hold 0, 1 and 4 maps of the shuffle, each calls
    sgx_exchange(shuffle) once; a second round adds maps on a different spread (2, 0, 1).
    Every rank's fetched blocks and decoded / sorted / summed reads of its reducers over ALL
    maps of both rounds equal the oracle's canonical sequences."""
    run_world(tmp_path, 3, "host", codec, R, n, counts_by_round=[[0, 1, 4], [2, 0, 1]])


def test_exchange_spark_map_counts_host_backend(sgx_lib, oracle_lib, tmp_path):
    """Spark's map counts per executor: 64 maps on one rank, none and 3 on the others, then
    a second round with 0 / 40 / 1, host backend (three executors sharing the GPU)."""
    run_world(tmp_path, 3, "host", "fixed", 256, 2_000, counts_by_round=[[64, 0, 3], [0, 40, 1]])


def test_exchange_per_shuffle_rank_without_maps_in_every_round(sgx_lib, oracle_lib, tmp_path):
    """A rank that never holds a map still takes part in every round and reads its reducers;
    a round where nobody holds a map is a no-op collective."""
    run_world(tmp_path, 4, "host", "fixed", 300, 20_000, counts_by_round=[[3, 0, 2, 0], [0, 0, 0, 0], [0, 2, 0, 0]])


@pytest.mark.parametrize("world,codec,R,n", [(2, "fixed", 1024, 200_000), (4, "fixed", 1024, 100_000),
                                             (4, "fixed", 3, 5_000), (2, "kryo", 200, 60_000),
                                             (4, "kryo", 200, 40_000),
                                             (4, "kryo+lz4", 200, 40_000), (2, "kryo+lz4", 7, 20_000)])
def test_exchange_host_backend_ranks_share_one_gpu(sgx_lib, oracle_lib, tmp_path, world, codec, R, n):
    """One map per rank per round, three rounds, each exchanged by sgx_exchange(shuffle)."""
    run_world(tmp_path, world, "host", codec, R, n)


@pytest.mark.parametrize("placement", ["even", "bytes"])
def test_exchange_eight_ranks_share_one_gpu(sgx_lib, oracle_lib, tmp_path, placement):
    """C2's rank count (P = 8) through the product's exchange, 8 executors sharing cuda:0 over
    the host backend: every rank's fetched blocks, decoded / sorted / summed reads of its
    reducer range equal the oracle's canonical sequences, with both reducer placements."""
    run_world(tmp_path, 8, "host", "fixed", 1024, 250_000, placement=placement,
              keys="zipf" if placement == "bytes" else "uniform", counts_by_round=[[1] * 8, [1] * 8])


@pytest.mark.parametrize("world,codec,R,n", [(4, "fixed", 4096, 100_000), (2, "fixed", 1024, 100_000),
                                             (4, "kryo+lz4", 1024, 40_000), (3, "fixed", 5, 5_000)])
def test_exchange_byte_balanced_placement_zipf(sgx_lib, oracle_lib, tmp_path, world, codec, R, n):
    """Config C3's skew (Zipf(1.1) keys) with SGX_PLACE_BYTES: the shuffle's ranges are the
    byte-balanced placement of the first round's lengths, and they hold for the later rounds
    (a reducer's blocks of every round on one rank: what the reader fetches across rounds)."""
    run_world(tmp_path, world, "host", codec, R, n, placement="bytes", keys="zipf",
              counts_by_round=[[1] * world, [2] + [1] * (world - 1), [0] * (world - 1) + [2]])


@pytest.mark.parametrize("world,R", [(2, 1024), (4, 1024), (3, 64)])
def test_exchange_terasort_c4(sgx_lib, oracle_lib, tmp_path, world, R):
    """Config C4's exchange leg: 100 B TeraSort records (10-byte keys) under a RangePartitioner
    (PART_RANGE_BYTES10), uneven maps per rank, two rounds.  Each rank's fetched blocks equal
    the oracle's byte for byte and its sorted read equals its reducers' sorted canonical
    sequences; the rank-order concatenation of every rank's sorted read is the whole input
    sorted by key (ascending RangePartitioner: partition order is key order)."""
    import oracle

    counts = [[1] * world, [2] + [0] * (world - 1)]
    n = 30_000
    run_world(tmp_path, world, "host", "fixed", R, n, counts_by_round=counts, rb=100)
    got = np.concatenate([np.load(tmp_path / f"sorted{r}.npy") for r in range(world)])
    allrecs = np.concatenate([batch(oracle, *x, n, "uniform", 100) for x in all_maps(world, counts, 1)])
    keys = allrecs[:, :10]
    want = allrecs[np.lexsort(keys.T[::-1])]
    assert got.shape == want.shape
    # keys sorted globally; records equal as a multiset in key order (ties: stable per reducer)
    assert np.array_equal(got[:, :10], want[:, :10])
    assert np.array_equal(np.sort(got.view("V100").reshape(-1)), np.sort(want.view("V100").reshape(-1)))


@pytest.mark.parametrize("world,R,keys", [(2, 1024, "uniform"), (4, 200, "uniform"), (8, 1024, "uniform"),
                                          (3, 4096, "zipf")])
def test_exchange_p2p_from_padded_maps(sgx_lib, oracle_lib, tmp_path, world, R, keys):
    """The direct peer gather: under a communicator every map is written in ONE
    pass (padded, SGX_FLAG_PAD_ANY_SIZE so the test's maps qualify) and each rank writes the
    blocks other ranks own straight from the map's fragments into their receive buffers,
    mapped through IPC handles (separate processes sharing cuda:0).  Blocks and reads as the
    oracle's; the bytes moved equal the published lengths (no sub-bin slack)."""
    import sparkucx_amd as sgx

    run_world(tmp_path, world, "host", "fixed", R, 150_000, keys=keys,
              placement="bytes" if keys == "zipf" else "even",
              counts_by_round=[[1] * world, [2] + [0] * (world - 2) + [1]], flags=sgx.FLAG_PAD_ANY_SIZE)


def test_exchange_p2p_terasort_padded(sgx_lib, oracle_lib, tmp_path):
    """C4's exchange over the peer gather from padded 100 B TeraSort maps (RangePartitioner)."""
    import oracle
    import sparkucx_amd as sgx

    counts = [[1, 1, 1], [2, 0, 0]]
    run_world(tmp_path, 3, "host", "fixed", 1024, 30_000, counts_by_round=counts, rb=100, flags=sgx.FLAG_PAD_ANY_SIZE)
    got = np.concatenate([np.load(tmp_path / f"sorted{r}.npy") for r in range(3)])
    allrecs = np.concatenate([batch(oracle, *x, 30_000, "uniform", 100) for x in all_maps(3, counts, 1)])
    assert np.array_equal(got[:, :10], allrecs[np.lexsort(allrecs[:, :10].T[::-1])][:, :10])


@pytest.mark.parametrize("world,rb", [(3, 16), (2, 100)])
def test_exchange_falls_back_when_a_rank_cannot_map_peers(sgx_lib, oracle_lib, tmp_path, world, rb):
    """One rank cannot map its receive buffer for the peer gather (SGX_FLAG_TEST_P2P_UNAVAILABLE
    stands for a failing hipIpcGetMemHandle): every rank learns it from the same all-gather
    before any byte moved, the round runs again over contiguous pieces (the padded maps copied
    contiguous once), and the engines write later maps two-pass.  Blocks and reads as the
    oracle's in every round; bytes moved = bytes published."""
    import sparkucx_amd as sgx

    flags = [sgx.FLAG_PAD_ANY_SIZE] * world
    flags[1] |= sgx.FLAG_TEST_P2P_UNAVAILABLE
    run_world(tmp_path, world, "host", "fixed", 1024, 60_000 if rb == 16 else 30_000,
              counts_by_round=[[1] * world, [2] + [0] * (world - 2) + [1]], rb=rb, flags=flags)


@pytest.mark.parametrize("codec", ["fixed", "kryo+lz4"])
def test_exchange_staged_all_to_all_no_p2p(sgx_lib, oracle_lib, tmp_path, codec):
    """SGX_FLAG_NO_P2P_EXCHANGE: the host all-to-all of contiguous map outputs (two-pass
    writes under a communicator), uneven maps."""
    import sparkucx_amd as sgx

    run_world(tmp_path, 3, "host", codec, 200, 30_000, counts_by_round=[[0, 1, 4], [2, 0, 1]],
              flags=sgx.FLAG_NO_P2P_EXCHANGE)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_exchange_rccl_one_gpu_per_rank(sgx_lib, oracle_lib, tmp_path, world):
    import torch

    if torch.cuda.device_count() < world:
        pytest.skip(f"needs {world} GPUs (RCCL refuses ranks sharing a device)")
    run_world(tmp_path, world, "rccl", "fixed", 1024, 300_000)
    uneven = [[k % 3 for k in range(world)], [1] + [0] * (world - 1)]
    run_world(tmp_path, world, "rccl", "kryo+lz4", 200, 50_000, counts_by_round=uneven)
    run_world(tmp_path, world, "rccl", "fixed", 1024, 20_000, counts_by_round=uneven, rb=100)
    # Spark's map counts: many small maps on some ranks (packed sends), few large on others
    many = [[64 if k == 0 else (3 if k % 2 else 0) for k in range(world)], [1] * world]
    run_world(tmp_path, world, "rccl", "kryo+lz4", 200, 3_000, counts_by_round=many)


def test_bench_multi_rank_path_rehearsal(tmp_path):
    """bench.py's N > 1 path (the driver's scaling run) end to end with 2 ranks on this box:
    torch.distributed.run, one engine per rank, the host-collective exchange standing in for
    RCCL (which needs a GPU per rank); rank 0 prints one JSON line with the contract's keys."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.join(root, "bench.py"),
           "--gpus", "2", "--comm", "host", "--records", str(1 << 20), "--partitions", "64", "--steps", "3",
           "--warmup", "1"]
    p = subprocess.run(cmd, cwd=root, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "xgmi_roofline"):
        assert k in d, k
    assert d["n_gpus"] == 2 and d["steps"] == 3 and d["scaling"] == "weak" and d["value"] > 0
    assert d["verified_lengths_sum"] is True
    assert d["xgmi_roofline"]["recv_bytes_max_over_mean"] < 1.1
