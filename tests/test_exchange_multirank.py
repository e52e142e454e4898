"""The product's exchange with several ranks (ucx/UcxWorkerWrapper.scala:96-186
is what it replaces).  Each process is one executor with its own engine: it writes its own
map on the GPU (K1-K4, Kryo framing, LZ4), ``sgx_exchange`` runs the counts all-gather,
``sgx_plan_exchange``, the all-to-all into the [source rank][my reducers] receive layout,
and the rank then fetches its reducers' blocks (canonical order) and reads them back
decoded, sorted and summed -- all compared with the oracle.

* ``host`` backend (sgx_comm_init_host over a gloo group): 2 and 4 ranks SHARE cuda:0 (RCCL
  refuses two ranks on one device); runs on the one-GPU box.
* ``rccl`` backend (sgx_comm_init, ncclAllGather + ncclAllToAllv over xGMI): one GPU per rank;
  skipped unless the box has enough GPUs (the driver's 8-GPU node runs it).
"""
import datetime
import os
import socket
import traceback

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


_ZIPF = {}


def batch(oracle, rank, k, n, keys="uniform"):
    if keys == "zipf":  # config C3's key distribution: Zipf(1.1) ranks over 2^20 keys
        if "cdf" not in _ZIPF:
            _ZIPF["cdf"] = oracle.zipf_cdf(1.1, 1 << 20)
        return oracle.gen_zipf16(n + 101 * rank + 7 * k, 0xB0 + 16 * k + rank, _ZIPF["cdf"],
                                 value_base=(rank << 40) | (k << 36))
    return oracle.gen_uniform16(n + 101 * rank + 7 * k, 0xA0 + 16 * k + rank, value_base=(rank << 40) | (k << 36))


def worker(rank, world, port, backend, codec, R, n, result_dir, placement="even", keys="uniform"):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=90))
    msg = "ok"
    try:
        import oracle
        import sparkucx_amd as sgx

        e = sgx.ShuffleEngine(device=rank if backend == "rccl" else 0, comm_timeout_ms=60_000)
        if backend == "rccl":
            uid = [sgx.get_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            e.comm_init(world, rank, uid[0])
        else:
            e.comm_init_host(world, rank)
        sid = 1
        e.register_shuffle(sid, R, serializer=sgx.SER_FIXED if codec == "fixed" else sgx.SER_KRYO)
        if codec == "kryo+lz4":
            e.set_compression(sid, "lz4", 4096)
        if placement == "bytes":
            e.set_reducer_placement(sid, "bytes")
        mine = [r for r in range(R) if sgx.reducer_owner(r, R, world) == rank]
        for k in range(3):  # three rounds: map slots reused, receive buffers recycled
            mid = k * world + rank
            recs = batch(oracle, rank, k, n, keys)
            e.write_map(sid, mid, recs, len(recs), 16)
            e.exchange(sid, mid)
            e.sync()
            outs = [oracle.map_write(batch(oracle, r, k, n, keys), R) for r in range(world)]
            seqs = oracle.canonical_reducer_sequences(outs, R, 16)
            maps = [k * world + r for r in range(world)]
            r0, r1 = e.round_reducers(sid, mid)
            if placement == "bytes":
                mine = list(range(r0, r1))
                if codec == "fixed":  # the placement every rank must have computed
                    want_b = sgx.balanced_ranges(np.stack([c * 16 for _, c in outs]))
                    if (r0, r1) != (int(want_b[rank]), int(want_b[rank + 1])):
                        msg = f"round {k}: placement [{r0}, {r1}) differs from {want_b.tolist()}"
                        break
            elif (r0, r1) != ((mine[0], mine[-1] + 1) if mine else (r0, r0)):
                msg = f"round {k}: even placement [{r0}, {r1}) differs"
                break
            if not mine:
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
                    for (out, counts) in outs:
                        o = oracle.offsets(counts)
                        s = oracle.kryo_serialize(out[o[r]:o[r + 1]])
                        if codec == "kryo+lz4":
                            s, _ = oracle.lz4_frame_partitions(s, np.array([0, len(s)], np.int64), 4096)
                        blocks.append(np.asarray(s, np.uint8).reshape(-1))
                want = np.concatenate(blocks) if blocks else np.zeros(0, np.uint8)
            if not np.array_equal(data, want):
                msg = f"round {k}: fetched blocks differ ({data.size} vs {want.size} bytes)"
                break
            got = e.read_records(sid, maps, mine[0], mine[-1] + 1).reshape(-1, 16)
            if not np.array_equal(got, np.concatenate([seqs[r] for r in mine])):
                msg = f"round {k}: decoded records differ"
                break
            got = e.read_sorted(sid, maps, mine[0], mine[-1] + 1).reshape(-1, 16)
            if not np.array_equal(got, oracle.reduce_sorted(seqs[mine[0]:mine[-1] + 1])):
                msg = f"round {k}: sorted read differs"
                break
            gk, gs = e.read_grouped(sid, maps, mine[0], mine[-1] + 1, sgx.AGG_SUM)
            wk, ws = oracle.reduce_grouped(seqs[mine[0]:mine[-1] + 1], "sum")
            if not (np.array_equal(gk, wk) and np.array_equal(gs, ws)):
                msg = f"round {k}: reduceByKey sums differ"
                break
        st = e.stats()
        if msg == "ok" and st.count["alltoall"] < 3:
            msg = f"only {st.count['alltoall']} all-to-all rounds recorded"
        e.close()
    except Exception:  # noqa: BLE001 - reported through the result file
        msg = traceback.format_exc()
    finally:
        with open(os.path.join(result_dir, f"rank{rank}"), "w") as f:
            f.write(msg)
        dist.destroy_process_group()


def run_world(tmp_path, world, backend, codec, R, n, placement="even", keys="uniform"):
    import torch.multiprocessing as mp

    mp.start_processes(worker, args=(world, free_port(), backend, codec, R, n, str(tmp_path), placement, keys),
                       nprocs=world, start_method="spawn", join=True)
    msgs = {r: (tmp_path / f"rank{r}").read_text() for r in range(world)}
    bad = {r: m for r, m in msgs.items() if m != "ok"}
    assert not bad, "\n".join(f"rank {r}: {m}" for r, m in bad.items())


@pytest.mark.parametrize("world,codec,R,n", [(2, "fixed", 1024, 200_000), (4, "fixed", 1024, 100_000),
                                             (4, "fixed", 3, 5_000), (2, "kryo", 200, 60_000),
                                             (4, "kryo", 200, 40_000),
                                             (4, "kryo+lz4", 200, 40_000), (2, "kryo+lz4", 7, 20_000)])
def test_exchange_host_backend_ranks_share_one_gpu(sgx_lib, oracle_lib, tmp_path, world, codec, R, n):
    run_world(tmp_path, world, "host", codec, R, n)


@pytest.mark.parametrize("placement", ["even", "bytes"])
def test_exchange_eight_ranks_share_one_gpu(sgx_lib, oracle_lib, tmp_path, placement):
    """C2's rank count (P = 8) through the product's exchange, 8 executors sharing cuda:0 over
    the host backend: every rank's fetched blocks, decoded / sorted / summed reads of its
    reducer range equal the oracle's canonical sequences, with both reducer placements."""
    run_world(tmp_path, 8, "host", "fixed", 1024, 250_000, placement=placement,
              keys="zipf" if placement == "bytes" else "uniform")


@pytest.mark.parametrize("world,codec,R,n", [(4, "fixed", 4096, 100_000), (2, "fixed", 1024, 100_000),
                                             (4, "kryo+lz4", 1024, 40_000), (3, "fixed", 5, 5_000)])
def test_exchange_byte_balanced_placement_zipf(sgx_lib, oracle_lib, tmp_path, world, codec, R, n):
    """Config C3's skew (Zipf(1.1) keys) with SGX_PLACE_BYTES: every rank's round range is the
    byte-balanced placement of the all-gathered lengths, and what it fetches and reads back
    for that range equals the oracle's canonical sequences."""
    run_world(tmp_path, world, "host", codec, R, n, placement="bytes", keys="zipf")


@pytest.mark.parametrize("world", [2, 4, 8])
def test_exchange_rccl_one_gpu_per_rank(sgx_lib, oracle_lib, tmp_path, world):
    import torch

    if torch.cuda.device_count() < world:
        pytest.skip(f"needs {world} GPUs (RCCL refuses ranks sharing a device)")
    run_world(tmp_path, world, "rccl", "fixed", 1024, 300_000)
    run_world(tmp_path, world, "rccl", "kryo+lz4", 200, 50_000)


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
