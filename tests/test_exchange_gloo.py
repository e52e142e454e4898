"""CPU, world_size 2 and 4 over gloo: the multi-rank exchange logic end to end.

Each rank plays one executor.  Its map output (partition-contiguous 16 B records) is
produced by the oracle — standing in for the GPU kernels, which this container cannot
run — and everything above it is the product's host logic: the counts all-gather, the
exchange plan from libsgx.so (sgx_plan_exchange: send/recv counts and displacements and
the regroup copy list) and the all-to-all.  Every rank must end up holding, for each of
its reducers, the canonical sequence (source rank ascending, input order inside a block)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_batch(oracle, rank, n, R):
    recs = oracle.gen_uniform16(n + 37 * rank, 0xE0 + rank, value_base=rank << 40)
    return oracle.map_write(recs, R)


def worker(rank, world, port, R, n, result_dir, codec="fixed"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle
        import sparkucx_amd as sgx

        out, counts = rank_batch(oracle, rank, n, R)
        if codec == "kryo":  # the Kryo-framed map output (byte-granular blocks)
            lengths = torch.from_numpy(np.diff(oracle.kryo_partition_offsets(out, counts)))
            out = oracle.kryo_serialize(out)
        else:
            lengths = torch.from_numpy(counts * 16)
        gathered = [torch.zeros_like(lengths) for _ in range(world)]
        dist.all_gather(gathered, lengths)  # the counts exchange
        L = torch.stack(gathered).numpy()
        sc, sd, rc, rd, items = sgx.plan_exchange(L, rank, 4096 if codec == "fixed" else 0)
        send = torch.from_numpy(out.reshape(-1).copy())
        recv = torch.empty(int(rc.sum()), dtype=torch.uint8)
        dist.all_to_all_single(recv, send, output_split_sizes=rc.tolist(), input_split_sizes=sc.tolist())
        recv = recv.numpy()
        regrouped = np.empty_like(recv)
        for so, do, nb in items:
            regrouped[do:do + nb] = recv[so:so + nb]
        # canonical per-reducer sequences, from every rank's (deterministic) batch
        outs = [rank_batch(oracle, r, n, R) for r in range(world)]
        seqs = oracle.canonical_reducer_sequences(outs, R, 16)
        mine = [r for r in range(R) if sgx.reducer_owner(r, R, world) == rank]
        if codec == "kryo":  # per-record framing: the blocks' concatenation frames the sequence
            want = np.concatenate([oracle.kryo_serialize(seqs[r].reshape(-1, 16)) for r in mine]) if mine \
                else np.zeros(0, np.uint8)
        else:
            want = np.concatenate([seqs[r] for r in mine]).reshape(-1) if mine else np.zeros(0, np.uint8)
        ok = np.array_equal(regrouped, want)
        with open(os.path.join(result_dir, f"rank{rank}"), "w") as f:
            f.write("ok" if ok else f"mismatch {regrouped.size} vs {want.size}")
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,R,n,codec", [(2, 1024, 20_000, "fixed"), (2, 200, 5_000, "fixed"),
                                             (2, 3, 1_000, "fixed"), (4, 1024, 8_000, "fixed"),
                                             (4, 3, 500, "fixed"), (2, 200, 5_000, "kryo"),
                                             (4, 64, 3_000, "kryo")])
def test_multi_rank_exchange_over_gloo(tmp_path, sgx_lib, oracle_lib, world, R, n, codec):
    mp.start_processes(worker, args=(world, free_port(), R, n, str(tmp_path), codec), nprocs=world,
                       start_method="spawn", join=True)
    for r in range(world):
        assert (tmp_path / f"rank{r}").read_text() == "ok"
