"""CPU, world_size 2 over gloo: the multi-rank exchange logic end to end.

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


def worker(rank, world, port, R, n, result_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle
        import sparkucx_amd as sgx

        out, counts = rank_batch(oracle, rank, n, R)
        lengths = torch.from_numpy(counts * 16)
        gathered = [torch.zeros_like(lengths) for _ in range(world)]
        dist.all_gather(gathered, lengths)  # the counts exchange
        L = torch.stack(gathered).numpy()
        sc, sd, rc, rd, items = sgx.plan_exchange(L, rank, 4096)
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
        want = np.concatenate([seqs[r] for r in mine]).reshape(-1) if mine else np.zeros(0, np.uint8)
        ok = np.array_equal(regrouped, want)
        with open(os.path.join(result_dir, f"rank{rank}"), "w") as f:
            f.write("ok" if ok else f"mismatch {regrouped.size} vs {want.size}")
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("R,n", [(1024, 20_000), (200, 5_000), (3, 1_000)])
def test_two_rank_exchange_over_gloo(tmp_path, sgx_lib, oracle_lib, R, n):
    world = 2
    mp.start_processes(worker, args=(world, free_port(), R, n, str(tmp_path)), nprocs=world,
                       start_method="spawn", join=True)
    for r in range(world):
        assert (tmp_path / f"rank{r}").read_text() == "ok"
