#!/usr/bin/env python3
"""Multi-rank exchange on the GPU path (launch with torch.distributed.run, one process per
rank): every rank writes its own map (K1-K4), sgx_exchange pushes it to the reducer owners
over RCCL (counts all-gather + ncclAllToAllv), then each rank fetches its reducers' blocks
(canonical order), reads them sorted and grouped, and checks everything against the
oracle.  On a one-GPU box all ranks share cuda:0 if RCCL accepts that (probe); the driver's
8-GPU node runs the same code with one GPU per rank.  Prints one line per rank."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch
    import torch.distributed as dist

    import oracle
    import sparkucx_amd as sgx

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    ndev = torch.cuda.device_count()
    dev = int(os.environ.get("LOCAL_RANK", "0")) % max(1, ndev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    R, n = int(os.environ.get("MP_R", "1024")), int(os.environ.get("MP_N", "300000"))
    e = sgx.ShuffleEngine(device=dev)
    uid = [sgx.get_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(uid, src=0)
    e.comm_init(world, rank, uid[0])
    e.register_shuffle(1, R)

    def batch(r, k):
        return oracle.gen_uniform16(n + 101 * r + 7 * k, 0xA0 + 16 * k + r, value_base=(r << 40) | (k << 36))

    ok = True
    for k in range(3):  # three rounds: map slots reused, receive buffers recycled
        mid = k * world + rank
        e.write_map(1, mid, batch(rank, k), n + 101 * rank + 7 * k, 16)
        e.exchange(1, mid)
        e.sync()
        outs = [oracle.map_write(batch(r, k), R) for r in range(world)]
        seqs = oracle.canonical_reducer_sequences(outs, R, 16)
        mine = [r for r in range(R) if sgx.reducer_owner(r, R, world) == rank]
        maps = [k * world + r for r in range(world)]
        mids = [m for r in mine for m in maps]
        rids = [r for r in mine for _ in maps]
        data, _ = e.fetch_blocks(1, mids, rids)
        want = np.concatenate([seqs[r] for r in mine]).reshape(-1)
        ok &= np.array_equal(data, want)
        got = e.read_sorted(1, maps, mine[0], mine[-1] + 1).reshape(-1, 16)
        ok &= np.array_equal(got, oracle.reduce_sorted(seqs[mine[0]:mine[-1] + 1]))
        gk, gs = e.read_grouped(1, maps, mine[0], mine[-1] + 1, sgx.AGG_SUM)
        wk, ws = oracle.reduce_grouped(seqs[mine[0]:mine[-1] + 1], "sum")
        ok &= np.array_equal(gk, wk) and np.array_equal(gs, ws)
    st = e.stats()
    print(f"rank {rank}/{world} dev {dev}: {'ok' if ok else 'MISMATCH'} alltoall x{st.count['alltoall']} "
          f"{st.ms['alltoall'] / max(1, st.count['alltoall']):.3f} ms", flush=True)
    e.close()
    dist.destroy_process_group()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
