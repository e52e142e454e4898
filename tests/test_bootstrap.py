"""CPU, several processes: the id bootstrap over TCP (§8(f) row 4, replacing the
ExecutorAdded / IntroduceAllExecutors RPC of rpc/UcxDriverRpcEndpoint.scala:21-42).  Rank 0
serves a 128-byte id, ranks 1..n-1 join (possibly before the server is up) and must all
receive the same bytes and the world size; a missing rank makes the server time out."""
import os
import socket

import pytest
import torch.multiprocessing as mp


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def worker(rank, world, port, result_dir):
    import time

    import sparkucx_amd as sgx

    uid = bytes((i * 7 + 3) & 0xFF for i in range(128))
    if rank == 0:
        time.sleep(0.3)  # joiners start first: they must retry until the server listens
        sgx.bootstrap_serve(port, world, uid, 20_000)
        out = "ok"
    else:
        got, n = sgx.bootstrap_join("127.0.0.1", port, rank, 20_000)
        out = "ok" if (got == uid and n == world) else f"bad {n}"
    with open(os.path.join(result_dir, f"rank{rank}"), "w") as f:
        f.write(out)


@pytest.mark.parametrize("world", [2, 5])
def test_bootstrap_distributes_the_id(tmp_path, sgx_lib, world):
    mp.start_processes(worker, args=(world, free_port(), str(tmp_path)), nprocs=world, start_method="spawn",
                       join=True)
    for r in range(world):
        assert (tmp_path / f"rank{r}").read_text() == "ok"


def test_bootstrap_server_times_out_without_joiners(sgx_lib):
    with pytest.raises(sgx_lib.ShuffleError, match="joined before the timeout"):
        sgx_lib.bootstrap_serve(free_port(), 3, b"x" * 128, 300)


def test_bootstrap_join_times_out_without_server(sgx_lib):
    with pytest.raises(sgx_lib.ShuffleError, match="could not join"):
        sgx_lib.bootstrap_join("127.0.0.1", free_port(), 1, 300)
