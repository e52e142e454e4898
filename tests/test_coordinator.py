"""The exchange's ordering protocol (sparkucx_amd.coordinator, the Python mirror of the JVM's
GpuExchangeCoordinator.scala) driving the real engine's collective.

Three executor processes share cuda:0 over the host collective backend; the driver is a
thread of the test process (no GPU) connected by FIFO queues, as Spark RPC connects the
driver endpoint and the executors.  Two shuffles are read by reduce tasks that start on
different executors in opposite orders (executor 0 asks for A then B, executor 2 for B then A):
without the driver's one global sequence the executors would enter different collectives
and hang; with it every executor runs A and B in the same order and every read of every
executor's reducers equals the oracle.  Executor 0 writes no map of B and first learns of B
from its GpuRunExchange (it registers B from the request's spec before the collective).

A third shuffle's first round fails on executor 1 before the collective (its registration
raises once): executor 1 joins the round's all-gather through sgx_exchange_fail, every
executor's exchange of that round fails together (no waiting for the timeout), the driver
forgets the round, and the readers' retry runs a second round that succeeds (the driver
broadcasts shuffle 3 exactly twice; the readers waiting on the first round see its error)."""
import datetime
import os
import socket
import threading
import traceback

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


# maps per (shuffle, executor): map id -> (records, seed)
MAPS = {
    1: {0: [100, 101], 1: [102], 2: []},      # A: R = 300, fixed codec
    2: {0: [], 1: [200], 2: [201, 202]},      # B: R = 64, Kryo + LZ4
    3: {0: [300], 1: [], 2: [301]},           # C: R = 128, fixed codec; executor 1 fails once
}


def specs():
    from sparkucx_amd import SER_FIXED, SER_KRYO
    from sparkucx_amd.coordinator import ShuffleSpec

    return {1: ShuffleSpec(1, 300), 2: ShuffleSpec(2, 64, serializer=SER_KRYO, lz4_block=4096),
            3: ShuffleSpec(3, 128, serializer=SER_FIXED)}


def records(oracle, mid):
    return oracle.gen_uniform16(20_000 + 37 * mid, 0xC0 + mid, value_base=mid << 32)


def all_maps(sid):
    return sorted(m for ms in MAPS[sid].values() for m in ms)


def executor(rank, world, port, driver_q, my_q, result_dir):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=120))
    msg = "ok"
    try:
        import oracle
        import sparkucx_amd as sgx
        from sparkucx_amd.coordinator import ExchangeCoordinator
        from sparkucx_amd.hostcomm import TorchDistributedCollectives

        e = sgx.ShuffleEngine(device=0, comm_timeout_ms=60_000)
        # the engine's collectives on their own group (the comm thread uses it; this thread
        # uses the default group for the test's own bookkeeping)
        e.comm_init_host(world, rank, TorchDistributedCollectives(dist.new_group(backend="gloo")))
        sp = specs()
        failed_once = []

        def register(spec):
            if rank == 1 and spec.shuffle_id == 3 and not failed_once:
                failed_once.append(1)
                raise RuntimeError("injected: registering shuffle 3 failed")
            spec.register(e)

        co = ExchangeCoordinator(e, driver_q, my_q, register=register, timeout_s=120)
        # map tasks: register on first use, write
        for sid in (1, 2, 3):
            for mid in MAPS[sid][rank]:
                co.ensure_registered(sp[sid])
                recs = records(oracle, mid)
                e.write_map(sid, mid, recs, len(recs), 16)
        dist.barrier()  # the map stages are complete before any reduce task starts

        # reduce tasks: executor 0 asks for A then B, executor 2 for B then A, executor 1 for B
        order = {0: (1, 2), 1: (2,), 2: (2, 1)}[rank]
        threads, errs = [], []

        def reader(sid):
            try:
                co.await_exchange(sp[sid], all_maps(sid))
            except Exception:  # noqa: BLE001
                errs.append(traceback.format_exc())

        for sid in order:  # started back to back: their requests race to the driver
            t = threading.Thread(target=reader, args=(sid,))
            t.start()
            threads.append(t)
        for t in threads:
            t.join()
        if errs:
            raise RuntimeError(errs[0])
        for sid in (1, 2):
            co.await_exchange(sp[sid], all_maps(sid))  # completed rounds: returns at once
        ran = [k for k, _ in co.ran]
        if sorted(ran) != sorted([(1, tuple(all_maps(1))), (2, tuple(all_maps(2)))]):
            raise RuntimeError(f"rounds run here: {co.ran}")
        seen = [None] * world
        dist.all_gather_object(seen, ran)
        if any(s != seen[0] for s in seen):
            raise RuntimeError(f"executors ran the exchanges in different orders: {seen}")
        # every executor reads its reducers of A and B (fixed codec and Kryo + LZ4)
        for sid in (1, 2):
            R = sp[sid].num_partitions
            outs = [oracle.map_write(records(oracle, m), R) for m in all_maps(sid)]
            seqs = oracle.canonical_reducer_sequences(outs, R, 16)
            r0, r1 = e.shuffle_reducers(sid)
            got = e.read_records(sid, all_maps(sid), r0, r1).reshape(-1, 16)
            want = np.concatenate(seqs[r0:r1]) if r1 > r0 else np.zeros((0, 16), np.uint8)
            if not np.array_equal(got, want):
                raise RuntimeError(f"shuffle {sid}: records of [{r0}, {r1}) differ")
            k, s = e.read_grouped(sid, all_maps(sid), r0, r1, sgx.AGG_SUM)
            wk, ws = oracle.reduce_grouped(seqs[r0:r1], "sum")
            if not (np.array_equal(k, wk) and np.array_equal(s, ws)):
                raise RuntimeError(f"shuffle {sid}: sums of [{r0}, {r1}) differ")

        # shuffle C: the first round fails everywhere at once, the retry succeeds.  A reader
        # sees the failure when it was waiting for that round; one that asks after the failed
        # round has already run (and been forgotten) starts the retry instead, so at least
        # the executor whose request started the round sees it, not necessarily every one.
        # Which readers see it is pinned deterministically (every reader waiting on the round
        # when it fails, and the retry is one round) in
        # test_coordinator_protocol.py::test_every_waiting_reader_sees_the_failed_round_and_the_retry_is_one_round.
        first_error = None
        for attempt in range(3):
            try:
                co.await_exchange(sp[3], all_maps(3))
                break
            except sgx.ShuffleError as ex:
                first_error = first_error or str(ex)
        else:
            raise RuntimeError("shuffle 3 never exchanged")
        saw = [None] * world
        dist.all_gather_object(saw, first_error is not None)
        if not any(saw):
            raise RuntimeError("the injected failure did not fail the first round anywhere")
        R = sp[3].num_partitions
        outs = [oracle.map_write(records(oracle, m), R) for m in all_maps(3)]
        seqs = oracle.canonical_reducer_sequences(outs, R, 16)
        r0, r1 = e.shuffle_reducers(3)
        got = e.read_records(3, all_maps(3), r0, r1).reshape(-1, 16)
        want = np.concatenate(seqs[r0:r1]) if r1 > r0 else np.zeros((0, 16), np.uint8)
        if not np.array_equal(got, want):
            raise RuntimeError("shuffle 3: records differ after the retried round")
        dist.barrier()
        co.stop()
        e.close()
    except Exception:  # noqa: BLE001 - reported through the result file
        msg = traceback.format_exc()
    finally:
        with open(os.path.join(result_dir, f"rank{rank}"), "w") as f:
            f.write(msg)
        dist.destroy_process_group()


def test_coordinator_orders_exchanges_and_fails_rounds_together(sgx_lib, oracle_lib, tmp_path):
    import torch.multiprocessing as mp

    from sparkucx_amd.coordinator import DriverEndpoint

    world = 3
    ctx = mp.get_context("spawn")
    driver_q = ctx.Queue()
    ex_q = {r: ctx.Queue() for r in range(world)}
    drv = DriverEndpoint(driver_q, ex_q)
    t = threading.Thread(target=drv.serve, daemon=True)
    t.start()
    port = free_port()
    procs = [ctx.Process(target=executor, args=(r, world, port, driver_q, ex_q[r], str(tmp_path)))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=400)
    driver_q.put(("stop",))
    t.join(timeout=10)
    for p in procs:
        if p.is_alive():
            p.kill()
    msgs = {r: (tmp_path / f"rank{r}").read_text() if (tmp_path / f"rank{r}").exists() else "no result"
            for r in range(world)}
    bad = {r: m for r, m in msgs.items() if m != "ok"}
    assert not bad, "\n".join(f"executor {r}: {m}" for r, m in bad.items())
    # the driver broadcast A and B once each and C twice (the failed attempt, then the retry)
    keys = [(k[0], a) for k, a in drv.sequence]
    assert sorted(keys) == [(1, 1), (2, 1), (3, 1), (3, 2)], drv.sequence
