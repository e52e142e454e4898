"""The exchange-ordering protocol of sparkucx_amd.coordinator (mirror of the JVM's
GpuExchangeCoordinator.scala) against a stand-in collective, on the CPU: executors are threads,
the collective is a barrier per round, so the protocol's guarantees are checked
deterministically (tests/test_coordinator.py drives the real engine on the GPU).

Pinned here:
* every reader that waits for a round when it fails sees the failure, on every executor
  (the round fails on all ranks together), and the readers' retry is one new round;
* an executor reports a failed round to the driver BEFORE it drops the round's promise, so a
  retry request from that executor can never reach the driver ahead of the failure report
  (it would be dropped as a duplicate and the reader would wait for the whole timeout);
* a reader that times out keeps the round's promise: a round that was only slow still
  completes it, and the next reader returns without a new round."""
import queue
import threading

import pytest


class _World:
    """A collective per round: each rank's k-th exchange/exchange_fail meets the others' k-th;
    the round fails on every rank if any rank joined it marked failed."""

    def __init__(self, n):
        self.n = n
        self.lock = threading.Lock()
        self.rounds = {}

    def join(self, rank, k, failed):
        with self.lock:
            r = self.rounds.setdefault(k, {"bar": threading.Barrier(self.n), "failed": False})
            r["failed"] |= failed
        r["bar"].wait(timeout=10)
        return not r["failed"]


class _Engine:
    def __init__(self, world, rank, block=None):
        self.world, self.rank, self.k = world, rank, 0
        self.block = block or {}

    def exchange(self, sid):
        ev = self.block.get(sid)
        if ev is not None:
            ev.wait(timeout=10)
        k, self.k = self.k, self.k + 1
        if not self.world.join(self.rank, k, False):
            from sparkucx_amd import IllegalStateException

            raise IllegalStateException(f"round {k} failed on another rank")

    def exchange_fail(self, num_partitions):
        k, self.k = self.k, self.k + 1
        self.world.join(self.rank, k, True)
        from sparkucx_amd import IllegalStateException

        raise IllegalStateException("joined the round marked failed")

    def sync(self):
        pass


class _Tagged:
    """An executor's view of the driver inbox: records (rank, message) in arrival order."""

    def __init__(self, q, rank, log, lock):
        self.q, self.rank, self.log, self.lock = q, rank, log, lock

    def put(self, msg):
        with self.lock:
            self.log.append((self.rank, msg))
            self.q.put(msg)


def _setup(world_n, fail_rank=None, fail_sid=None, block=None, timeout_s=10.0):
    from sparkucx_amd.coordinator import DriverEndpoint, ExchangeCoordinator

    world = _World(world_n)
    driver_q = queue.Queue()
    ex_q = {r: queue.Queue() for r in range(world_n)}
    drv = DriverEndpoint(driver_q, ex_q)
    log, lock = [], threading.Lock()
    cos = []
    for r in range(world_n):
        failed = []

        def register(spec, r=r, failed=failed):
            if r == fail_rank and spec.shuffle_id == fail_sid and not failed:
                failed.append(1)
                raise RuntimeError("injected registration failure")

        cos.append(ExchangeCoordinator(_Engine(world, r, block), _Tagged(driver_q, r, log, lock), ex_q[r],
                                       register=register, timeout_s=timeout_s))
    return drv, driver_q, cos, log


def test_every_waiting_reader_sees_the_failed_round_and_the_retry_is_one_round():
    import sparkucx_amd as sgx
    from sparkucx_amd.coordinator import ShuffleSpec

    n = 3
    drv, driver_q, cos, log = _setup(n, fail_rank=1, fail_sid=3)
    spec = ShuffleSpec(3, 128)
    maps = [300, 301]
    results = {}

    def reader(r):
        try:
            cos[r].await_exchange(spec, maps)
            results[r] = "ok"
        except sgx.ShuffleError as ex:
            results[r] = ex

    ts = [threading.Thread(target=reader, args=(r,)) for r in range(n)]
    for t in ts:
        t.start()
    # every reader's request is queued before the driver runs: all of them wait for attempt 1
    for _ in range(500):
        if driver_q.qsize() == n:
            break
        threading.Event().wait(0.01)
    assert driver_q.qsize() == n
    srv = threading.Thread(target=drv.serve, daemon=True)
    srv.start()
    for t in ts:
        t.join(timeout=20)
    assert all(isinstance(results.get(r), sgx.IllegalStateException) for r in range(n)), results
    # the retries: one new round, which succeeds everywhere
    ts = [threading.Thread(target=reader, args=(r,)) for r in range(n)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=20)
    assert all(results.get(r) == "ok" for r in range(n)), results
    assert [(k[0], a) for k, a in drv.sequence] == [(3, 1), (3, 2)]
    for co in cos:
        assert [a for _, a in co.ran] == [2]
    # per executor: the failure report of attempt 1 precedes its retry request
    for r in range(n):
        mine = [m for rr, m in log if rr == r]
        fail_at = next(i for i, m in enumerate(mine) if m[0] == "failed" and m[3] == 1)
        reqs = [i for i, m in enumerate(mine) if m[0] == "request"]
        # (a retry finds the round already run when another executor's request started it)
        assert 1 <= len(reqs) <= 2 and reqs[0] < fail_at and all(i > fail_at for i in reqs[1:]), mine
    driver_q.put(("stop",))
    for co in cos:
        co.stop()


def test_a_timed_out_reader_keeps_the_round():
    import sparkucx_amd as sgx
    from sparkucx_amd.coordinator import ShuffleSpec

    slow = threading.Event()
    drv, driver_q, cos, log = _setup(1, block={5: slow}, timeout_s=0.3)
    srv = threading.Thread(target=drv.serve, daemon=True)
    srv.start()
    spec = ShuffleSpec(5, 16)
    with pytest.raises(sgx.DeviceTimeout if hasattr(sgx, "DeviceTimeout") else sgx.ShuffleError):
        cos[0].await_exchange(spec, [1, 2])
    slow.set()  # the slow round completes the promise the timed-out reader left
    cos[0].timeout_s = 10
    cos[0].await_exchange(spec, [1, 2])
    assert [(k[0], a) for k, a in drv.sequence] == [(5, 1)]
    assert [a for _, a in cos[0].ran] == [1]
    driver_q.put(("stop",))
    cos[0].stop()
