"""Who calls the collective, and when: the Python mirror of the JVM's GpuExchangeCoordinator
(jvm/.../gpu/GpuExchangeCoordinator.scala), the protocol that orders ``sgx_exchange`` calls.

``sgx_exchange(e, shuffle_id)`` is a collective: every executor of the exchange world must
call it, in the same order relative to its other exchanges.  Spark has no such step -- the
reference pulls each block on demand (spark_3_0/UcxShuffleReader.scala:74-103,
spark_3_0/UcxShuffleClient.scala:17-47) -- so the first reduce task of a shuffle on ANY
executor asks the driver, and the driver, single-threaded, turns those requests into ONE
global sequence of exchanges that it sends to every executor (the reference's rpc/ package
has the same shape: rpc/UcxDriverRpcEndpoint.scala:21-42, rpc/UcxExecutorRpcEndpoint.scala:
19-39).  Readers on different executors may ask for different shuffles in different orders;
every executor still runs the collectives in the driver's order, on one comm thread.

The JVM code cannot be compiled in this image (no JDK), so this module restates its protocol
over any FIFO message channels (``put`` / ``get``: multiprocessing queues in the tests, Spark
RPC's per-sender ordering in the JVM) and is driven against the real engine by
tests/test_coordinator.py:

* key of an exchange: (shuffle id, the shuffle's FULL map id set) -- every reduce task of the
  stage computes the same key whatever its own partition range; a re-run map stage has new
  map ids and gets a new round;
* the request carries the shuffle's ``ShuffleSpec``: an executor that ran no task of the
  shuffle registers it before joining the collective;
* a failed round (sgx_exchange fails on every rank together: a rank's local error travels in
  the round's first all-gather; a rank that fails before calling it, e.g. while registering
  the shuffle, joins that all-gather through sgx_exchange_fail) is reported to the driver,
  which forgets the key so that a retried task starts a new round.  Rounds carry an attempt
  number, so a late failure report of attempt k never cancels attempt k + 1.
"""
from __future__ import annotations

import queue
import threading
from dataclasses import dataclass, field
from typing import Callable, Dict, Optional, Sequence, Tuple

from . import _lib


@dataclass(frozen=True)
class ShuffleSpec:
    """GpuShuffleSpec: the engine registration of a shuffle, decided once on the driver."""

    shuffle_id: int
    num_partitions: int
    kind: int = _lib.PART_HASH
    bounds: Optional[Tuple] = None
    ascending: bool = True
    record_bytes: int = 16
    serializer: int = _lib.SER_FIXED
    lz4_block: int = 0
    placement_bytes: bool = False

    def register(self, engine) -> None:
        import numpy as np

        b = None if self.bounds is None else np.asarray(self.bounds)
        engine.register_shuffle(self.shuffle_id, self.num_partitions, self.kind, b, self.ascending,
                                self.record_bytes, serializer=self.serializer)
        if self.lz4_block:
            engine.set_compression(self.shuffle_id, "lz4", self.lz4_block)
        if self.placement_bytes:
            engine.set_reducer_placement(self.shuffle_id, "bytes")


# messages: ("request", sid, maps, spec) / ("failed", sid, maps, attempt) executor -> driver;
#           ("run", sid, maps, spec, attempt) driver -> executor; ("stop",) to either
Key = Tuple[int, Tuple[int, ...]]


class DriverEndpoint:
    """GpuDriverEndpoint: de-duplicates requests and broadcasts one global exchange sequence
    (every executor, in rank order, in request arrival order)."""

    def __init__(self, inbox, executors: Dict[int, object]):
        self.inbox = inbox
        self.executors = executors  # rank -> that executor's inbox
        self.done: Dict[Key, int] = {}  # key -> attempt of the round broadcast for it
        self.attempts: Dict[Key, int] = {}
        self.sequence = []  # (key, attempt) broadcast, in order (tests inspect it)

    def handle(self, msg) -> bool:
        kind = msg[0]
        if kind == "request":
            _, sid, maps, spec = msg
            key = (sid, tuple(maps))
            if key not in self.done:
                a = self.attempts[key] = self.attempts.get(key, 0) + 1
                self.done[key] = a
                self.sequence.append((key, a))
                for r in sorted(self.executors):
                    self.executors[r].put(("run", sid, tuple(maps), spec, a))
        elif kind == "failed":
            _, sid, maps, attempt = msg
            key = (sid, tuple(maps))
            if self.done.get(key) == attempt:
                del self.done[key]
        elif kind == "stop":
            return False
        return True

    def serve(self) -> None:
        while self.handle(self.inbox.get()):
            pass


@dataclass
class _Promise:
    event: threading.Event = field(default_factory=threading.Event)
    error: Optional[BaseException] = None


class ExchangeCoordinator:
    """Executor side: the exchanges, run on one comm thread in the driver's order, and the
    readers' barrier (``await_exchange``)."""

    def __init__(self, engine, driver_inbox, my_inbox, register: Optional[Callable[[ShuffleSpec], None]] = None,
                 timeout_s: float = 120.0):
        self.engine = engine
        self.driver = driver_inbox
        self.inbox = my_inbox
        self.timeout_s = timeout_s
        self._registered = set()
        self._register = register or self._register_default
        self._promises: Dict[Key, _Promise] = {}
        self._lock = threading.Lock()
        self._reg_lock = threading.Lock()
        self.ran = []  # keys in the order this executor ran them
        self._thread = threading.Thread(target=self._comm_loop, name="sgx-comm", daemon=True)
        self._thread.start()

    def ensure_registered(self, spec: ShuffleSpec) -> None:
        with self._reg_lock:  # map tasks (writers) and the comm thread register alike
            if spec.shuffle_id in self._registered:
                return
            self._register(spec)
            self._registered.add(spec.shuffle_id)

    def _register_default(self, spec: ShuffleSpec) -> None:
        spec.register(self.engine)

    def _promise(self, key: Key) -> _Promise:
        with self._lock:
            p = self._promises.get(key)
            if p is None:
                p = self._promises[key] = _Promise()
            return p

    def _comm_loop(self) -> None:
        while True:
            msg = self.inbox.get()
            if msg[0] == "stop":
                return
            _, sid, maps, spec, attempt = msg
            key = (sid, tuple(maps))
            p = self._promise(key)
            try:
                try:
                    self.ensure_registered(spec)  # an executor that ran no task of the shuffle
                except BaseException:
                    # the round's collective still needs this rank: join it marked failed
                    # (sgx_exchange_fail raises; the registration is retried next round)
                    self.engine.exchange_fail(spec.num_partitions)
                    raise
                self.engine.exchange(sid)
                self.engine.sync()
                self.ran.append((key, attempt))
            except BaseException as ex:  # noqa: BLE001 - handed to the waiting readers
                # report first, then drop the promise: a reader that asks again only finds no
                # promise once the driver's inbox holds the failure ahead of its new request
                # (one sender's messages stay in order), so the request starts a new round
                # instead of being dropped as a duplicate of the failed one
                self.driver.put(("failed", sid, tuple(maps), attempt))
                with self._lock:
                    if self._promises.get(key) is p:
                        del self._promises[key]  # a later task may ask again
                p.error = ex
            p.event.set()

    def await_exchange(self, spec: ShuffleSpec, all_maps: Sequence[int]) -> None:
        """The reader's barrier: the shuffle's exchange over its full map set has completed on
        this executor (GpuShuffleReader.read -> awaitExchange)."""
        key = (spec.shuffle_id, tuple(sorted(int(m) for m in all_maps)))
        p = self._promise(key)
        if not p.event.is_set():
            self.driver.put(("request", key[0], key[1], spec))
        if not p.event.wait(self.timeout_s):
            # the promise stays: the round may only be slow, and the driver keeps the key as
            # broadcast, so the next reader waits on this one (the comm thread completes it)
            raise _lib.DeviceTimeout(f"exchange of shuffle {spec.shuffle_id} did not complete")
        if p.error is not None:
            raise _lib.IllegalStateException(f"exchange of shuffle {spec.shuffle_id} failed: {p.error}")

    def stop(self) -> None:
        self.inbox.put(("stop",))
        self._thread.join(timeout=10)


def drain(q) -> list:
    """Every message currently queued (test helper)."""
    out = []
    while True:
        try:
            out.append(q.get_nowait())
        except queue.Empty:
            return out
