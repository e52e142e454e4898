#!/usr/bin/env python3
"""Benchmark: shuffled GB/s (partition+exchange) for BASELINE.json's workload.

  python bench.py [--gpus N] [--steps K] [--warmup W]            (N=1 by default)
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

A step is one pass of the hot path over one batch: every rank partitions its own batch of
records resident in HBM (the single-pass padded write: sampled histogram, K4 stable
write-combining scatter into sub-bins, the scan of the true counts on a second stream) and,
for N > 1, pushes it to the reducer owners (lengths all-gather + the direct peer gather into
their IPC-mapped receive buffers over xGMI).  Weak scaling: 2^28 records per GPU (config C1
at N=1; config C2's 2^31 total at N=8).  value = record bytes x records of all ranks /
max-rank time.

Also reported (rank 0): the roofline of the dominant kernel (K4 scatter) from HIP events
on the engine's compute stream over the timed region, the stage breakdown, and the CPU
baseline (the oracle's multi-threaded C restatement, timed on this host on a bounded
sample of the same workload).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "shuffled GB/s (partition+exchange) at 1/2/4/8 GPUs; % of HBM/xGMI roofline"
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8 TB/s spec
ALGO_BYTES_PER_REC = 32    # 16 B read + 16 B write per record
XGMI_LINK_GBS = 153.0      # per directed link; one link per GPU pair


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=["c1", "c3", "c4"], default="c1",
                    help="c1/c2: uniform 16 B records, R=1024 (the default line); c3: Zipf(1.1) keys, "
                         "R=4096; c4: TeraSort 100 B records (10 B keys), RangePartitioner R=1024 with "
                         "bounds sampled from the data (rank 0's batch, sketch on the GPU)")
    ap.add_argument("--records", type=int, default=0,
                    help="records per GPU (default 2^28; c4: 2^25, i.e. C4's 2^28 records at N=8)")
    ap.add_argument("--partitions", type=int, default=0, help="default: 1024 (c3: 4096)")
    ap.add_argument("--dist", choices=["uniform", "zipf"], default=None)
    ap.add_argument("--seed", type=int, default=0x5EEDC0DE)
    ap.add_argument("--num-chunks", type=int, default=0)
    ap.add_argument("--no-split", action="store_true",
                    help="R > 1024: one lane-ordered K4 pass instead of the two-level split (A/B measurement)")
    ap.add_argument("--no-padded", action="store_true",
                    help="hash maps take the two-pass map side (histogram + scan + scatter) instead of the "
                         "single-pass padded write (A/B measurement, DESIGN.md §6.1)")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=16.0,
                    help="budget of the CPU baseline's timed legs (plus ~5 s of C0 and setup)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-live-pmc", action="store_true",
                    help="N=1: skip the two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) that measure this "
                         "run's HBM bytes per launch (roofline.traffic); the committed profiles/pmc_map.json is used")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--comm", choices=["rccl", "host"], default="rccl",
                    help="N > 1 exchange backend: RCCL over xGMI (the product path) or host collectives "
                         "over gloo (lets several ranks share one GPU to rehearse the N > 1 path)")
    ap.add_argument("--placement", choices=["even", "bytes"], default=None,
                    help="N > 1 reducer placement: even (floor(r*P/R); the default) or bytes (contiguous "
                         "ranges balancing each rank's received bytes; the default for c3's skewed keys)")
    ap.add_argument("--self-exchange", action="store_true",
                    help="N=1 only: run every step's exchange through a one-rank RCCL communicator "
                         "(lengths all-gather + the peer gather into its own receive buffer), to measure the "
                         "overlap of map k+1 with the exchange of map k on one GPU (a rehearsal, never the "
                         "default line)")
    ap.add_argument("--compress", action="store_true",
                    help="with --serializer kryo: spark.shuffle.compress=true (LZ4 frames, Spark's default)")
    ap.add_argument("--map-tasks", type=int, default=1,
                    help="N=1 without an exchange: map writes issued by this many concurrent threads "
                         "(Spark runs one map task per executor core; each thread gets its own engine "
                         "stream, so one map's small kernels overlap another's scatter)")
    ap.add_argument("--serializer", choices=["fixed", "kryo"], default="fixed",
                    help="kryo: also frame each map output as Spark's Kryo stream (SURVEY §8(f) row 2)")
    ap.add_argument("--batches", type=int, default=1,
                    help="> 1: every map goes through the writer call sequence Spark drives "
                         "(GpuShuffleWriter: sgx_map_begin, this many sgx_map_append batches -- 2^22 records "
                         "each at C1 with 64 -- as retained device slices of the resident input, "
                         "sgx_map_commit) instead of one sgx_write_map")
    ap.add_argument("--host-batches", action="store_true",
                    help="with --batches: the batches come from pageable host memory (a copy of the input), as "
                         "the JVM writer hands them (SGX_MEM_HOST, staged through the engine's pinned buffers)")
    ap.add_argument("--no-p2p", action="store_true",
                    help="N > 1 / --self-exchange: move the exchange's bytes by RCCL send / recv (or the host "
                         "all-to-all) over contiguous map outputs, with two-pass map writes, instead of the "
                         "direct peer gather out of single-pass padded maps (A/B, DESIGN.md §8)")
    ap.add_argument("--no-overlap-writes", action="store_true",
                    help="SGX_FLAG_NO_OVERLAP_WRITES: every map write on one stream (default: consecutive "
                         "writes alternate between two streams, so one write's K4 starts on the CUs the "
                         "previous one's last workgroups free)")
    ap.add_argument("--roofline-steps", type=int, default=5,
                    help="with overlapping writes: K4 launches timed after the timed region with overlap off, "
                         "for the roofline object (an overlapped launch's interval includes its wait for CUs)")
    a = ap.parse_args()
    a.record_bytes = 100 if a.workload == "c4" else 16
    a.records = a.records or (1 << 25 if a.workload == "c4" else 1 << 28)
    a.partitions = a.partitions or (4096 if a.workload == "c3" else 1024)
    a.dist = a.dist or ("zipf" if a.workload == "c3" else "uniform")
    a.placement = a.placement or ("bytes" if a.workload == "c3" else "even")
    if a.record_bytes != 16 and (a.serializer != "fixed" or a.dist != "uniform"):
        ap.error("c4 (100 B TeraSort records) runs with the fixed codec and its own key generator")
    return a


def _cpu_share():
    """Threads the CPU baseline may use: the affinity mask, capped by a cgroup CPU quota when
    one is set (cgroup v2 cpu.max or v1 cfs quota).  Returns (threads, affinity, quota)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota = None
    for path, parse in (("/sys/fs/cgroup/cpu.max", lambda t: t.split()),
                        ("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", lambda t: [t.strip(), open(
                            "/sys/fs/cgroup/cpu/cpu.cfs_period_us").read().strip()])):
        try:
            with open(path) as f:
                q, per = parse(f.read())
            if q not in ("max", "-1"):
                quota = max(1, int(int(q) / int(per)))
            break
        except (OSError, ValueError):
            continue
    return (min(aff, quota) if quota else aff), aff, quota


def _time_leg(fn, seconds):
    fn()  # warm-up (page faults, thread start)
    t0 = time.perf_counter()
    reps = 0
    while True:
        fn()
        reps += 1
        dt = time.perf_counter() - t0
        if dt >= seconds:
            return reps, dt


def cpu_baseline(args):
    """SURVEY §8(d) CPU baseline: the oracle's C restatement of the map-side write (pthreads:
    per-thread histogram, prefix, stable scatter; oracle/shuffle_oracle.c orc_map_write) on
    bounded samples of the BASELINE configs' per-GPU inputs, with every usable core and with
    one; C0 (groupByKey 2 x 5M -> 200) also runs the reduce-side grouping of the restatement
    (numpy, one thread).  ``value`` is the C1 all-cores leg, the workload of the GPU line."""
    import numpy as np

    import oracle

    threads, aff, quota = _cpu_share()
    per = max(0.5, args.cpu_baseline_seconds / 8.0)
    legs = {}

    def leg(name, recs, R, kind=oracle.PART_HASH, bounds=None):
        rb = recs.shape[1]
        for nt in (threads, 1):
            sample = recs if nt > 1 else recs[: max(1, len(recs) // 4)]
            reps, dt = _time_leg(lambda: oracle.map_write(sample, R, kind, bounds, True, nthreads=nt), per)
            legs[f"{name}_{'all' if nt > 1 else '1'}core"] = {
                "GBs": round(rb * len(sample) * reps / dt / 1e9, 3), "threads": nt, "records": len(sample),
                "record_bytes": rb, "partitions": R, "reps": reps, "seconds": round(dt, 2)}

    n = 1 << 24
    recs = oracle.gen_uniform16(n, args.seed)
    leg("C1_uniform_R1024", recs, 1024)
    del recs
    recs = oracle.gen_zipf16(n, args.seed, oracle.zipf_cdf(1.1, 1 << 24))
    leg("C3_zipf_R4096", recs, 4096)
    del recs
    nt = n * 16 // 100
    recs = oracle.gen_terasort100(nt, args.seed)
    keys = recs[np.random.default_rng(7).choice(nt, 20 * 1024, replace=False), :10]
    keys = keys[np.lexsort(keys.T[::-1])]
    bounds = np.ascontiguousarray(keys[[int(len(keys) / 1024 * (i + 1)) for i in range(1023)]])
    leg("C4_terasort_R1024", recs, 1024, oracle.PART_RANGE_BYTES10, bounds)
    del recs
    # C0: two maps of 5M (Long, Long) records -> 200 reducers, groupByKey on the reduce side
    t0 = time.perf_counter()
    outs = [oracle.map_write(oracle.gen_uniform16(5_000_000, args.seed + m), 200, nthreads=threads) for m in range(2)]
    t1 = time.perf_counter()
    keys_, starts, vals = oracle.reduce_grouped(oracle.canonical_reducer_sequences(outs, 200, 16), "group")
    t2 = time.perf_counter()
    legs["C0_groupByKey_2x5M_R200"] = {"map_side_s": round(t1 - t0, 3), "reduce_group_s": round(t2 - t1, 3),
                                       "records": 10_000_000, "groups": int(len(keys_)),
                                       "threads_map_side": threads, "threads_reduce": 1}
    c1 = legs["C1_uniform_R1024_allcore"]
    return {"value": c1["GBs"], "unit": "GB/s", "cores": threads, "kind": "port",
            "affinity_cores": aff, "cgroup_cpu_quota": quota,
            "sample": f"map-side write (orc_map_write) of {c1['records']} uniform 16 B records, R=1024, "
                      f"{c1['reps']} reps in {c1['seconds']} s on {threads} threads; other legs below",
            "legs": legs}


def load_pmc(dist, n, R, rb=16, padded=True):
    """HBM bytes per launch of K4 and of the whole map side from the committed rocprofv3 PMC
    summary of the same layout (profiles/pmc_map.json, written by tools/summarize_prof.py),
    or None."""
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_map.json")) as f:
            return json.load(f).get(f"{dist}_n{n}_R{R}_rb{rb}" + ("" if padded else "_twopass"))
    except (OSError, ValueError):
        return None


def live_pmc(args):
    """HBM bytes of this workload's map side, measured now: two rocprofv3 --pmc passes
    (FETCH_SIZE, then WRITE_SIZE: one counter per pass, nothing else traced) over
    tools/prof_map.py writing the same records, partitions and layout twice, run as child
    processes before this process touches the GPU.  Per kernel: the median launch's counter
    x launches per write; reads are FETCH_SIZE x 2 KiB (gfx950 counts half of a wide stream,
    MI355X_MICROARCH.md), writes WRITE_SIZE x 1 KiB.  Returns the pmc_map.json shape, or None."""
    import csv
    import glob
    import shutil
    import subprocess
    import tempfile

    exe = shutil.which("rocprofv3")
    if exe is None:
        return None
    flags = 256 if args.no_padded else 0
    if args.no_split:
        flags |= 32  # FLAG_NO_SPLIT_SCATTER (sparkucx_amd is not imported yet)
    cmd_tail = ["--", sys.executable, os.path.join(ROOT, "tools", "prof_map.py"), "--iters", "2",
                "--records", str(args.records), "--partitions", str(args.partitions), "--dist", args.dist,
                "--record-bytes", str(args.record_bytes), "--flags", str(flags), "--num-chunks", str(args.num_chunks),
                "--batches", str(args.batches)]
    per = {}
    tmp = tempfile.mkdtemp(prefix="sgx_pmc_")
    try:
        for counter in ("FETCH_SIZE", "WRITE_SIZE"):
            d = os.path.join(tmp, counter)
            r = subprocess.run([exe, "--pmc", counter, "--output-format", "csv", "-d", d, "-o", "run"] + cmd_tail,
                               stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, timeout=180)
            files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
            if r.returncode != 0 or not files:
                return None
            vals = {}
            for f in files:
                with open(f) as fh:
                    for row in csv.DictReader(fh):
                        if row["Counter_Name"] == counter:
                            k = row["Kernel_Name"].split("(")[0].replace("void ", "").strip()
                            vals.setdefault(k, []).append(float(row["Counter_Value"]))
            per[counter] = vals
    except (OSError, subprocess.SubprocessError):
        return None
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    import statistics

    algo = 2 * args.record_bytes * args.records
    side = {"read": 0.0, "write": 0.0}
    k4 = {"kernel": None, "hbm_bytes_per_launch": 0, "read_bytes": 0, "write_bytes": 0, "algorithmic_bytes": algo}
    names = set(per["FETCH_SIZE"]) | set(per["WRITE_SIZE"])
    for k in sorted(names):
        if k.replace("sgx::", "").startswith(("k_gen", "k_lds_order_probe")):
            continue  # the input generator; the engine-start LDS ordering check
        f, w = per["FETCH_SIZE"].get(k, []), per["WRITE_SIZE"].get(k, [])
        calls = max(len(f), len(w)) / 2.0  # launches per write (two writes)
        rd = statistics.median(f) * 2 * 1024 if f else 0.0
        wr = statistics.median(w) * 1024 if w else 0.0
        side["read"] += rd * calls
        side["write"] += wr * calls
        if k.replace("sgx::", "").startswith("k_scatter") and rd + wr > 1e6:  # (not the guarded fallback's no-op)
            k4["kernel"] = k if k4["kernel"] is None else k4["kernel"] + " + " + k
            k4["hbm_bytes_per_launch"] += int((rd + wr) * calls)
            k4["read_bytes"] += int(rd * calls)
            k4["write_bytes"] += int(wr * calls)
    tot = side["read"] + side["write"]
    return {"scatter": k4, "map_side": {"hbm_bytes_per_write": int(tot), "read_bytes": int(side["read"]),
                                        "write_bytes": int(side["write"]), "algorithmic_bytes": algo,
                                        "ratio": round(tot / algo, 4)},
            "source": "live: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over tools/prof_map.py in this bench run"}


def _exchange_name(args, world, self_x):
    if world == 1 and not self_x:
        return None
    ctl = "RCCL" if args.comm == "rccl" or self_x else "host collectives (gloo)"
    if args.no_p2p:
        data = "RCCL grouped send/recv" if ctl == "RCCL" else "host all-to-all"
    else:
        data = "direct peer gather (IPC-mapped receive buffers)"
    return f"{data}, {ctl} control" + (", 1 rank (rehearsal)" if self_x else
                                       " (rehearsal: ranks share one GPU)" if args.comm == "host" else "")


def _workload_name(args, n, R, world, self_x):
    x = _exchange_name(args, world, self_x)
    if args.workload == "c4":
        w = f"C4: {n} x 100 B TeraSort records per GPU, RangePartitioner R={R} (sampled bounds), partition+scatter"
    elif args.workload == "c3":
        w = f"C3: {n} x 16 B Zipf(1.1) records per GPU, HashPartitioner R={R}, partition+scatter"
    elif world == 1:
        w = "C1: 2^28 x 16 B, HashPartitioner R=1024, partition+scatter per GPU" if (n, R) == (1 << 28, 1024) else \
            f"C1-shaped: {n} x 16 B, HashPartitioner R={R}, partition+scatter per GPU"
    else:
        w = f"C2: {n} x 16 B per GPU ({n * world} total), R={R}, partition"
    return w + (f" + {x}" if x else "")


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE", file=sys.stderr)
    # this run's HBM bytes first, in child processes, before this one touches the GPU
    live = None
    if world == 1 and not args.no_live_pmc and args.serializer == "fixed" and not args.self_exchange:
        live = live_pmc(args)
    import numpy as np
    import torch

    import sparkucx_amd as sgx

    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("gloo", rank=rank, world_size=world)
    device = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(device)

    n, R, rb = args.records, args.partitions, args.record_bytes
    eng = sgx.ShuffleEngine(device=device, num_chunks=args.num_chunks,
                            flags=(sgx.FLAG_NO_SPLIT_SCATTER if args.no_split else 0) |
                            (sgx.FLAG_NO_PADDED_MAP if args.no_padded else 0) |
                            (sgx.FLAG_NO_P2P_EXCHANGE if args.no_p2p else 0) |
                            (sgx.FLAG_NO_OVERLAP_WRITES if args.no_overlap_writes else 0))
    self_x = args.self_exchange and world == 1
    if world > 1 and args.comm == "host":
        eng.comm_init_host(world, rank)
    elif self_x:
        eng.comm_init(1, 0, sgx.get_unique_id())
    elif world > 1:
        uid = [sgx.get_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        eng.comm_init(world, rank, uid[0])
    buf = eng.alloc(n * rb)
    bounds = None
    if rb == 100:
        # TeraSort: 10 random key bytes + a 90 B payload; RangePartitioner bounds from the
        # data (RangePartitioner.sketch + determineBounds, the GPU sketch), computed on rank 0
        # and shared, as Spark's driver does
        eng.gen_terasort100(buf, n, args.seed + rank, index_base=rank * n)
        bl = [eng.range_bounds([buf], [n], 100, R) if rank == 0 else None]
        if dist is not None:
            dist.broadcast_object_list(bl, src=0)
        bounds = bl[0]
    elif args.dist == "uniform":
        eng.gen_uniform16(buf, n, args.seed + rank, value_base=rank * n)
    else:
        ranks = np.arange(1, (1 << 24) + 1, dtype=np.float64)
        cdf = np.cumsum(ranks ** -1.1)
        cdf /= cdf[-1]
        eng.gen_zipf16(buf, n, args.seed + rank, cdf, value_base=rank * n)
    sid = 1
    if rb == 100:
        eng.register_shuffle(sid, R, sgx.PART_RANGE_BYTES10, bounds, True, 100)
    else:
        eng.register_shuffle(sid, R, serializer=sgx.SER_KRYO if args.serializer == "kryo" else sgx.SER_FIXED)
    if args.placement == "bytes":
        eng.set_reducer_placement(sid, "bytes")
    if args.compress:
        if args.serializer != "kryo":
            raise SystemExit("--compress needs --serializer kryo (spark.shuffle.compress applies to serialized streams)")
        eng.set_compression(sid, "lz4")

    last = {"mid": None}  # the map the last step wrote (read back by the Kryo leg below)
    # concurrent map tasks (N = 1, no exchange): task j writes steps j, j + T, ... into its own
    # map slot on its own thread, i.e. its own engine stream
    tasks = args.map_tasks if (world == 1 and not self_x) else 1
    slots = max(2, tasks)

    nbatch = max(1, args.batches)
    cuts = [n * j // nbatch for j in range(nbatch + 1)]
    host = None
    if args.host_batches:
        if nbatch == 1:
            raise SystemExit("--host-batches needs --batches > 1")
        host = buf.to_numpy(n * rb)  # pageable host copy of the input (not timed)

    def step(k):
        mid = (k % slots) * world + rank  # alternating map slots per rank (one per task)
        if nbatch == 1:
            eng.write_map(sid, mid, buf, n, rb)
        else:
            # GpuShuffleWriter's sequence: begin, the batches (device slices the caller keeps
            # until the commit), commit -- one pass over every batch at the commit
            eng.map_begin(sid, mid)
            for j in range(nbatch):
                if host is not None:
                    eng.map_append(sid, mid, host[cuts[j] * rb:cuts[j + 1] * rb], cuts[j + 1] - cuts[j], rb)
                else:
                    eng.map_append(sid, mid, buf, cuts[j + 1] - cuts[j], rb, offset=cuts[j] * rb, retained=True)
            eng.map_commit(sid, mid)
        if args.compress:
            # the map task commits: its partition lengths, i.e. the LZ4 framing of its Kryo
            # streams, which the engine does when the lengths are first needed -- inside the step,
            # as Spark's map task does before it ends
            eng.map_lengths(sid, mid, R)
        if world > 1 or self_x:
            # this step's map through the shuffle's exchange (sgx_exchange_maps: the pipelined
            # form -- the all-to-all of map k runs on the exchange stream while map k+1 is
            # written on the compute stream)
            eng.exchange(sid, [mid])
        last["mid"] = mid

    def barrier():
        if dist is not None:
            dist.barrier()
        eng.sync()
        torch.cuda.synchronize()

    pool = None
    if tasks > 1:
        import concurrent.futures as cf

        pool = cf.ThreadPoolExecutor(max_workers=tasks)

    def run(nsteps):
        if pool is None:
            for k in range(nsteps):
                step(k)
            return
        # one job per task: its steps in order, all in its own slot; a job the pool runs on an
        # already-busy thread just serializes (the barriers separate the phases' slot reuse)
        jobs = [pool.submit(lambda j=j: [step(k) for k in range(j, nsteps, tasks)]) for j in range(tasks)]
        for f in jobs:
            f.result()

    run(max(args.warmup, tasks))
    barrier()
    eng.stats_reset()
    barrier()
    t0 = time.perf_counter()
    run(args.steps)
    barrier()
    dt = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    st = eng.stats()
    # The K4 roofline from launches that do not overlap.  With overlapping writes
    # (the engine's default) a K4 is dispatched while the previous one's last workgroups still
    # run, so its HIP-event interval -- and its rocprofv3 duration -- include the wait for their
    # CUs: the timed region gives the throughput, these launches the kernel's own time.
    k4_alone = None
    if (not args.no_overlap_writes and world == 1 and not self_x and tasks == 1 and args.roofline_steps > 0
            and args.serializer == "fixed"):
        eng.set_overlap_writes(False)
        run(2)
        barrier()
        eng.stats_reset()
        run(args.roofline_steps)
        barrier()
        st_alone = eng.stats()
        eng.set_overlap_writes(True)
        k4_alone = st_alone.ms["scatter"] / max(1, st_alone.count["scatter"])

    verified = None
    lens = eng.map_lengths(sid, rank, R)
    layout = eng.map_layout(sid, last["mid"])
    if not args.no_verify:
        verified = bool(lens.sum() == rb * n) if args.serializer == "fixed" else bool(lens.sum() >= 4 * n)
    xgmi = None
    xbytes = None
    if world > 1 or self_x:
        # what the exchange moved against the blocks' lengths: the peer gather sends a padded
        # map's blocks from its fragments, so exactly the lengths (no sub-bin slack)
        xb = eng.exchange_bytes()
        t = torch.tensor([xb["sent"], xb["kept"], float(lens.sum()) * args.steps], dtype=torch.float64)
        if dist is not None:
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
        xbytes = {"sent_to_peers": float(t[0]), "kept_local": float(t[1]), "published": float(t[2]),
                  "moved_over_published": round(float((t[0] + t[1]) / max(t[2], 1.0)), 6),
                  "rounds_per_rank": xb["rounds"]}
    if world > 1:
        # bytes this rank's map sends over xGMI (reducer r lives on rank floor(r*P/R))
        r0, r1 = eng.shuffle_reducers(sid)  # this rank's reducers (fixed by the shuffle's first round)
        rr = torch.tensor([r0, r1], dtype=torch.int64)
        allr = [torch.zeros(2, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(allr, rr)
        owner = np.zeros(R, dtype=np.int64)
        for j, t in enumerate(allr):
            owner[int(t[0]):int(t[1])] = j
        sent = float(lens[owner != rank].sum())
        a2a_ms = st.ms["alltoall"] / max(1, st.count["alltoall"])
        # bytes each rank receives (load balance of the reducer ranges, config C3)
        recv = torch.zeros(world, dtype=torch.float64)
        for j in range(world):
            recv[j] = float(lens[owner == j].sum())
        dist.all_reduce(recv, op=dist.ReduceOp.SUM)
        t = torch.tensor([sent, a2a_ms], dtype=torch.float64)
        tmax = t.clone()
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        peak = XGMI_LINK_GBS * world * (world - 1)
        ach = float(t[0]) / (float(tmax[1]) * 1e-3) / 1e9
        xgmi = {"bound": "xgmi", "achieved": round(ach, 1), "peak": peak, "unit": "GB/s",
                "frac": round(ach / peak, 4), "bytes_per_step": float(t[0]),
                "alltoall_ms_max_rank": round(float(tmax[1]), 4),
                "recv_bytes_max_over_mean": round(float(recv.max() / recv.mean()), 4),
                "note": "all ranks' cross-GPU bytes / slowest rank's ncclAllToAllv time; peak = P(P-1) x 153 GB/s"}

    if rank == 0:
        ms_per_step = dt * 1e3 / args.steps
        total_bytes = float(rb) * n * world * args.steps
        value = total_bytes / dt / 1e9
        sc_ms_timed = st.ms["scatter"] / max(1, st.count["scatter"])
        sc_ms = k4_alone if k4_alone is not None else sc_ms_timed
        algo = 2 * rb  # the record read once and written once
        achieved = algo * n / (sc_ms * 1e-3) / 1e9
        padded = layout in (sgx.LAYOUT_PADDED, sgx.LAYOUT_SERIALIZED_PADDED)
        pmc = live or load_pmc(args.dist if rb == 16 else "terasort", n, R, rb, padded) or {}
        k4_pmc, side_pmc = pmc.get("scatter") or {}, pmc.get("map_side") or {}
        side_ms = (st.ms["hist"] + st.ms["scan"] + st.ms["scatter"]) / max(1, st.count["scatter"])
        side_src = "stage events (K1+K2 / sample, K3, K4)"
        if layout == sgx.LAYOUT_PADDED:
            # the padded write's K3 runs on its tail stream beside the next write (its stage
            # interval spans the next map's kernels): the write is the sample and K4
            side_ms = (st.ms["hist"] + st.ms["scatter"]) / max(1, st.count["scatter"])
            side_src = "stage events (sample, K4; the tail's K3 overlaps the next write)"
        if world == 1 and not self_x and tasks == 1 and not args.compress and args.serializer == "fixed" and host is None:
            # a step is exactly one map write: its wall time is the map side as a map task sees
            # it, host calls included -- the padded write's tail (K3 + the guarded fallback) runs
            # on a second stream behind K4 and overlaps the next write, so its stage interval
            # would count time the next map's kernels use
            side_ms, side_src = ms_per_step, "timed step (one map write per step)"
        side_ach = algo * n / (side_ms * 1e-3) / 1e9
        out = {
            "metric": METRIC, "value": round(value, 2), "unit": "GB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int64",
            "data": (f"synthetic {args.dist} (Long,Long) 16 B records, splitmix64 seed {args.seed:#x}+rank"
                     if rb == 16 else f"synthetic TeraSort 100 B records (10 random key bytes), seed {args.seed:#x}+rank, "
                     f"{len(bounds)} bounds sampled from rank 0's batch"),
            "config": {"workload": _workload_name(args, n, R, world, self_x), "map_tasks": tasks,
                       "writer": "sgx_write_map (one batch)" if nbatch == 1 else (
                           f"sgx_map_begin + {nbatch} x sgx_map_append (~{n // nbatch} records each, " +
                           ("pageable host batches" if host is not None else "retained device batches") +
                           ") + sgx_map_commit"),
                       "map_tasks_note": None if tasks == 1 else (
                           "concurrent map tasks: stage event times include the other tasks' kernels, "
                           "so the roofline fields are not per-kernel figures (DESIGN.md §9)"),
                       "records_per_gpu": n, "partitions": R, "record_bytes": rb,
                       "map_layout": "padded (single pass: sampled histogram, K4 into sub-bins, K3 over the "
                                     "streams' counts)" if padded else "contiguous (two-pass: K1+K2 histogram, K3, K4)",
                       "parallelism": f"dp{world} (map shards per GPU, reducers owned "
                                      + ("floor(r*P/R))" if args.placement == "even" else "in byte-balanced ranges)"),
                       "exchange": _exchange_name(args, world, self_x),
                       "overlap_writes": not args.no_overlap_writes},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": k4_pmc.get("hbm_bytes_per_launch"),
                         "kernel": k4_pmc.get("kernel", "K4 scatter"), "algo_bytes_per_record": algo,
                         "traffic_source": pmc.get("source"),
                         "launch_ms": round(sc_ms, 4),
                         "launch_ms_source": (f"{args.roofline_steps} K4 launches right after the timed region, "
                                              "overlapping writes off (HIP events on K4's stream)")
                         if k4_alone is not None else "the timed region's K4 launches (HIP events on K4's stream)",
                         "timed_region_k4_interval_ms": round(sc_ms_timed, 4)},
            # the whole map side (K1+K2 histogram, K3 scan, K4 scatter, their memsets) against
            # the same 32 B/record: what north_star's partition+scatter target is quoted on
            "roofline_map_side": {"bound": "hbm", "achieved": round(side_ach, 1), "peak": HBM_PEAK_GBS,
                                  "unit": "GB/s", "frac": round(side_ach / HBM_PEAK_GBS, 4),
                                  "ms": round(side_ms, 4), "ms_source": side_src, "algo_bytes_per_record": algo,
                                  "traffic": side_pmc.get("hbm_bytes_per_write"),
                                  "traffic_over_algorithmic": side_pmc.get("ratio")},
            "stages_ms_per_step": {k: round(v / max(1, st.count[k]), 4) for k, v in st.ms.items() if st.count[k]},
            "stages_note": ("HIP-event intervals per stage on the stage's own stream; with overlapping writes a "
                            "stage's interval includes its wait for the CUs the previous write's K4 holds (hist = the "
                            "pad sample), so they do not add up to ms_per_step (DESIGN.md §6.1)")
            if padded and not args.no_overlap_writes else "HIP-event intervals per stage",
            # the HBM bytes the map side's design must move per record -- two-pass: 3 x record
            # bytes (the histogram reads the whole record for its 8 B key; K4 reads + writes it);
            # padded: 2 x record bytes + the sampled lines (one 128 B line in 128) -- as a
            # stream rate against 8 TB/s
            "map_side_design_hbm": (lambda bpr: {"bytes_per_record": bpr, "achieved": round(bpr * n / side_ms / 1e6, 1),
                                                 "frac": round(bpr * n / side_ms / 1e6 / HBM_PEAK_GBS, 4)})(
                (2 * rb + rb / 128.0) if padded else 3 * rb),
            "verified_lengths_sum": verified,
        }
        if xgmi is not None:
            out["xgmi_roofline"] = xgmi
        if xbytes is not None:
            out["exchange_bytes"] = xbytes
            # the whole step against HBM: the map side's design bytes plus the exchange reading
            # every published byte once and writing it once into a reducer's buffer (per GPU,
            # over the timed step: on one GPU the gather shares HBM with the next map's K4, so
            # the map side's own stage figure is stretched and this is the step's roofline)
            bpr = (2 * rb + rb / 128.0) if padded else 3 * rb
            per_gpu = bpr * n + 2.0 * xbytes["published"] / args.steps / world
            ach = per_gpu / (ms_per_step * 1e-3) / 1e9
            out["step_design_hbm"] = {"bytes_per_gpu_step": per_gpu, "achieved": round(ach, 1),
                                      "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                                      "note": "map side design bytes + 2 x published bytes, per GPU, / ms_per_step"}
        if host is not None:
            # the whole step is the writer's ingest: host batches -> pinned -> HBM, then the
            # commit's one pass; the map side alone is in roofline_map_side's stage figures
            out["host_ingest"] = {"GBs": round(rb * n / (ms_per_step * 1e-3) / 1e9, 2), "bytes_per_step": rb * n,
                                  "note": "pageable host batches through two pinned staging buffers (64 MiB pieces), "
                                          "H2D overlapping the next batch's staging copy"}
        if args.serializer == "kryo":
            ser_ms = st.ms["serialize"] / max(1, st.count["serialize"])
            kbytes = float(lens.sum())
            out["config"]["serializer"] = ("KryoSerializer, spark.shuffle.compress=" +
                                           ("true (lz4, 32 KiB blocks)" if args.compress else "false"))
            out["kryo"] = {"kernel": "k_kryo_ser16", "ms": round(ser_ms, 4), "published_bytes": kbytes,
                           "achieved_GBs": round(16.0 * n / (ser_ms * 1e-3) / 1e9, 1)}
            if args.compress:
                c_ms = st.ms["compress"] / max(1, st.count["compress"])
                out["lz4"] = {"kernel": "k_lz4_blocks", "ms": round(c_ms, 4), "framed_bytes": kbytes,
                              "note": "k_lz4_blocks + k_xxh32_blocks: one wave per 32 KiB block, LZ4_compress_default's "
                                      "search 64 positions per batch, several sequences per batch (DESIGN.md §13)"}
            if world == 1:
                # reduce side of the same shuffle: every block of the last map, decoded on the GPU
                dst = eng.alloc(n * 16)
                last_mid = last["mid"]
                for _ in range(3):
                    eng.stats_reset()
                    eng.read_records(sid, [last_mid], 0, R, dst=dst)
                st2 = eng.stats()
                de_ms = st2.ms["deserialize"] / max(1, st2.count["deserialize"])
                out["kryo"]["deserialize"] = {
                    "kernel": "k_kryo_deser16", "ms": round(de_ms, 4),
                    "achieved_GBs": round(16.0 * n / (de_ms * 1e-3) / 1e9, 1),
                    "gather_ms": round(st2.ms["regroup"] / max(1, st2.count["regroup"]), 4)}
                if args.compress:
                    out["lz4"]["decompress_ms"] = round(st2.ms["decompress"] / max(1, st2.count["decompress"]), 4)
                dst.free()
        if world == 1 and args.serializer == "fixed" and rb == 16:
            # the consumer side of the layout: every block of the last map gathered reducer by
            # reducer into HBM (sgx_fetch_blocks; a padded map's blocks come from its
            # fragments, a contiguous map's from one range each)
            dst = eng.alloc(n * rb)
            # one untimed call first: the process's first launch of the gather kernel loads
            # its code object (milliseconds, inside the stage's events)
            eng.fetch_blocks(sid, [last["mid"]] * R, list(range(R)), dst=dst)
            eng.stats_reset()
            for _ in range(3):
                eng.fetch_blocks(sid, [last["mid"]] * R, list(range(R)), dst=dst)
            st2 = eng.stats()
            g_ms = st2.ms["regroup"] / max(1, st2.count["regroup"])
            out["fetch_all_blocks"] = {"kernel": "k_gather_frags" if padded else "k_gather_items", "ms": round(g_ms, 4),
                                       "achieved_GBs": round(algo * n / (g_ms * 1e-3) / 1e9, 1),
                                       "note": "R blocks of one map into device memory, read + write per record"}
            dst.free()
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args)
        elif world == 1:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    eng.unregister_shuffle(sid)
    buf.free()
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
