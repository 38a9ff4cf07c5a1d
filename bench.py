"""Benchmark: partitioned pattern query on MI355X (BASELINE.json configs[1] "C2" at N=1, configs[4] "C5"
at N>1).

    every e1=StockStream[price > 20] -> e2=StockStream[price > e1.price] within 10 sec
    partition with (symbol of StockStream)
    N = 1: 1,048,576 synthetic keys (C2);  N > 1: 2^23 keys per GPU (C5: 64M keys on 8 GPUs)

A step = one micro-batch of 2^24 synthetic stock ticks per GPU (already resident in HBM) pushed
through the C-ABI (key grouping + NFA advance) and polled (matches ordered by trigger seq, left in
HBM).  `value` = input events/sec of the whole job (all ranks).

N > 1: one process per GPU.  The global stream is arrival ordered (16,000 events per ms at N=8); each
rank holds a contiguous slice of every step (2^24 events); the slice is resharded by key without any
host synchronisation (HIP stable pack into fixed-size destination blocks, one equal-split RCCL
all_to_all over xGMI, unpack into a padded batch whose padding the engine drops as null-key events:
siddhi-1_amd/reshard.py BlockResharder), and each rank runs its engine on the keys it owns
(weak scaling: keys and events per GPU fixed).  The engine's stream waits for the exchange on the
device (sg_wait_stream); every timed step pushes one resharded slice and reshards the next one while
the engine works on it.

The roofline object prices the NFA advance kernel with the algorithmic byte model of DESIGN.md
 over its HIP-event-timed duration.  cpu_baseline times the CPU oracle (the
single-threaded restatement of the reference engine) on a bounded prefix of the same stream.
At N=1 `other_configs` adds BASELINE configs[2] (C3, counting + logical sequence) and configs[3]
(C4, absent state, playback clock) on the general device engine.
"""
import argparse
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)


def algorithmic_bytes(st):
    """16 B/event in + 16 B per touched key header (r+w) + 2*16 B per live partial of a
    touched key at batch start + 16 B per new partial + 24 B per emitted match."""
    return (16 * st["events"] + 16 * st["keys_touched"] + 32 * st["live_at_batch_start"]
            + 16 * st["partials_created"] + 24 * st["matches"])


def pmc_traffic_general(cfg, summary="pmc_traffic_general.json"):
    """NFA-kernel HBM bytes per pushed batch of a general-engine config (or, from pmc_traffic_variants.json, of a
    C2 workload variant: every advance kernel of the push) from the committed PMC summary
    (tools/pmc_general_summary.py), only when it was measured on these exact kernel sources; (None, None)
    otherwise"""
    try:
        import hashlib
        t = json.load(open(os.path.join(ROOT, "tools", summary)))
        h = hashlib.sha1()
        for f in t["sources"]:
            h.update(open(os.path.join(ROOT, "siddhi-1_amd", "csrc", f), "rb").read())
        if t.get("kernel_src_sha1") == h.hexdigest() and cfg in t["configs"]:
            return t["configs"][cfg]["traffic_bytes_per_step"], t["profiles"]
    except (OSError, ValueError, KeyError):
        pass
    return None, None


def pmc_traffic():
    """HBM bytes per launch of the advance kernel from the committed PMC summary (tools/pmc_summary.py),
    only when it was measured on this exact kernel source; None otherwise."""
    try:
        import hashlib
        t = json.load(open(os.path.join(ROOT, "tools", "pmc_traffic.json")))
        src = open(os.path.join(ROOT, "siddhi-1_amd", "csrc", "p2_jit.hip"), "rb").read()
        if t.get("kernel_src_sha1") == hashlib.sha1(src).hexdigest():
            return t["traffic_bytes_per_launch"], t["profiles"]
    except (OSError, ValueError, KeyError):
        pass
    return None, None


def delta(a, b):
    return {k: b[k] - a[k] for k in a}


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def distinct_cores(n):
    """up to n CPUs of this process's affinity mask, spread over the L3 caches first (round-robin over the
    L3 domains: the oracle's per-shard state is tens of MB, and threads that share an L3 evict each other's)
    and on distinct physical cores (one SMT sibling each); [] when the mask does not hold n such cores"""
    def rd(path):
        with open(path) as f:
            return f.read().strip()
    try:
        seen, groups = set(), {}
        for c in sorted(os.sched_getaffinity(0)):
            base = f"/sys/devices/system/cpu/cpu{c}/"
            core = (rd(base + "topology/physical_package_id"), rd(base + "topology/core_id"))
            if core in seen:
                continue
            seen.add(core)
            try:
                l3 = rd(base + "cache/index3/id")
            except OSError:
                l3 = core[0]
            groups.setdefault((core[0], l3), []).append(c)
        out, lists = [], [g for _, g in sorted(groups.items())]
        while len(out) < n and any(lists):
            for g in lists:
                if g and len(out) < n:
                    out.append(g.pop(0))
        return out if len(out) >= n else []
    except (AttributeError, OSError):
        return []


def cpu_quota():
    """CPUs this process may use: the cgroup v2 quota (cpu.max), the affinity mask, whichever is smaller"""
    q = None
    try:
        lim, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if lim != "max":
            q = float(lim) / float(per)
    except (OSError, ValueError):
        pass
    try:
        aff = len(os.sched_getaffinity(0))
        q = min(q, aff) if q else aff
    except (AttributeError, OSError):
        pass
    return q


def keep_heap():
    """glibc: freed memory stays in the arenas (no trim), and blocks up to 32 MB come from the arenas instead of
    one mmap each: the oracle's per-push temporaries then reuse pages instead of faulting fresh ones, and the
    partition-parallel threads do not serialise on the process's memory-map lock (page faults, munmap)"""
    try:
        import ctypes
        libc = ctypes.CDLL("libc.so.6")
        libc.mallopt(-1, 1 << 30)          # M_TRIM_THRESHOLD
        libc.mallopt(-2, 256 << 20)        # M_TOP_PAD
        libc.mallopt(-3, 32 << 20)         # M_MMAP_THRESHOLD (glibc's maximum)
    except (OSError, AttributeError):
        pass


def two_phase(T, pins, body):
    """T persistent threads (thread r pinned to pins[r]) run body(r, 0) untimed, meet at a barrier, then run
    body(r, 1) timed; returns (timed wall seconds, per-thread busy seconds).  The same thread runs both halves
    of its shards: glibc gives each thread an arena of its own, and a thread started later can inherit another
    thread's arena, so a fresh thread per half would free the first half's blocks into arenas other threads
    allocate from (arena-lock contention, remote NUMA memory) -- the timed half would measure the allocator"""
    import threading
    busy, err = [0.0] * T, []
    ready, go = threading.Barrier(T + 1), threading.Barrier(T + 1)

    def work(r):
        try:
            if pins:
                os.sched_setaffinity(0, {pins[r]})   # (the calling thread)
            body(r, 0)
        except BaseException as e:   # noqa: BLE001 (re-raised on the main thread)
            err.append(e)
        ready.wait()
        go.wait()
        if err:
            return
        try:
            t = time.perf_counter()
            body(r, 1)
            busy[r] = time.perf_counter() - t
        except BaseException as e:   # noqa: BLE001
            err.append(e)

    th = [threading.Thread(target=work, args=(r,)) for r in range(T)]
    for x in th:
        x.start()
    ready.wait()
    t0 = time.perf_counter()
    go.wait()
    for x in th:
        x.join()
    el = time.perf_counter() - t0
    if err:
        raise err[0]
    return el, busy


def cpu_baseline(sa, synth, n_keys, batch, seconds):
    """SURVEY §8(d) CPU legs, the CPU oracle (the C++ restatement of the reference engine; the reference
    JVM is not runnable here or on the box) on the host cores of the GPU box:
      (i)  faithful single thread on the first events of the same C2 stream (the reference serialises a
           pattern query on one lock, so one core is its own parallelism for this query) -> `value`;
      (ii) partition-parallel: T threads, keys sharded key % T, one oracle engine per thread over the
           same prefix of the stream (an upper bound for any CPU engine; T = the box's CPU share);
      (iii) C1 (BASELINE configs[0]): the unpartitioned query, one key, 1 event per ms, single thread.
    Each leg is bounded to about `seconds` of CPU work."""
    import threading
    from oracle_backend import build_oracle
    keep_heap()
    lib = build_oracle()
    app = sa.parse_app(synth.C2_QUERY)
    cq = sa.compile_query(app, app.queries[0], sa.StringDictionary())
    eng = sa.NativeEngine(lib, "sgo_", cq.ir, n_keys=n_keys)
    chunk = 1 << 19
    done, busy = 0, 0.0
    while busy < seconds and done < batch * 4:
        d = synth.stock_ticks(done, chunk, n_keys)
        t = time.perf_counter()
        eng.push(0, done, d["ts"], [d["symbol"], d["price"], d["volume"]], None, d["key"])
        eng.poll()
        busy += time.perf_counter() - t
        done += chunk
    eng.close()
    single = done / busy
    # (ii) partition-parallel over the box's CPU share: the cgroup CPU quota when there is one, else
    # OMP_NUM_THREADS (set to the GPU's share on the GPU boxes), else nproc.  One oracle engine per thread;
    # the chunks are cut contiguous before the timed region, so each thread's loop is two foreign calls per
    # chunk (ctypes drops the GIL around them) and the threads share nothing but the allocator.
    quota = cpu_quota()
    T = max(1, int(quota) if quota else int(os.environ.get("OMP_NUM_THREADS", 0)) or (os.cpu_count() or 1))
    T = int(os.environ.get("SG_CPU_THREADS", T))   # (tools/cpu_leg.py: scaling sweeps)
    total = int(min(batch * 4, single * seconds * T * 0.5)) // (T * chunk) * (T * chunk) or T * chunk
    d = synth.stock_ticks(0, total, n_keys)
    # S = 4T key shards (key % S), one oracle engine each, four per thread (a shard's chunks run in order on
    # its thread)
    S = 4 * T
    own = d["key"] % np.uint32(S)
    # each shard's events in two halves: the first half runs untimed (the engines' state reaches its
    # steady size — the 10 s windows fill — and its memory is faulted in), the second half is timed
    shards = []
    for r in range(S):
        idx = np.nonzero(own == r)[0]
        ts, key = d["ts"][idx], (d["key"][idx] // np.uint32(S)).astype(np.uint32)
        cols = [d["symbol"][idx], d["price"][idx], d["volume"][idx]]
        h = len(idx) // 2
        shards.append([[(a, np.ascontiguousarray(ts[a:min(a + chunk, hi)]),
                         [np.ascontiguousarray(c[a:min(a + chunk, hi)]) for c in cols],
                         np.ascontiguousarray(key[a:min(a + chunk, hi)])) for a in range(lo, hi, chunk)]
                       for lo, hi in ((0, h), (h, len(idx)))])
    del d
    timed = sum(len(x[1]) for sh in shards for x in sh[1])

    def run_shard(e, part):
        for a, ts, cols, key in part:   # local arrival seqs (the per-key order is the global one)
            e.push(0, a, ts, cols, None, key)
            e.discard()

    # each thread on a physical core of its own, spread over the L3 domains: the quota counts CPUs, two
    # threads on SMT siblings share a core, and threads sharing an L3 thrash it (a shard's state is tens of
    # MB at 2^20 keys: one thread alone has the whole L3).  Every engine is created by the thread that runs
    # it, so its memory is first touched on that core's NUMA node.
    pins = [] if os.environ.get("SG_CPU_NOPIN") else distinct_cores(T)
    engs = [None] * S

    def make(sh):
        engs[sh] = sa.NativeEngine(lib, "sgo_", cq.ir, n_keys=(n_keys + S - 1) // S)
        return engs[sh]

    # one thread alone on shard 0 (its own engine, on the first pinned core): the per-thread rate of this
    # same sample.  The single-thread `value` above runs the stream's first seconds, before the 10 s windows
    # fill, and is faster per event than the steady state here, so scaling is measured against this instead
    alone = [0.0]

    def solo():
        if pins:
            os.sched_setaffinity(0, {pins[0]})
        e0 = sa.NativeEngine(lib, "sgo_", cq.ir, n_keys=(n_keys + S - 1) // S)
        run_shard(e0, shards[0][0])
        t = time.perf_counter()
        run_shard(e0, shards[0][1])
        alone[0] = sum(len(x[1]) for x in shards[0][1]) / (time.perf_counter() - t)
        e0.close()

    th0 = threading.Thread(target=solo)
    th0.start()
    th0.join()
    alone = alone[0]
    # thread r owns shards r, r + T, ... in both halves: an engine's memory is allocated and freed by one thread
    def body(r, half):
        for sh in range(r, S, T):
            run_shard(engs[sh] if half else make(sh), shards[sh][half])

    el, busy = two_phase(T, pins, body)
    par = timed / el
    # each thread's own rate on its shards (events / its busy time) against the one thread alone: the wall-clock
    # value above is set by the slowest thread, and on a shared host one pinned core can be slowed by other work
    ev_r = [sum(len(x[1]) for sh in range(r, S, T) for x in shards[sh][1]) for r in range(T)]
    thr_vs_alone = [round(ev_r[r] / busy[r] / alone, 3) if busy[r] > 0 else None for r in range(T)]
    for e in engs:
        e.close()
    # (iii) C1: unpartitioned, one key, R = 1 event per ms (10,000 events per 10 s window)
    app1 = sa.parse_app(synth.C1_QUERY)
    cq1 = sa.compile_query(app1, app1.queries[0], sa.StringDictionary())
    e1 = sa.NativeEngine(lib, "sgo_", cq1.ir, n_keys=1)
    c1_done, c1_busy, c1_chunk = 0, 0.0, 1 << 16
    while c1_busy < seconds / 2 and c1_done < 10_000_000:
        d = synth.stock_ticks(c1_done, c1_chunk, 1, rate_per_ms=1)
        t = time.perf_counter()
        e1.push(0, c1_done, d["ts"], [d["symbol"], d["price"], d["volume"]])
        e1.poll()
        c1_busy += time.perf_counter() - t
        c1_done += c1_chunk
    e1.close()
    return {"value": single, "unit": "events/s", "cores": 1, "kind": "port",
            "sample": f"first {done} events of the C2 stream ({n_keys} keys), CPU oracle (faithful single-thread "
                      f"restatement of the reference engine; reference JVM unavailable on the box)",
            "cpu_model": cpu_model(), "nproc": os.cpu_count(),
            "partition_parallel": {"value": par, "unit": "events/s", "threads": T, "cpu_quota": quota,
                                   "one_thread_same_sample": alone,
                                   "pinned_cpus": pins,
                                   "per_thread_scaling": par / alone / T,
                                   "per_thread_rate_vs_alone": thr_vs_alone,
                                   "median_thread_vs_alone": sorted(x for x in thr_vs_alone if x is not None)[T // 2]
                                   if any(x is not None for x in thr_vs_alone) else None,
                                   "vs_single_prefix": par / single / T,
                                   "thread_busy_s": [round(b, 3) for b in busy],
                                   "sample": f"first {total} events of the C2 stream, keys sharded key % {S} (4 shards "
                                             f"per thread, the same ones in both halves), one oracle engine per shard; "
                                             f"each shard's first half untimed, its second half ({timed} events) timed"},
            "C1": {"value": c1_done / c1_busy, "unit": "events/s", "cores": 1,
                   "sample": f"first {c1_done} events of the C1 stream (unpartitioned, 1 event per ms, "
                             f"within 10 sec), single-thread oracle"}}


def cpu_general(sa, query, make_batch, n_keys, batch, warm, playback, seconds, label):
    """SURVEY §8(d) CPU legs of one general-engine config (BASELINE configs[2] / [3]), the CPU oracle on the GPU
    box's host cores over the SAME stream the GPU leg runs: its batches in order, each pushed with the playback
    clock first advanced to the batch's last event (as the GPU leg and InputHandler.send(Event[]) do), in chunks
    (one advance per batch, so chunking changes nothing).  The GPU leg's warm-up batches run untimed first, then
    the timed events, each part bounded by time:
      (i)  single thread (the reference runs a partitioned pattern query under one lock) -> `value`;
      (ii) partition-parallel over the box's CPU share: keys sharded key % 4T, four oracle engines per pinned
           thread, each shard's events of the same batches (the same clock advances), the same untimed /
           timed split; an upper bound for any CPU engine."""
    from oracle_backend import build_oracle
    keep_heap()
    lib = build_oracle()
    app = sa.parse_app(query)
    cq = sa.compile_query(app, app.queries[0], sa.StringDictionary())
    chunk = 1 << 18
    cache = {}

    def get(b):
        if b not in cache:
            cache.clear()
            cache[b] = make_batch(b)
        return cache[b]

    def cols(d, sl):
        return [d["symbol"][sl], d["price"][sl], d["volume"][sl]]

    # (i) single thread: untimed warm-up (the GPU leg's warm-up batches, at most seconds / 3), then timed
    eng = sa.NativeEngine(lib, "sgo_", cq.ir, n_keys=n_keys)
    pos, busy, t_warm, done = 0, 0.0, 0.0, 0
    advanced = -1
    while True:
        b, off = divmod(pos, batch)
        d = get(b)
        warmup = b < warm and t_warm < seconds / 3
        if not warmup and busy >= seconds:
            break
        hi = min(batch, off + chunk)
        t = time.perf_counter()
        if playback and advanced != b:
            eng.advance_time(int(d["ts"][-1]))
            eng.discard()
            advanced = b
        sl = slice(off, hi)
        eng.push(0, pos, d["ts"][sl], cols(d, sl), None, d["key"][sl])
        eng.discard()
        el = time.perf_counter() - t
        if warmup:
            t_warm += el
        else:
            busy += el
            done += hi - off
        pos += hi - off
    eng.close()
    t0_ev = pos - done
    single = done / busy
    # (ii) partition-parallel: the same untimed prefix [0, t0_ev), then a timed range sized for ~seconds / 2
    quota = cpu_quota()
    T = max(1, int(quota) if quota else int(os.environ.get("OMP_NUM_THREADS", 0)) or (os.cpu_count() or 1))
    T = int(os.environ.get("SG_CPU_THREADS", T))
    S = 4 * T
    n_timed = max(chunk, int(single * T * 0.5 * seconds / 2))
    end = t0_ev + n_timed
    pins = distinct_cores(T)
    parts = [[[], []] for _ in range(S)]   # per shard: (untimed, timed) lists of (batch, seq base, arrays)
    for b in range(0, (end + batch - 1) // batch):
        d = get(b)
        lo, hi = b * batch, min((b + 1) * batch, end)
        last = int(d["ts"][-1])
        own = d["key"][: hi - lo] % np.uint32(S)
        for half, (a, z) in enumerate(((lo, min(hi, t0_ev)), (max(lo, t0_ev), hi))):
            if a >= z:
                continue
            for r in range(S):
                idx = np.nonzero(own[a - lo:z - lo] == r)[0] + (a - lo)
                parts[r][half].append((last, a, np.ascontiguousarray(d["ts"][idx]),
                                       [np.ascontiguousarray(c[idx]) for c in cols(d, slice(None))],
                                       (d["key"][idx] // np.uint32(S)).astype(np.uint32)))
    cache.clear()
    engs = [None] * S

    def run(e, lst):
        last_adv = None
        for last, a, ts, cs, key in lst:   # local arrival seqs (the per-key order is the global one)
            if playback and last != last_adv:
                e.advance_time(last)
                e.discard()
                last_adv = last
            if len(ts):
                e.push(0, e._sg_next, ts, cs, None, key)
                e._sg_next += len(ts)
                e.discard()

    def body(r, half):
        for sh in range(r, S, T):
            if half == 0:
                engs[sh] = sa.NativeEngine(lib, "sgo_", cq.ir, n_keys=(n_keys + S - 1) // S)
                engs[sh]._sg_next = 0
            run(engs[sh], parts[sh][half])

    el, busy_t = two_phase(T, pins, body)
    par = n_timed / el
    for e in engs:
        e.close()
    return {"value": single, "unit": "events/s", "cores": 1, "kind": "port",
            "sample": f"events [{t0_ev}, {t0_ev + done}) of the {label} stream after [0, {t0_ev}) untimed "
                      f"({warm} warm-up batch(es) of the GPU leg, capped), CPU oracle single thread, pushed in the GPU "
                      f"leg's batches (playback clock per batch)" if playback else
                      f"events [{t0_ev}, {t0_ev + done}) of the {label} stream after [0, {t0_ev}) untimed, CPU oracle "
                      f"single thread",
            "partition_parallel": {"value": par, "unit": "events/s", "threads": T, "cpu_quota": quota,
                                   "pinned_cpus": pins, "per_thread_vs_single": par / single / T,
                                   "thread_busy_s": [round(x, 3) for x in busy_t],
                                   "sample": f"events [{t0_ev}, {end}) after the same untimed prefix, keys sharded "
                                             f"key % {S}, four oracle engines per thread"}}


def to_dev(torch, d, dev):
    return {k: torch.from_numpy(v.view(np.int32) if v.dtype == np.uint32 else v).to(dev) for k, v in d.items()}


def run_general(sa, synth, torch, dev, query, make_batch, n_keys, batch, steps, warmup, cap, playback=False,
                extra_in=0, label=None):
    """One of the general-engine configs: events/s over `steps` timed batches (HBM-resident), then the
    same batches again with SG_CFG_TIMING for the roofline of the NFA kernels (k_gen_batch + the timer
    sweeps): the §8d byte model over their exact counters (extra_in: bytes per event of referenced
    attributes beyond key/price/ts) / their HIP-event time.  The timing run also counts the touched keys'
    live partials before each batch, so it is kept apart from `value`."""
    app = sa.parse_app(query)
    cq = sa.compile_query(app, app.queries[0], sa.StringDictionary())
    bats = [to_dev(torch, make_batch(s), dev) for s in range(warmup + steps)]
    lastts = [int(b["ts"][-1].item()) for b in bats]
    torch.cuda.synchronize()
    res = _run_general(sa, cq, bats, lastts, n_keys, batch, steps, warmup, cap, playback, 0, dev)
    tm = _run_general(sa, cq, bats, lastts, n_keys, batch, steps, warmup, cap, playback,
                      sa.native.SG_CFG_TIMING, dev)["delta"]
    d = res.pop("delta")
    bytes_ = algorithmic_bytes(tm) + extra_in * tm["events"]
    sec = tm["advance_ns"] / 1e9
    gbs = bytes_ / sec / 1e9 if sec > 0 else 0.0
    traffic, tsrc = pmc_traffic_general(label) if label else (None, None)
    res["roofline"] = {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                       "frac": gbs / HBM_PEAK_GBS, "traffic": traffic, "traffic_unit": "bytes/step",
                       "traffic_source": tsrc,
                       "traffic_per_alg_byte": traffic / (bytes_ / steps) if traffic else None,
                       "kernel": res.pop("kernels"),
                       "alg_bytes_per_step": bytes_ / steps, "kernel_ms_per_step": sec * 1e3 / steps,
                       "alg_bytes_per_event": bytes_ / max(1, tm["events"]),
                       "counters_per_step": {k: tm[k] / steps for k in ("keys_touched", "live_at_batch_start",
                                                                       "partials_created", "matches")}}
    assert d["matches"] == tm["matches"] and d["partials_created"] == tm["partials_created"]
    return res


def _run_general(sa, cq, bats, lastts, n_keys, batch, steps, warmup, cap, playback, flags, dev):
    eng = sa.NativeEngine(sa.load_hip_library(), "sg_", cq.ir, n_keys=n_keys, max_batch=batch,
                          partial_capacity=cap, match_capacity=2 * batch, device=dev.index or 0, flags=flags)

    def step(s):
        t = bats[s]
        if playback:  # InputHandler.send(Event[]): the clock moves to the last event first (A.9)
            eng.advance_time(lastts[s])
            m = eng.poll_device()
            eng.release(m)
        eng.push(0, s * batch, (batch, t["ts"].data_ptr(), [t["symbol"].data_ptr(), t["price"].data_ptr(),
                                                            t["volume"].data_ptr()], t["key"].data_ptr()),
                 [0, 1, 2], mem=sa.native.SG_MEM_DEVICE)
        m = eng.poll_device()
        n = int(m.n)
        eng.release(m)
        return n

    for s in range(warmup):
        step(s)
    eng.synchronize()
    st0 = eng.stats()
    t0 = time.perf_counter()
    for s in range(warmup, warmup + steps):
        step(s)
    eng.synchronize()
    el = time.perf_counter() - t0
    d = delta(st0, eng.stats())
    kernels = eng.describe()
    eng.close()
    return {"value": batch * steps / el, "unit": "events/s", "ms_per_step": el / steps * 1e3,
            "keys": n_keys, "batch_events": batch, "matches_per_step": d["matches"] / steps,
            "partials_scanned_per_step": d["partials_scanned"] / steps, "engine": "general", "delta": d,
            "kernels": kernels}


def variant_batches_np(synth, kind, K, B):
    """numpy batches of a C2 workload variant for the CPU legs (bit-identical to the device generators): batch b of
    the Zipf stream, or of the random-walk stream (the walk is stateful: stepped from batch 0 when b goes back)"""
    st = {"walk": None, "next": 0}

    def make(b):
        if kind == "zipf":
            return synth.zipf_ticks(b * B, B, K)
        if st["walk"] is None or b < st["next"]:
            st["walk"], st["next"] = synth.RandomWalk(K), 0
        while True:
            d = synth.stock_ticks(st["next"] * B, B, K)
            d["price"] = st["walk"].step(d["key"], st["next"] * B)
            st["next"] += 1
            if st["next"] > b:
                return d
    return make


def c2_variant(sa, synth, torch, dev, kind, K, B, steps, warmup, cpu_seconds, no_cpu):
    """SURVEY §8(d) workload variants of C2 (same query, same engine, same pipelined loop as the headline):
    `zipf` — partition keys Zipf(s=1.1) over the 2^20 keys (the hottest key ~12 % of every batch; keys far above the
    batch's mean run go to the hot-key pipeline, which advances all their partials at once instead of one lane
    walking them), `walk` — per-key random-walk prices (partials live longer, more of them per key: the register
    window overflows into the HBM pass more often).  HBM-resident batches generated on the device; roofline of the
    advance (staged pass + hot-key pipeline + HBM pass) over the §8d byte model; the CPU oracle on the same stream."""
    app = sa.parse_app(synth.C2_QUERY)
    cq = sa.compile_query(app, app.queries[0], sa.StringDictionary())
    walk = synth.RandomWalk(K, torch=torch, device=dev) if kind == "walk" else None
    bats = []
    for s in range(warmup + steps):
        if kind == "zipf":
            d = synth.zipf_ticks_torch(torch, s * B, B, K, dev)
        else:
            d = synth.stock_ticks_torch(torch, s * B, B, K, dev)
            d["price"] = walk.step(d["key"], s * B)
        bats.append(d)
    torch.cuda.synchronize()
    eng = sa.NativeEngine(sa.load_hip_library(), "sg_", cq.ir, n_keys=K, max_batch=B, partial_capacity=256,
                          match_capacity=2 * B, device=dev.index or 0, flags=sa.native.SG_CFG_TIMING)

    def step(s):
        t = bats[s]
        eng.push(0, s * B, (B, t["ts"].data_ptr(), [t["symbol"].data_ptr(), t["price"].data_ptr(),
                                                    t["volume"].data_ptr()], t["key"].data_ptr()),
                 [0, 1, 2], mem=sa.native.SG_MEM_DEVICE)
        take_all(eng, True)

    for s in range(warmup):
        step(s)
    eng.synchronize()
    take_all(eng, False)
    st0 = eng.stats()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(warmup, warmup + steps):
        step(s)
    eng.synchronize()
    take_all(eng, False)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    d = delta(st0, eng.stats())
    kernels = eng.describe()
    eng.close()
    del bats
    torch.cuda.empty_cache()
    launches = max(1, d["advance_launches"])
    adv_s = d["advance_ns"] / 1e9 / launches
    alg = algorithmic_bytes(d) / launches
    gbs = alg / adv_s / 1e9 if adv_s > 0 else 0.0
    traffic, traffic_src = pmc_traffic_general("C2_" + kind, "pmc_traffic_variants.json")
    out = {"value": B * steps / el, "unit": "events/s", "ms_per_step": el / steps * 1e3, "keys": K,
           "batch_events": B, "partial_capacity": 256, "engine": "two-state (C2)",
           "workload": ("C2 with Zipf(s=1.1) partition keys over 1,048,576 keys (key = bijection of the Zipf rank; the "
                        "hottest ~12 % of the events)") if kind == "zipf" else
                       ("C2 with per-key random-walk prices: p <- clamp(p + 0.25 N(0,1), 1, 100) at each of the key's "
                        "events, initial U[10, 40]"),
           "roofline": {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS,
                        "traffic": traffic, "traffic_source": traffic_src,
                        "kernel": "k_adv_m + k_hot_* + k_adv_m_h + k_adv_m_k (NFA advance)",
                        "alg_bytes_per_launch": alg, "kernel_ms_per_launch": adv_s * 1e3,
                        "hbm_pass_and_hot_ms_per_launch": d["advance_hbm_ns"] / 1e6 / launches},
           "stages_ms_per_step": {"group": d["group_ns"] / 1e6 / steps, "advance": d["advance_ns"] / 1e6 / steps,
                                  "order": d["order_ns"] / 1e6 / steps},
           "work_per_step": {k: d[k] / steps for k in ("matches", "partials_created", "partials_scanned", "keys_touched",
                                                       "live_at_batch_start", "window_spills", "hot_keys",
                                                       "hot_events")},
           "kernels": kernels}
    if not no_cpu:
        out["cpu_baseline"] = cpu_general(sa, synth.C2_QUERY, variant_batches_np(synth, kind, K, B), K, B, warmup,
                                          False, cpu_seconds, "C2_" + kind)
    return out


def take_all(eng, ready):
    """poll + release device matches until none is left (a window that wraps the ring comes in two polls);
    ready=True takes only the batches already complete"""
    while True:
        m = eng.poll_device(ready=ready)
        n = int(m.n)
        eng.release(m)
        if n == 0:
            return


def pcie_inclusive(sa, synth, torch, dev, cq, n_keys, batch, steps):
    """C2 with the batches handed over in HOST memory (sg_batch.mem = SG_MEM_HOST, pinned buffers):
    the engine's H2D copies of ts / key / the filtered column are inside the timed region.  Reported
    beside `value` (which starts from HBM-resident inputs), never as it."""
    eng = sa.NativeEngine(sa.load_hip_library(), "sg_", cq.ir, n_keys=n_keys, max_batch=batch,
                          partial_capacity=64, match_capacity=2 * batch, device=dev.index or 0,
                          flags=sa.native.SG_CFG_ASYNC_HOST)
    bats = []
    for s in range(steps + 1):
        d = synth.stock_ticks(s * batch, batch, n_keys)
        pin = {k: torch.from_numpy(v.view(np.int32) if v.dtype == np.uint32 else v).pin_memory().numpy()
               for k, v in d.items()}
        pin["key"] = pin["key"].view(np.uint32)
        pin["symbol"] = pin["symbol"].view(np.uint32)
        bats.append(pin)

    def step(s):   # pinned host batch (kept until its matches are polled: SG_CFG_ASYNC_HOST)
        d = bats[s]
        eng.push(0, s * batch, d["ts"], [d["symbol"], d["price"], d["volume"]], None, d["key"])
        take_all(eng, True)

    step(0)
    eng.synchronize()
    take_all(eng, False)
    t0 = time.perf_counter()
    for s in range(1, steps + 1):
        step(s)
    eng.synchronize()
    take_all(eng, False)
    el = time.perf_counter() - t0
    eng.close()
    hbytes = batch * (8 + 4 + 4)   # ts, key id, price (the one column the filters read)
    return {"value": batch * steps / el, "unit": "events/s", "ms_per_step": el / steps * 1e3,
            "h2d_bytes_per_step": hbytes, "h2d_GBps": hbytes * steps / el / 1e9,
            "what": "C2 from pinned host batches (SG_MEM_HOST, SG_CFG_ASYNC_HOST): H2D of ts/key/price on the "
                    "engine's grouping stream overlapping the previous batch's advance + ordering, ready polls"}


def output_inclusive(sa, synth, torch, dev, n_keys, batch, steps):
    """C2 with its select list projected on the device (sg_set_projection: e1.symbol, e1.price, e2.price,
    e2.price - e1.price) and every step's matches + projected columns copied to host memory (the
    callback-side cost the reference pays in QuerySelector + StreamCallback).  Beside `value`."""
    cp = importlib.import_module("siddhi-1_amd.compiler")
    strings = sa.StringDictionary()
    app = sa.parse_app(synth.C2_QUERY)
    cq = sa.compile_query(app, app.queries[0], strings)
    eng = sa.NativeEngine(sa.load_hip_library(), "sg_", cq.ir, n_keys=n_keys, max_batch=batch, partial_capacity=64,
                          match_capacity=2 * batch, device=dev.index or 0)
    eng.set_projection(*cp.projection_program(cq, strings))
    W = 3   # warmup steps: the pinned host staging grows to the largest window before the timed region
    bats = [synth.stock_ticks_torch(torch, s * batch, batch, n_keys, dev) for s in range(steps + W)]
    torch.cuda.synchronize()

    def step(s, ready=True):
        t = bats[s]
        eng.push(0, s * batch, (batch, t["ts"].data_ptr(), [t["symbol"].data_ptr(), t["price"].data_ptr(),
                                                            t["volume"].data_ptr()], t["key"].data_ptr()),
                 [0, 1, 2], mem=sa.native.SG_MEM_DEVICE)
        # matches + projected select list to host memory (pinned staging) of the completed batches
        return eng.poll(copy=False, ready=ready)

    def rest():   # the batches still in flight (a window that wraps the output ring comes in two parts)
        eng.synchronize()
        got = 0
        while True:
            k = len(eng.poll(copy=False))
            got += k
            if k == 0:
                return got

    for s in range(W):
        step(s)
    rest()
    t0 = time.perf_counter()
    n = 0
    for s in range(W, W + steps):
        n += len(step(s))
    n += rest()
    el = time.perf_counter() - t0
    eng.close()
    per = 8 + 4 + 8 + 16 + 8 + 4 * 9   # trigger, key, ts, 2 slot seqs, 2 chain lengths, 4 items (8 B + null)
    return {"value": batch * steps / el, "unit": "events/s", "ms_per_step": el / steps * 1e3,
            "matches_per_step": n / steps, "d2h_bytes_per_step": n / steps * per,
            "d2h_GBps": n * per / el / 1e9,
            "what": "C2 with the select list projected on the device and every step's matches + projected "
                    "columns copied to host memory (sg_poll_matches + sg_get_projection to host)"}


LINE_MAX = 8192   # the driver recovers the JSON line from a bounded stdout tail (BENCH_r05: a 23.5 KB line was lost)


def _r(x, n=4):
    """a float rounded to n significant digits (None and non-floats unchanged)"""
    if isinstance(x, float):
        return float(f"{x:.{n}g}")
    return x


def compact_line(out, detail_path):
    """The ONE stdout line: the contract's headline fields, the roofline of the advance kernel, the CPU baseline, and
    every other leg summarised to {value, ms_per_step, frac, traffic_ratio}.  The full record (per-leg counters,
    samples, kernel lists) goes to `detail_path`, which the line names.  Bounded by LINE_MAX."""
    keep = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data")
    line = {k: out[k] for k in keep}
    c = out["config"]
    line["config"] = {"workload": c["workload"], "keys_per_gpu": c["keys_per_gpu"],
                      "batch_events_per_gpu": c["batch_events_per_gpu"], "parallelism": c["parallelism"]}
    rf = out["roofline"]
    line["roofline"] = {k: rf.get(k) if k in ("achieved", "peak", "frac") else _r(rf.get(k), 6)
                        for k in ("bound", "achieved", "peak", "unit", "frac", "traffic", "kernel", "alg_bytes_per_launch",
                                  "kernel_ms_per_launch")}
    if rf.get("isolated"):
        line["roofline"]["isolated"] = {k: _r(v) for k, v in rf["isolated"].items()}
    line["stages_ms_per_step"] = {k: _r(v) for k, v in out["stages_ms_per_step"].items()}
    if out.get("stages_ms_isolated"):
        line["stages_ms_isolated"] = {k: _r(v) for k, v in out["stages_ms_isolated"].items()}
    cb = out.get("cpu_baseline")
    if cb:
        line["cpu_baseline"] = {"value": _r(cb["value"]), "unit": cb["unit"], "cores": cb["cores"], "kind": cb["kind"],
                                "sample": f"{cb['sample'].split(' (')[0]}, single-thread CPU oracle",
                                "partition_parallel": {"value": _r(cb["partition_parallel"]["value"]),
                                                       "threads": cb["partition_parallel"]["threads"]}}
    extra = {}
    for name, r in (out.get("other_configs") or {}).items():
        x = r.get("roofline") or {}
        per = x.get("alg_bytes_per_step") or x.get("alg_bytes_per_launch")
        e = {"value": _r(r["value"]), "ms_per_step": _r(r["ms_per_step"]), "frac": _r(x.get("frac"))}
        e["traffic_ratio"] = _r(x["traffic"] / per) if x.get("traffic") and per else None
        if r.get("cpu_baseline"):
            e["cpu"] = _r(r["cpu_baseline"]["value"])
        extra[name] = e
    for name in ("pcie_inclusive", "output_inclusive", "fanout_one_gpu", "api_inclusive", "api_async", "api_columnar",
                 "api_columnar_cat", "merge_inclusive"):
        r = out.get(name)
        if r:
            e = {"value": _r(r.get("value")), "ms_per_step": _r(r.get("ms_per_step"))}
            if name == "fanout_one_gpu":
                e["ratio_to_single"] = _r(r["ratio_to_single"])
                e["host_syncs_per_push"] = r["host_syncs_per_push"]
            if "error" in r:
                e["error"] = str(r["error"])[:200]
            extra[name] = e
    if extra:
        line["extra"] = extra
    line["detail"] = detail_path
    s = json.dumps(line, separators=(",", ":"))
    if len(s) > LINE_MAX:   # never lose the headline: drop the summaries first
        line.pop("extra", None)
        s = json.dumps(line, separators=(",", ":"))
    return s


def write_detail(out, rank):
    """the full record beside the line: SG_BENCH_DETAIL, else profiles/bench_detail_last.json; the path written
    (or None when it cannot be written)"""
    path = os.environ.get("SG_BENCH_DETAIL") or os.path.join("profiles", "bench_detail_last.json")
    try:
        full = path if os.path.isabs(path) else os.path.join(ROOT, path)
        os.makedirs(os.path.dirname(full), exist_ok=True)
        with open(full, "w") as f:
            json.dump(out, f, indent=1)
        return path
    except OSError:
        return None


def progress(msg):
    """a progress line on stderr (the JSON line stays the only stdout output)"""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def fanout_one_gpu(sa, synth, torch, dev, cq, n_keys, batch, steps):
    """The C-ABI's own multi-device fan-out (sg_config.n_devices, csrc/sg_sharded.cpp) rehearsed with two shards
    on this one GPU, against the single engine on the same device batches with the same host polls (the fan-out
    merges the shards' matches into host memory, so both legs poll to the host).  The shards share the GPU: the
    ratio prices the fan-out's own work (the device split, the per-push host wait for the per-owner totals, the
    host seq maps and merge), not a speed-up.  `host_syncs_per_push` = sg_stats.host_syncs / pushes."""
    W = 4   # (the stream's live population and the fan-out's host staging reach their steady size over ~4 pushes)
    bats = [synth.stock_ticks_torch(torch, s * batch, batch, n_keys, dev) for s in range(steps + W)]
    torch.cuda.synchronize()
    res = {}
    for label, devs in (("single", None), ("fanout", [dev.index or 0] * 2)):
        eng = sa.NativeEngine(sa.load_hip_library(), "sg_", cq.ir, n_keys=n_keys, max_batch=batch,
                              partial_capacity=64, match_capacity=2 * batch, device=dev.index or 0, devices=devs)

        def step(s):
            t = bats[s]
            eng.push(0, s * batch, (batch, t["ts"].data_ptr(), [t["symbol"].data_ptr(), t["price"].data_ptr(),
                                                                t["volume"].data_ptr()], t["key"].data_ptr()),
                     [0, 1, 2], mem=sa.native.SG_MEM_DEVICE)
            return len(eng.poll(copy=False))

        for s in range(W):
            step(s)
        eng.synchronize()
        st0 = eng.stats()
        t0 = time.perf_counter()
        n = sum(step(s) for s in range(W, W + steps))
        el = time.perf_counter() - t0
        st = eng.stats()
        eng.close()
        res[label] = {"value": batch * steps / el, "ms_per_step": el / steps * 1e3, "matches_per_step": n / steps,
                      "host_syncs_per_push": (st["host_syncs"] - st0["host_syncs"]) / steps,
                      "host_staged_bytes": st["host_staged_bytes"]}
    f, s1 = res["fanout"], res["single"]
    return {"value": f["value"], "unit": "events/s", "ms_per_step": f["ms_per_step"], "n_shards": 2,
            "single_engine_same_polls": s1["value"], "ratio_to_single": f["value"] / s1["value"],
            "matches_per_step": f["matches_per_step"], "host_syncs_per_push": f["host_syncs_per_push"],
            "host_staged_bytes": f["host_staged_bytes"], "keys": n_keys, "batch_events": batch,
            "what": "C2 through sg_engine_create(n_devices = 2) with both shards on this GPU, device batches, "
                    "blocking polls to host memory (the fan-out merges there); beside it the single engine with "
                    "the same polls"}


def api_inclusive(sa, synth, n_keys, chunk, chunks):
    """C2 through the product API end to end (SiddhiManager -> InputHandler.send(Event[]) -> the HIP engine
    -> QueryCallback.receive, one callback per trigger with the projected select list): the host side the
    reference's users run (InputHandler.java:51-97, QueryCallback.java:62-107).  Event objects are built
    before the timed region; the key dictionary, columnar packing, push, poll, projection and callback
    dispatch are inside it.  A bounded sample (chunk x chunks events), beside `value`."""
    mgr = sa.SiddhiManager(n_keys=n_keys, max_batch=chunk)
    rt = mgr.createSiddhiAppRuntime(synth.C2_QUERY)
    got = [0, 0]

    class Count(sa.QueryCallback):
        def receive(self, timestamp, in_events, remove_events):
            got[0] += 1
            got[1] += len(in_events)

    rt.addCallback("query1", Count())
    rt.start()
    ih = rt.getInputHandler("StockStream")
    names = [f"S{k}" for k in range(n_keys)]
    batches = []
    for c in range(chunks + 1):
        d = synth.stock_ticks(c * chunk, chunk, n_keys)
        batches.append([sa.Event(t, [names[k], p, v]) for t, k, p, v in
                        zip(d["ts"].tolist(), d["key"].tolist(), d["price"].tolist(), d["volume"].tolist())])
    ih.send(batches[0])
    t0 = time.perf_counter()
    for c in range(1, chunks + 1):
        ih.send(batches[c])
    el = time.perf_counter() - t0
    rt.shutdown()
    return {"value": chunk * chunks / el, "unit": "events/s", "events": chunk * chunks, "chunk": chunk,
            "keys": n_keys, "callbacks": got[0], "matches": got[1],
            "device_projection": bool(rt.queries[0].device_projection),
            "what": "C2 through SiddhiManager / InputHandler.send(Event[]) / QueryCallback, one send per chunk "
                    "(host Python runtime + HIP engine), bounded sample"}


def api_async(sa, synth, n_keys, n, batch_max=1 << 16):
    """C2 through the product API with the input stream declared
    @async(buffer.size, batch.size.max) and one InputHandler.send(Event) per event (the reference's usual
    producer loop; StreamJunction.java:280-317 + StreamHandler.java:58-85): the runtime buffers the sends,
    pushes batch.size.max-event batches and delivers the callbacks from ready polls, so the host packs the
    next batch while the device runs the last one.  Event objects are built before the timed region."""
    mgr = sa.SiddhiManager(n_keys=n_keys, max_batch=batch_max)
    rt = mgr.createSiddhiAppRuntime(f"@async(buffer.size='{batch_max}', batch.size.max='{batch_max}')\n" +
                                    synth.C2_QUERY)
    got = [0, 0]

    class Count(sa.QueryCallback):
        def receive(self, timestamp, in_events, remove_events):
            got[0] += 1
            got[1] += len(in_events)

    rt.addCallback("query1", Count())
    rt.start()
    ih = rt.getInputHandler("StockStream")
    names = [f"S{k}" for k in range(n_keys)]
    d = synth.stock_ticks(0, n + batch_max, n_keys)
    evs = [sa.Event(t, [names[k], p, v]) for t, k, p, v in
           zip(d["ts"].tolist(), d["key"].tolist(), d["price"].tolist(), d["volume"].tolist())]
    for e in evs[:batch_max]:   # (warm-up: engine creation, the JIT'd kernel, the key dictionary)
        ih.send(e)
    rt.flush()
    t0 = time.perf_counter()
    for e in evs[batch_max:]:
        ih.send(e)
    rt.flush()
    el = time.perf_counter() - t0
    rt.shutdown()
    return {"value": n / el, "unit": "events/s", "events": n, "batch_size_max": batch_max, "keys": n_keys,
            "callbacks": got[0], "matches": got[1], "device_projection": bool(rt.queries[0].device_projection),
            "what": "C2 through SiddhiManager with @async(batch.size.max) on the input stream, one "
                    "InputHandler.send(Event) per event, QueryCallback per trigger (host runtime + HIP engine, "
                    "ready polls), bounded sample"}


def api_columnar(sa, synth, n_keys, chunk, chunks, strings="object"):
    """C2 through the columnar host API end to end (SiddhiManager -> InputHandler.send_columns with the
    symbol column dictionary-encoded (pandas.Categorical over the 2^20 key names) -> the HIP engine ->
    ColumnarQueryCallback with the projected select list as arrays).  Columns are built before the timed
    region; key interning, push, poll, projection decode and the callbacks are inside it.  A bounded
    sample, beside `value`.  strings="categorical": the callback takes its STRING items dictionary-encoded
    too (ColumnarQueryCallback.string_columns) instead of as str objects."""
    import pandas as pd
    mgr = sa.SiddhiManager(n_keys=n_keys, max_batch=chunk)
    rt = mgr.createSiddhiAppRuntime(synth.C2_QUERY)
    got = [0, 0]

    class Count(sa.ColumnarQueryCallback):
        string_columns = strings

        def receive_columns(self, timestamps, columns, trigger_seq):
            got[0] += 1
            got[1] += len(timestamps)

    rt.addCallback("query1", Count())
    rt.start()
    ih = rt.getInputHandler("StockStream")
    cats = pd.Index([f"S{k}" for k in range(n_keys)])
    batches = []
    for c in range(chunks + 1):
        d = synth.stock_ticks(c * chunk, chunk, n_keys)
        batches.append((d["ts"], [pd.Categorical.from_codes(d["key"].astype(np.int64), categories=cats),
                                  d["price"], d["volume"]]))
    ih.send_columns(*batches[0])   # (interns the categories once: outside the timed region)
    t0 = time.perf_counter()
    for c in range(1, chunks + 1):
        ih.send_columns(*batches[c])
    el = time.perf_counter() - t0
    rt.shutdown()
    return {"value": chunk * chunks / el, "unit": "events/s", "events": chunk * chunks, "chunk": chunk,
            "keys": n_keys, "callbacks": got[0], "matches": got[1],
            "device_projection": bool(rt.queries[0].device_projection),
            "string_columns": strings,
            "what": "C2 through SiddhiManager / InputHandler.send_columns (dictionary-encoded symbols) / "
                    "ColumnarQueryCallback, one send per chunk (host runtime + HIP engine), bounded sample"}


def merge_leg(sa, lib, eng, step, first, steps, rank, world, dist, dev, B, torch, cap):
    """N > 1 (north_star: "per-partition output is merged back in timestamp order on the host"): `steps` more
    steps after the timed region, each rank's matches polled to host memory (pinned staging) and written to a
    /dev/shm segment, then rank 0 merges the ranks' runs into timestamp order (sg_merge_ts: stable, equal
    timestamps in rank order, parallel merge path over the host's CPU share).  Beside `value`, never as it.
    Every fallible part reports into a flag all ranks reduce, so the ranks stay in step and a failure ends the
    leg (recorded here) instead of hanging a collective."""
    import ctypes as C
    import numpy as np_
    port = os.environ.get("MASTER_PORT", "0")
    base = f"/dev/shm/sgmerge_{port}_"
    mine = [base + f"{rank}_{x}" for x in ("hdr", "ts", "key")]
    flag = torch.ones(1, dtype=torch.int32, device=dev)

    def agree(ok):
        flag.fill_(1 if ok else 0)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        return bool(flag.item())

    err = None
    try:
        hdr = np_.memmap(mine[0], dtype=np_.int64, mode="w+", shape=(2,))
        tsb = np_.memmap(mine[1], dtype=np_.int64, mode="w+", shape=(cap,))
        keyb = np_.memmap(mine[2], dtype=np_.uint32, mode="w+", shape=(cap,))
        ok = True
    except Exception as e:   # noqa: BLE001 (reported in the line)
        err, ok = repr(e), False
    res = None
    try:
        if not agree(ok):
            return {"error": err or "another rank could not create its segment"}
        runs = None
        if rank == 0:
            try:
                runs = [(np_.memmap(base + f"{r}_hdr", dtype=np_.int64, mode="r", shape=(2,)),
                         np_.memmap(base + f"{r}_ts", dtype=np_.int64, mode="r", shape=(cap,)),
                         np_.memmap(base + f"{r}_key", dtype=np_.uint32, mode="r", shape=(cap,))) for r in range(world)]
                ok = True
            except Exception as e:   # noqa: BLE001
                err, ok = repr(e), False
        if not agree(ok):
            return {"error": err or "rank 0 could not map the segments"}
        lib.sg_merge_ts.argtypes = [C.c_uint32, C.POINTER(C.c_void_p), C.POINTER(C.c_uint64), C.c_uint32, C.c_void_p]
        lib.sg_merge_ts.restype = C.c_int
        threads = max(1, int(cpu_quota() or 1))
        order = np_.empty(world * cap, dtype=np_.uint64) if rank == 0 else None
        got = [0]

        def sink():   # this rank's matches (a window that wraps the ring comes in two polls), global key ids
            n = 0
            while True:
                m = eng.poll(copy=False)
                k = len(m)
                if k == 0:
                    break
                if n + k > cap:
                    raise RuntimeError("merge segment full")
                tsb[n:n + k] = m.ts
                keyb[n:n + k] = m.key * np_.uint32(world) + np_.uint32(rank)
                n += k
            hdr[0] = n
            got[0] += n

        merged, merge_s = 0, 0.0
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for s in range(first, first + steps):
            try:
                step(s, sink)
                ok = True
            except Exception as e:   # noqa: BLE001
                err, ok = repr(e), False
            if not agree(ok):
                break
            if rank == 0:
                try:
                    tm = time.perf_counter()
                    lens = [int(h[0]) for h, _, _ in runs]
                    ptrs = (C.c_void_p * world)(*[t.ctypes.data if n else None for (_, t, _), n in zip(runs, lens)])
                    ln = (C.c_uint64 * world)(*lens)
                    rc = lib.sg_merge_ts(world, ptrs, ln, threads, order.ctypes.data)
                    if rc != 0:
                        raise RuntimeError(f"sg_merge_ts {rc}")
                    merged += sum(lens)
                    merge_s += time.perf_counter() - tm
                    ok = True
                except Exception as e:   # noqa: BLE001
                    err, ok = repr(e), False
            if not agree(ok):
                break
        else:
            torch.cuda.synchronize()
            dist.barrier()
            el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
            dist.all_reduce(el, op=dist.ReduceOp.MAX)
            el = float(el.item())
            res = {"value": B * world * steps / el, "unit": "events/s", "steps": steps, "ms_per_step": el / steps * 1e3,
                   "matches_per_step": merged / steps if rank == 0 else None,
                   "merge_ms_per_step": merge_s / steps * 1e3 if rank == 0 else None,
                   "merge_records_per_s": merged / merge_s if rank == 0 and merge_s > 0 else None,
                   "merge_threads": threads,
                   "what": "C5 steps with each rank's matches polled to host memory and merged by rank 0 into "
                           "timestamp order (sg_merge_ts over /dev/shm segments; equal timestamps in rank order)"}
        if res is None:
            res = {"error": err or "a rank failed"}
        return res
    finally:
        try:
            dist.barrier()   # rank 0 has unmapped nothing yet: every rank removes its own segment after it
        except Exception:    # noqa: BLE001
            pass
        for f in mine:
            try:
                os.remove(f)
            except OSError:
                pass


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 64 steps of 2^24 events: 1.07e9 events per run (>= 1e9)
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=1 << 24)
    ap.add_argument("--keys", type=int, default=None, help="keys per GPU (default: 2^20 at N=1 (C2), 2^23 at N>1 (C5))")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="skip the C3 / C4 lines")
    ap.add_argument("--legs", default=None, help="comma-separated subset of the other legs to run (experiments)")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    dist = None
    # test hooks for rehearsing the N > 1 path on one GPU: SG_BENCH_DEVICE pins every rank to one
    # device, SG_BENCH_BACKEND=gloo exchanges through host memory (the driver's runs use neither)
    local = int(os.environ.get("SG_BENCH_DEVICE", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        backend = os.environ.get("SG_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    sa = importlib.import_module("siddhi-1_amd")
    synth = importlib.import_module("siddhi-1_amd.synth")
    reshard = importlib.import_module("siddhi-1_amd.reshard")
    app = sa.parse_app(synth.C2_QUERY)
    cq = sa.compile_query(app, app.queries[0], sa.StringDictionary())
    B = args.batch
    K = args.keys or ((1 << 20) if world == 1 else (1 << 23))
    lib = sa.load_hip_library()
    rs = None
    if world > 1:   # fixed-size destination blocks: the padded batch the engine receives per step
        rs = reshard.BlockResharder(lib, B, world, ["price", "volume"], [torch.float32, torch.int32], dev)
    maxb = B if world == 1 else world * rs.cap
    flags = sa.native.SG_CFG_TIMING | (sa.native.SG_CFG_NULL_KEYS if world > 1 else 0)
    eng = sa.NativeEngine(lib, "sg_", cq.ir, n_keys=K, max_batch=maxb, partial_capacity=64,
                          match_capacity=2 * maxb, device=local, flags=flags)

    # inputs resident in HBM before timing: this rank's slice of every step of the global
    # arrival-ordered stream over world * K keys (events per ms scale with the job)
    total = args.warmup + args.steps
    batches = []
    # N > 1: one extra slice, so that every timed step also reshards the NEXT step's slice (below);
    # N = 1: ISO more steps after the timed region, run one at a time (the kernels alone on the GPU)
    ISO = 3
    # N > 1: MERGE more slices for the host timestamp-order merge leg after the timed region (merge_leg)
    MERGE = 0 if os.environ.get("SG_BENCH_NO_MERGE") else 4
    for s in range(total + (1 + MERGE if world > 1 else ISO)):
        base = s * world * B + rank * B
        # generated on the device, bit-identical to synth.stock_ticks (tests/test_synth.py)
        t = synth.stock_ticks_torch(torch, base, B, K * world, dev, rate_per_ms=2000 * world)
        if world > 1:
            del t["symbol"]
        batches.append(t)
    torch.cuda.synchronize()
    local_seq = [0]
    import ctypes as C
    lib.sg_wait_stream.argtypes = [C.c_void_p, C.c_void_p]

    def reshard_step(s):
        # HIP stable pack into destination blocks, RCCL all-to-all, unpack (no host sync)
        t = batches[s]
        return rs({"key": t["key"], "ts": t["ts"], "price": t["price"], "volume": t["volume"]})

    nxt = [reshard_step(0) if world > 1 else None]

    def step(s, sink=None):
        if world > 1:
            g = nxt[0]
            # the engine's stream waits for the exchange on the device (no host synchronisation)
            if lib.sg_wait_stream(eng.h, C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)) != 0:
                raise RuntimeError("sg_wait_stream failed")
            n = g["key"].numel()
            cols = (n, g["ts"].data_ptr(), [g["key"].data_ptr(), g["price"].data_ptr(), g["volume"].data_ptr()],
                    g["key"].data_ptr())
        else:
            t = batches[s]
            n = B
            cols = (B, t["ts"].data_ptr(), [t["symbol"].data_ptr(), t["price"].data_ptr(), t["volume"].data_ptr()],
                    t["key"].data_ptr())
        eng.push(0, local_seq[0], cols, [0, 1, 2], mem=sa.native.SG_MEM_DEVICE)
        local_seq[0] += n
        if world > 1:
            # the exchange of the next slice overlaps this step's engine work (own streams); the poll
            # waits for the step, so the exchange buffers the engine reads are never overwritten early
            nxt[0] = reshard_step(s + 1)
            del g
            if sink is None:
                take_all(eng, False)
            else:
                sink()
        else:
            # pipelined: the matches of the batches already complete; batch s's grouping runs while
            # batch s-1 advances (the engine's two streams), no host round trip between batches
            take_all(eng, True)

    def drain():   # the matches of the batches still in flight
        eng.synchronize()
        take_all(eng, False)

    for s in range(args.warmup):
        step(s)
    drain()
    st0 = eng.stats()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(args.warmup, total):
        step(s)
    drain()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t1 = time.perf_counter()
    st1 = eng.stats()
    el = t1 - t0
    if dist:
        tt = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())
    dst = delta(st0, st1)
    iso = None
    if world == 1:   # the same kernels without the two-stream overlap (each launch alone on the GPU)
        sti0 = eng.stats()
        for s in range(total, total + ISO):
            step(s)
            drain()
        iso = delta(sti0, eng.stats())
    merge = None
    if world > 1 and MERGE:
        merge = merge_leg(sa, lib, eng, step, total, MERGE, rank, world, dist, dev, B, torch, 2 * maxb)
    if rs is not None:
        rs.check()   # a destination block overflow would have dropped events: the run is invalid
    events_all = B * args.steps * world
    value = events_all / el

    launches = max(1, dst["advance_launches"])
    # the dominant kernel is the NFA advance: the LDS-staged pass k_adv_m plus the HBM pass k_adv_m_h / k_adv_m_k
    # (waves whose payload range did not fit LDS, keys whose window could overflow); the algorithmic
    # bytes cover every event of the batch, so they are priced over both passes' time
    adv_s = dst["advance_ns"] / 1e9 / launches
    adv_h_s = dst["advance_hbm_ns"] / 1e9 / launches
    alg = algorithmic_bytes(dst) / launches
    achieved = alg / adv_s / 1e9 if adv_s > 0 else 0.0
    traffic, traffic_src = pmc_traffic()
    if world != 1 or K != (1 << 20) or B != (1 << 24):   # the PMC passes were taken on the C2 shape only
        traffic, traffic_src = None, None
    out = {
        "metric": "input events/sec, partitioned pattern query, 1/2/4/8 GPU; % of HBM roofline",
        "value": value,
        "unit": "events/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": el / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (splitmix64 stock ticks, seeded, HBM-resident)",
        "config": {"workload": ("C2" if world == 1 else "C5") + ": every e1=StockStream[price>20] -> "
                               "e2=StockStream[price>e1.price] within 10 sec, partition with (symbol of StockStream), "
                               f"{K * world} keys",
                   "keys_per_gpu": K, "batch_events_per_gpu": B, "events_per_ms": 2000 * world,
                   "parallelism": f"key-sharded x{world}" + (" (RCCL all-to-all reshard per step, fixed blocks of "
                                                             f"{rs.cap} rows per destination)" if world > 1 else "")},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_unit": "bytes/launch",
                     "traffic_source": traffic_src,
                     "kernel": "k_adv_m + k_adv_m_h + k_adv_m_k (NFA advance)", "alg_bytes_per_launch": alg,
                     "kernel_ms_per_launch": adv_s * 1e3, "hbm_pass_ms_per_launch": adv_h_s * 1e3,
                     "note": "measured over the timed region, where batch i+1's grouping runs beside batch i's "
                             "advance (the kernels share the GPU); `isolated` = the same launches one batch at a "
                             "time"},
        "stages_ms_per_step": {"group": dst["group_ns"] / 1e6 / args.steps,
                               "advance": dst["advance_ns"] / 1e6 / args.steps,
                               "order": dst["order_ns"] / 1e6 / args.steps},
        "stages_ms_isolated": None if iso is None else {
            "group": iso["group_ns"] / 1e6 / ISO, "advance": iso["advance_ns"] / 1e6 / ISO,
            "order": iso["order_ns"] / 1e6 / ISO},
        "work_per_step": {k: dst[k] / args.steps for k in ("matches", "partials_created", "partials_scanned",
                                                           "keys_touched", "live_at_batch_start")},
    }
    if merge is not None:
        out["merge_inclusive"] = merge
    if iso is not None:
        a_iso = iso["advance_ns"] / 1e9 / max(1, iso["advance_launches"])
        g_iso = algorithmic_bytes(iso) / max(1, iso["advance_launches"]) / a_iso / 1e9 if a_iso > 0 else 0.0
        out["roofline"]["isolated"] = {"kernel_ms_per_launch": a_iso * 1e3, "achieved": g_iso,
                                       "frac": g_iso / HBM_PEAK_GBS}
    eng.close()
    del batches
    torch.cuda.empty_cache()
    if rank == 0:
        progress(f"C2: {out['value']:.3e} events/s ({out['ms_per_step']:.3f} ms per step)")
    if rank == 0 and world == 1 and not args.no_extra:
        steps = max(3, args.steps // 4)
        cb = 1 << 22
        # name: (query, batch maker, keys, batch events, warm-up batches, partial capacity, playback, extra bytes
        #        per event of referenced attributes, workload)
        gcfg = {
            "C3": (synth.C3_QUERY, lambda s: synth.stock_ticks(s * cb, cb, K), K, cb, 1, 8, False, 4,
                   "C3: every e1=S[price>20]<2:5>, e2=S[price>e1[last].price] or e3=S[volume>1000] within 10 sec "
                   "(SEQUENCE), 1,048,576 keys"),
            "C3_min1": (synth.C3_MIN1_QUERY, lambda s: synth.stock_ticks(s * cb, cb, K), K, cb, 1, 8, False, 4,
                        "C3 with e1<1:5> (C3 as written emits no match under the reference's SEQUENCE reset "
                        "semantics, DESIGN.md), 1,048,576 keys"),
            "C3_and": (synth.C3_AND_QUERY, lambda s: synth.stock_ticks(s * cb, cb, K), K, cb, 1, 8, False, 4,
                       "C3 with the logical AND: every e1=S[price>20]<1:5>, e2=S[price>e1[last].price] and "
                       "e3=S[volume>1000] within 10 sec (SEQUENCE), 1,048,576 keys (register-window count kernel)"),
            "P3": (synth.P3_QUERY, lambda s: synth.stock_ticks(s * cb, cb, K), K, cb, 1, 32, False, 0,
                   "3-state pattern: every e1=S[price>20] -> e2=S[price>e1.price] -> e3=S[price>e2.price] within "
                   "10 sec, 1,048,576 keys (chain kernel: register window per key, the wide window for the keys that outgrow it)"),
            "C4": (synth.C4_QUERY, lambda s: synth.burst_ticks(s * cb, cb, K, 1), K, cb, 1, 16, True, 0,
                   "C4: every e1=S[price>20] -> not S[price>e1.price] for 30 sec within 60 sec, @app:playback, "
                   "1,048,576 keys, one event per ms (distinct timer due times), 4,194,304-event batches, the "
                   "playback clock advanced per batch"),
            "C4_deep": (synth.C4_QUERY, lambda s: synth.burst_ticks(s * (cb // 16), cb // 16, K // 4, 16), K // 4, cb,
                        1, 64, True, 0,
                        "C4 with deeper per-key state: 262,144 keys, one key per ms in bursts of 16 events (up to "
                        "~16 live partials per key)"),
            # hundreds of live absent partials per key carried across pushes (C4's 30 s / 60 s
            # windows, 2,048 keys, a burst of 16 events per ms with falling prices so that partials die by their
            # timers, 2^16-event pushes = 4.1 s of event time; 8 warmup pushes fill the lists)
            "C4_deep_state": (synth.C4_QUERY, lambda s: synth.absent_deep_ticks(s * 4096, 4096, 2048, 16), 2048,
                              1 << 16, 8, 512, True, 0,
                              "C4 deep cross-batch state: 2,048 keys, bursts of 16 events per ms, 2^16-event pushes, "
                              "hundreds of live partials per key at every push"),
        }
        out["other_configs"] = {}
        legs = set(args.legs.split(",")) if args.legs else None
        for name, (q, mk, keys, bsz, warm, cap, pb, extra, wl) in gcfg.items():
            if legs is not None and name not in legs:
                continue
            r = dict(run_general(sa, synth, torch, dev, q, mk, keys, bsz, 16 if name == "C4_deep_state" else steps,
                                 warm, cap, playback=pb, extra_in=extra, label=name), workload=wl)
            if not args.no_cpu:
                r["cpu_baseline"] = cpu_general(sa, q, mk, keys, bsz, warm, pb, args.cpu_seconds / 3, name)
            out["other_configs"][name] = r
            progress(f"{name}: {r['value']:.3e} events/s")
        if "C4_deep_state" in out["other_configs"]:
            ds = out["other_configs"]["C4_deep_state"]["roofline"]["counters_per_step"]
            out["other_configs"]["C4_deep_state"]["live_per_touched_key_at_batch_start"] = \
                ds["live_at_batch_start"] / max(1.0, ds["keys_touched"])
    if rank == 0 and world == 1 and not args.no_extra:
        # SURVEY §8(d) workload variants of the headline config
        for kind in ("zipf", "walk"):
            if args.legs and "C2_" + kind not in args.legs.split(","):
                continue
            out.setdefault("other_configs", {})["C2_" + kind] = c2_variant(
                sa, synth, torch, dev, kind, K, B, max(4, args.steps // 8), 3, args.cpu_seconds / 3, args.no_cpu)
            progress(f"C2_{kind}: {out['other_configs']['C2_' + kind]['value']:.3e} events/s")
    if rank == 0 and world == 1 and not args.no_extra and not args.legs:
        out["pcie_inclusive"] = pcie_inclusive(sa, synth, torch, dev, cq, K, B, 4)
        out["output_inclusive"] = output_inclusive(sa, synth, torch, dev, K, B, 6)
        progress("pcie / output legs done")
        out["fanout_one_gpu"] = fanout_one_gpu(sa, synth, torch, dev, cq, K, 1 << 22, 6)
        progress("fan-out leg done")
        out["api_inclusive"] = api_inclusive(sa, synth, 1 << 16, 1 << 16, 16)
        out["api_async"] = api_async(sa, synth, 1 << 16, 1 << 20)
        out["api_columnar"] = api_columnar(sa, synth, 1 << 20, 1 << 20, 8)
        out["api_columnar_cat"] = api_columnar(sa, synth, 1 << 20, 1 << 20, 8, strings="categorical")
        progress("API legs done")
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(sa, synth, K, B, args.cpu_seconds)
    if rank == 0:
        print(compact_line(out, write_detail(out, rank)), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
