#!/usr/bin/env python3
"""Throughput bench: 2-term AND + BM25 top-10 over a Vacuum index on MI355X.

Workload (BASELINE.json metric "... on Wikipedia", configs[2], SURVEY.md 8d
"C3"): no en-Wikipedia dump exists offline, so the index is the Wikipedia-shaped
stand-in written by the build's writer in the reference's Vacuum layout: 5.5 M
docs, 5.64 M terms with the df histogram of the reference's en-Wikipedia index
(tools/gen_synthetic_log.py:8-16), 0.81 G postings; 100k two-term queries drawn
by the gen_synthetic_log.py:191-214 rule (seed 7); batches of 4096 queries per
GPU; k = 10.  (--workload c2: configs[1], 1 M synthetic Zipf docs; at N = 1 it
also runs as the `c2_synthetic_1m` leg.  --vacuum-dir: a real dump.)

A step = one batch through the engine with the batch's resolved queries
already resident in HBM:
  N = 1     plan + segment + replay kernels over the whole index;
  N > 1     three forms measured in one run, each rank 4096 queries per step:
            hybrid (the value): queries whose driver list has >= --heavy-blocks
              blocks run on every doc-range shard (rank r holds doc ids
              [N*r/W, N*(r+1)/W)), their events move through fixed slots by the
              engine's own RCCL all-to-all over xGMI (wsr_shard_step) and each
              owner replays its queries; the others run whole on the rank's
              full-index image;
            docshard: the same with every query sharded (--heavy-blocks 0, the
              north_star layout an index larger than one GPU needs);
            replica (control): full index per GPU, no collective.
value = queries completed by all ranks / max-over-ranks wall time (weak scaling).

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""
import argparse
import ctypes as C
import hashlib
import json
import math
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "queries/sec + p50 lat, 2-term AND BM25 top-10 on Wikipedia, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# Per-launch fabric bytes of the segment phase (scripts/gpu_prof.sh,
# scripts/pmc_bytes.py), one profile per workload: attached to lines of that
# workload only, with the file named in roofline.traffic_source.
PMC_PROFILES = {w: f"r06p/{w}_pmc_segment.json"
                for w in ("c3", "c2", "c4_mixed_1to5", "c5_phrase", "single_high", "realistic_mix")}
# The sources a counter profile describes (the kernels, their launch and the
# image they read): scripts/pmc_bytes.py records their hash in the profile and
# load_pmc attaches its traffic only to a run of sources that hash the same.
PMC_SRC = ("wiser_amd/csrc/kernels.hip", "wiser_amd/csrc/kernels.h", "wiser_amd/csrc/engine_types.h",
           "wiser_amd/csrc/engine.cc", "wiser_amd/csrc/index.cc", "wiser_amd/csrc/index.h")


def src_sha(root=ROOT):
    """sha256 (16 hex digits) of the PMC_SRC files, names and contents."""
    h = hashlib.sha256()
    for f in PMC_SRC:
        h.update(f.encode())
        with open(os.path.join(root, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]
DIAG = {}   # host-side diagnostics of the timed loop (rank 0's)
DEFERRED = []   # oracle work (parity checks, CPU baselines) run after every timed loop


def cpu_share():
    """Host CPUs this process may use: sched_getaffinity, the cgroup quota
    (cpu.max, v2; cfs_quota_us / period, v1) and the pool's documented per-GPU
    share (OMP_NUM_THREADS is set to it on the GPU box).  -> dict"""
    nproc = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = nproc
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    eff = aff if quota is None else max(1, min(aff, math.ceil(quota)))
    hint = os.environ.get("OMP_NUM_THREADS", "")
    share = int(hint) if hint.isdigit() and int(hint) > 0 else None
    return {"nproc": nproc, "affinity": aff, "cgroup_quota_cpus": quota, "effective_cpus": eff,
            "pool_share": share}


CPUS = cpu_share()
# host threads per GPU for builds, loads and the snippet stage: the pool's share
# when it is stated, else the effective CPUs (at most 16)
HOST_THREADS = max(1, min(CPUS["pool_share"] or 16, CPUS["effective_cpus"]))


def log(msg):
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3000,
                   help="timed steps (batches); the default makes the timed region >= 0.5 s")
    p.add_argument("--warmup", type=int, default=50)
    p.add_argument("--workload", choices=["c3", "c2"], default="c3",
                   help="c3 (default): the en-Wikipedia-shaped stand-in (BASELINE configs[2]); "
                        "c2: 1M synthetic Zipf docs (configs[1])")
    p.add_argument("--docs", type=int, default=1_000_000, help="C2 docs")
    p.add_argument("--vocab", type=int, default=500_000, help="C2 vocabulary")
    p.add_argument("--queries", type=int, default=100_000)
    p.add_argument("--batch", type=int, default=4096, help="queries per GPU per step")
    p.add_argument("--k", type=int, default=10)
    p.add_argument("--mode", choices=["auto", "shard", "replica"], default="auto",
                   help="N>1: auto = hybrid doc-range shards (the value) + every-query doc-range "
                        "shards + replicas (control), all in one run; shard = the sharded forms only; "
                        "replica = full index per GPU, queries split across ranks, no collective")
    p.add_argument("--exchange", choices=["rccl", "gloo"], default="rccl",
                   help="N>1 shards: the engine's own RCCL step (the measurement), or the same "
                        "fused step with the transfer over the launcher's gloo group (a multi-rank "
                        "rehearsal on one GPU; its speed is not the exchange's)")
    p.add_argument("--dist-backend", default="gloo",
                   help="the launcher's host-side group (rendezvous, RCCL id, barriers, timing "
                        "reduction); the data path is the engine's own RCCL exchange")
    p.add_argument("--index-dir", default=os.environ.get("WISER_BENCH_DIR", "/tmp/wiser_bench"))
    p.add_argument("--vacuum-dir", default=None,
                   help="configs[2]: an existing Vacuum dump (my.vacuum, my.tip, my.doc_length), "
                        "e.g. the reference's en-Wikipedia index, instead of the stand-in")
    p.add_argument("--linedoc", default=None,
                   help="configs[2]: build the index from this linedoc first (--format)")
    p.add_argument("--format", default="WITH_POSITIONS", choices=["WITH_POSITIONS", "TOKEN_ONLY"])
    p.add_argument("--cpu-seconds", type=float, default=16.0,
                   help="bounded CPU-baseline sample (oracle), rank 0 at N=1, split over the "
                        "thread counts measured")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--no-extra", action="store_true",
                   help="skip the secondary legs (N=1 only)")
    p.add_argument("--legs", default="",
                   help="comma list of secondary legs to run (default: all of c2_synthetic_1m, "
                        "end_to_end, c4_mixed_1to5, single_high, single_low, c5_phrase, realistic_mix, "
                        "c3_topics, serving, c1_snippets)")
    p.add_argument("--c3-docs", type=int, default=5_500_000)
    p.add_argument("--c3-term-scale", type=float, default=1.0)
    p.add_argument("--check", type=int, default=256, help="queries checked against the oracle")
    p.add_argument("--max-inflight", type=int, default=0,
                   help="timed loops: before launching step s, wait until the batch of step s-K has "
                        "finished (K batches in flight at most; 0: no host throttle)")
    p.add_argument("--heavy-blocks", type=int, default=-1,
                   help="N>1 hybrid: queries whose driver list has at least this many 128-posting "
                        "blocks run on every shard (RCCL exchange); the others run whole on the "
                        "rank's full-index image (0: every query is sharded; -1, the default: "
                        "max(64, 63 * N), so that each shard's part of a sharded query is at "
                        "least one full work item)")
    p.add_argument("--item-blocks", type=int, default=0,
                   help="driver blocks per work item at most for the headline batches "
                        "(wsr_batch_set_item_blocks; 0: the engine's default)")
    p.add_argument("--shard-group", type=int, default=8,
                   help="N>1 shards: heavy batches of this many consecutive steps share one "
                        "all-to-all (wsr_shard_steps)")
    p.add_argument("--shard-every", type=int, default=0,
                   help="N>1 shards: the heavy queries of this many consecutive steps go through "
                        "one sharded step (a heavy batch every that many steps; 0, the default: "
                        "enough steps for about 4096 heavy queries per rank, at most the log's "
                        "batches)")
    return p.parse_args()


def c3_dir(a):
    return os.path.join(a.index_dir, f"c3_wiki_{a.c3_docs}_{a.c3_term_scale:g}")


def in_child(code):
    """Run `code` (Python, with `w` = wiser_amd) in a child process and return
    the JSON it prints last.  Index builds run there: the writer's many
    threads and gigabytes of short-lived host memory stay out of the process
    whose HIP calls the timed loops measure (see snapshot); so does the
    serving leg (its own HIP runtime, as a server process has)."""
    prog = f"import sys, json, time\nsys.path.insert(0, {ROOT!r})\nimport wiser_amd as w\n{code}"
    r = subprocess.run([sys.executable, "-c", prog], capture_output=True, text=True)
    if r.returncode != 0:
        raise SystemExit(f"child build failed ({r.returncode}): {r.stderr[-2000:]}")
    return json.loads(r.stdout.strip().splitlines()[-1])


def ensure_c3(a):
    """The C3 stand-in and its 100k two-term log (built once per box, ~35 s)."""
    d = c3_dir(a)
    qlog = os.path.join(d, "two_term_100000.log")
    info = None
    if not os.path.exists(os.path.join(d, "READY")):
        os.makedirs(d, exist_ok=True)
        info = in_child(
            f"t = time.time()\n"
            f"st = w.build_wiki_standin({d!r}, n_docs={a.c3_docs}, term_scale={a.c3_term_scale!r}, "
            f"threads={HOST_THREADS})\n"
            f"w.gen_two_term_log({d!r}, {qlog!r}, n_queries=100000, seed=7)\n"
            f"print(json.dumps({{'docs': st.n_docs, 'terms': st.n_terms, 'postings': st.n_postings, "
            f"'vacuum_bytes': st.vacuum_bytes, 'avg_length': round(st.avg_length, 2), "
            f"'build_s': round(time.time() - t, 1)}}))")
        open(os.path.join(d, "READY"), "w").write("ok")
        log(f"C3 stand-in built: {info}")
    return d, qlog, info


def ensure_c2(a):
    idx = os.path.join(a.index_dir, f"c2_{a.docs}_{a.vocab}")
    qlog = os.path.join(idx, f"two_term_{a.queries}.log")
    if not os.path.exists(os.path.join(idx, "READY")):
        os.makedirs(idx, exist_ok=True)
        st = in_child(
            f"t = time.time()\n"
            f"st = w.build_synthetic({idx!r}, n_docs={a.docs}, vocab={a.vocab}, threads={HOST_THREADS})\n"
            f"w.gen_two_term_log({idx!r}, {qlog!r}, n_queries={a.queries}, seed=7)\n"
            f"print(json.dumps({{'docs': st.n_docs, 'terms': st.n_terms, 'postings': st.n_postings, "
            f"'gb': st.vacuum_bytes / 1e9, 's': time.time() - t}}))")
        open(os.path.join(idx, "READY"), "w").write("ok")
        log(f"built index {st['docs']} docs {st['terms']} terms {st['postings']} postings "
            f"{st['gb']:.2f} GB in {st['s']:.1f}s")
    return idx, qlog


def workload_text(a, idx, n_lines):
    if a.vacuum_dir or a.linedoc:
        return (f"Vacuum index {idx}: {n_lines} two-term AND queries (gen_synthetic_log.py:191-214 "
                f"rule, seed 7), {a.batch} queries per GPU per step, top-{a.k}")
    if a.workload == "c2":
        return (f"C2: {a.docs} synthetic Zipf docs (V={a.vocab}, s=1.07), {n_lines} two-term AND "
                f"queries (gen_synthetic_log rule, seed 7), {a.batch} queries per GPU per step, "
                f"top-{a.k}")
    return (f"C3 stand-in (en-Wikipedia-shaped): {a.c3_docs} docs, the en-Wikipedia df histogram "
            f"x {a.c3_term_scale:g} (gen_synthetic_log.py:8-16), {n_lines} two-term AND queries "
            f"(:191-214 rule, seed 7), {a.batch} queries per GPU per step, top-{a.k}, "
            "device-resident")


def ensure_index(a, rank, dist):
    """The headline index and its two-term log: the C3 stand-in (default), C2,
    or -- configs[2] proper -- an existing Vacuum dump (--vacuum-dir, e.g. the
    reference's en-Wikipedia dump) or one built here from a linedoc (--linedoc);
    the log is generated over the index's df table by the
    gen_synthetic_log.py:191-214 rule."""
    import wiser_amd as w
    built = None
    if a.vacuum_dir or a.linedoc:
        idx = a.vacuum_dir
        if a.linedoc:
            idx = os.path.join(a.index_dir, "linedoc_" + os.path.basename(a.linedoc))
        qlog = os.path.join(a.index_dir, f"log_{os.path.basename(idx.rstrip('/'))}_{a.queries}.log")
        if rank == 0 and not os.path.exists(qlog):
            os.makedirs(a.index_dir, exist_ok=True)
            if a.linedoc and not os.path.exists(os.path.join(idx, "READY")):
                t = time.time()
                st = w.build_from_linedoc(a.linedoc, idx, a.format)
                open(os.path.join(idx, "READY"), "w").write("ok")
                log(f"built index {st.n_docs} docs {st.n_terms} terms from {a.linedoc} "
                    f"in {time.time()-t:.1f}s")
            w.gen_two_term_log(idx, qlog, n_queries=a.queries, seed=7)
    elif a.workload == "c3":
        idx, qlog = c3_dir(a), os.path.join(c3_dir(a), "two_term_100000.log")
        if rank == 0:
            idx, qlog, built = ensure_c3(a)
    else:
        idx = os.path.join(a.index_dir, f"c2_{a.docs}_{a.vocab}")
        qlog = os.path.join(idx, f"two_term_{a.queries}.log")
        if rank == 0:
            idx, qlog = ensure_c2(a)
    if dist:
        dist.barrier()
    return idx, qlog, built


def resolve(eng, chunk, k):
    import wiser_amd as w
    from wiser_amd import _capi
    arr = (_capi.Query * len(chunk))()
    for i, terms in enumerate(chunk):
        arr[i] = eng.resolve(w.SearchQuery(terms, n_results=k))[0]
    return arr


def check_against_oracle(idx, chunk, hits, nh, k, n, phrase=False):
    """Compare the first n queries' results with the oracle now."""
    return verify_snapshot(snapshot(idx, chunk, hits, nh, k, n, phrase))


def snapshot(idx, chunk, hits, nh, k, n, phrase=False):
    """The first n queries' GPU results, copied, for a check against the
    oracle later (verify_snapshot).  The oracle runs in this process and holds
    the whole dictionary in a map: loaded before a timed loop it has slowed the
    host's HIP calls of that loop by up to 8x (profiles/r03_steprate.txt), so
    every bench check runs after all timed loops, on results of the last run."""
    got = [[(hits[i * k + j].doc_id, hits[i * k + j].score) for j in range(nh[i])]
           for i in range(min(n, len(chunk)))]
    phrases = list(phrase[:n]) if isinstance(phrase, (list, tuple)) else [bool(phrase)] * len(got)
    return {"idx": idx, "chunk": [list(t) for t in chunk[:n]], "got": got, "k": k, "phrases": phrases}


def verify_snapshot(snap):
    from oracle.oracle import OracleVacuum
    orc = OracleVacuum(snap["idx"])
    for terms, got, ph in zip(snap["chunk"], snap["got"], snap["phrases"]):
        want, _ = orc.search(terms, snap["k"], phrase=ph)
        if got != want:
            raise SystemExit(f"parity failure on {terms}: {got[:3]} vs {want[:3]}")
    orc.close()
    return len(snap["got"])


def cpu_rate(idx, lines, k, seconds, threads, phrases=None):
    """(queries, seconds) of the oracle over the log (cycled), `threads`
    persistent C++ workers sharing the read-only index for a bounded time."""
    from oracle.oracle import OracleVacuum
    orc = OracleVacuum(idx)
    try:
        return orc.bench_lines(lines, k, threads, seconds, phrases=phrases)
    finally:
        orc.close()


def cpu_thread_counts():
    """1 thread, the pool's per-GPU share, the effective CPUs, the affinity set."""
    xs = [1, CPUS["pool_share"] or 0, CPUS["effective_cpus"], CPUS["affinity"]]
    return sorted(set(x for x in xs if x and x >= 1))


def cpu_baseline(idx, lines, k, seconds, what):
    """the CPU restatement of VacuumEngine::Search (oracle/oracle.cc,
    -O3 -DNDEBUG like the reference, CMakeLists.txt:6,12) on the box's host
    cores, workers sharing the read-only index as the reference's gRPC threads
    share one engine (grpc_server_impl.h:260-263).  Timed at 1 thread, the
    pool's per-GPU share, the effective CPU count and the affinity set; `value`
    is the fastest of them and `cores` its thread count."""
    counts = cpu_thread_counts()
    runs = {}
    for t in counts:
        d, c = cpu_rate(idx, lines, k, seconds / len(counts), t)
        runs[t] = (d, c)
    best = max(runs, key=lambda t: runs[t][0] / runs[t][1])
    d, c = runs[best]
    out = {"value": round(d / c, 1), "unit": "queries/s", "cores": best, "kind": "port",
           "sample": (f"{d} queries of {what} (the log cycled), oracle restatement of "
                      f"VacuumEngine::Search (-O3 -DNDEBUG), {best} persistent worker threads over "
                      f"the shared index, {c:.1f}s"),
           "by_threads": {str(t): round(runs[t][0] / runs[t][1], 1) for t in counts},
           "single_thread": round(runs[1][0] / runs[1][1], 1),
           "effective_cpus": CPUS["effective_cpus"], "affinity_cpus": CPUS["affinity"],
           "nproc": CPUS["nproc"], "cgroup_quota_cpus": CPUS["cgroup_quota_cpus"],
           "pool_share": CPUS["pool_share"],
           "build": "-O3 -DNDEBUG", "cpu_model": cpu_model(),
           "timing": "one C call per thread count: workers started and parked before the clock, "
                     "results to preallocated arrays (orc_vacuum_bench_lines)"}
    top = max(counts)
    if top > best:
        out["note"] = (f"{top} threads ({runs[top][0] / runs[top][1]:.0f} q/s) are slower than {best}: "
                       "the box's cores beyond its per-GPU share are not this job's to use "
                       f"(pool share {CPUS['pool_share']}, nproc {CPUS['nproc']})")
    return out


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def roofline_of(acc, nbk, launch_ms, source, kernel="lean_kernel||segment_kernel"):
    """Algorithmic bytes per launch (wsr_list_bytes) over the
    launch duration of `kernel` (the segment phase, fork -> join, unless
    named)."""
    algo = acc["algo"] / nbk
    ach = algo / (launch_ms * 1e-3) / 1e9
    return {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4), "algo_bytes_per_launch": int(algo),
            "avg_launch_ms": round(launch_ms, 4), "launch_ms_source": source,
            "kernel": kernel}


LEG_MIN_BATCHES = int(os.environ.get("WSR_LEG_MIN_BATCHES", "16"))


def run_leg(eng, idx, items, k, batch, passes, check, cpu_seconds, class_form=False):
    """A secondary workload on one GPU: items = [(terms, is_phrase)] in
    batches of `batch` resident queries; the timed region runs every batch
    `passes` times (consecutive batches in flight, as the main leg).
    class_form: the batches are cut by the engine's batch former
    (wsr_class_order: the log's conjunctive queries, then its phrase queries,
    each cut into batches of `batch`), not in log order."""
    import wiser_amd as w
    from wiser_amd import _capi
    batches, chunks = [], []
    groups = [items[s:s + batch] for s in range(0, len(items), batch)]
    if class_form:
        allq = (_capi.Query * len(items))()
        for i, (terms, ph) in enumerate(items):
            allq[i] = eng.resolve(w.SearchQuery(terms, n_results=k, is_phrase=ph))[0]
        groups = [[items[i] for i in g] for g in w.class_batches(allq, batch)]
    for chunk in groups:
        arr = (_capi.Query * len(chunk))()
        for i, (terms, ph) in enumerate(chunk):
            arr[i] = eng.resolve(w.SearchQuery(terms, n_results=k, is_phrase=ph))[0]
        b = w.ResidentBatch(eng, batch, k)
        b.upload(arr)
        batches.append(b)
        chunks.append(chunk)
    # A batch runs again only after its last run: a log of few batches (C5's
    # 10k queries: 3) caps the batches in flight at that count, so the leg would
    # time its batches' latency, not the device's rate.  Copies of the batches
    # (the same queries, each run in full) keep LEG_MIN_BATCHES resident, as the
    # headline's 25 do.
    n_distinct = len(batches)
    for c in range(n_distinct, max(n_distinct, LEG_MIN_BATCHES)):
        chunk = chunks[c % n_distinct]
        arr = (_capi.Query * len(chunk))()
        for i, (terms, ph) in enumerate(chunk):
            arr[i] = eng.resolve(w.SearchQuery(terms, n_results=k, is_phrase=ph))[0]
        b = w.ResidentBatch(eng, batch, k)
        b.upload(arr)
        batches.append(b)
        chunks.append(chunk)
    for b in batches:
        b.run()
    w.sync(eng)
    lat = []
    for b in batches:
        t0 = time.perf_counter()
        b.run()
        b.fetch()
        lat.append((time.perf_counter() - t0) * 1e3)
    acc = kernel_accounting(eng, batches)
    w.sync(eng)
    # enough passes for >= 0.5 s of timed wall time (isolated batch times overstate it)
    passes = max(passes, int(500.0 / max(acc["seg"] + acc["plan"], 1e-3)) + 1)
    t0 = time.perf_counter()
    for _ in range(passes):
        for b in batches:
            b.run()
    w.sync(eng)
    el = time.perf_counter() - t0
    seg = [b.stats() for b in batches]   # each batch's last run: inside the timed loop
    timed_seg = sum(st.segment_ms for st in seg) / len(seg)
    snaps = []
    for i in range(len(batches) - 1, -1, -1):   # device error flags of every batch's last run (fetch raises)
        hits, nh = batches[i].fetch()
        # batch 0's last timed run and the last distinct batch's (a class-form
        # leg's phrase batch), checked after every timed loop (snapshot)
        if check and (i == 0 or (i == n_distinct - 1 and class_form)):
            snaps.append(snapshot(idx, [t for t, _ in chunks[i]], hits, nh, k, check,
                                  phrase=[p for _, p in chunks[i]]))
    nq = sum(len(c) for c in chunks) * passes   # (every resident batch, copies included)
    for b in batches:
        b.close()
    nbk = len(batches)
    out = {"value": round(nq / el, 1), "unit": "queries/s", "queries": len(items),
           "distinct_queries": len(items), "distinct_batches": n_distinct,
           "batch": batch, "batches_resident": nbk, "passes": passes, "ms_per_batch": round(el / (passes * nbk) * 1e3, 4),
           "p50_alone_ms": round(statistics.median(lat), 3),
           "segment_ms_per_batch": round(acc["seg"] / nbk, 4),
           "survivors_per_batch": int(acc["surv"] / nbk),
           "driver_blocks_per_batch": int(acc["dblk"] / nbk),
           "roofline": roofline_of(acc, nbk, timed_seg, "timed region"),
           "parity_checked_queries": 0}
    # the device's rate over the whole loop: a batch's algorithmic bytes per
    # batch interval (with many launches in flight each one's duration is
    # stretched by the others, so the per-launch figure reads low)
    per_batch = acc["algo"] / nbk / (el / (passes * nbk)) / 1e9
    out["roofline"]["achieved_per_batch"] = round(per_batch, 1)
    out["roofline"]["frac_per_batch"] = round(per_batch / HBM_PEAK_GBS, 4)

    def deferred():   # oracle work, after every timed loop of the run (see snapshot)
        out["parity_checked_queries"] = sum(verify_snapshot(sn) for sn in snaps)
        if cpu_seconds:
            lines = [t for t, _ in items]
            phr = [p for _, p in items]
            d, c = cpu_rate(idx, lines, k, cpu_seconds, HOST_THREADS, phrases=phr)
            out["cpu_baseline"] = {"value": round(d / c, 1), "cores": HOST_THREADS, "kind": "port",
                                   "sample": f"{d} queries of the leg's log (cycled), {HOST_THREADS} "
                                             f"persistent workers, {c:.1f}s"}
    DEFERRED.append(deferred)
    return out


def c2_leg(a, local, threads):
    """BASELINE configs[1] ("C2"), one GPU: 1M synthetic Zipf docs (V=500k,
    s=1.07), its 100k two-term log, batches of 4096, top-10, device-resident."""
    import wiser_amd as w
    idx, qlog = ensure_c2(a)
    t = time.time()
    eng = w.VacuumEngine(idx, device=local, threads=threads, positions=False)
    eng.Load()
    load_s = round(time.time() - t, 1)
    image = eng.image_info()
    items = [(l.split(), False) for l in open(qlog).read().splitlines()]
    leg = run_leg(eng, idx, items, a.k, a.batch, 4, a.check, 0 if a.no_cpu else a.cpu_seconds / 4)
    eng.close()
    leg.update({"load_s": load_s, "image": image,
                "workload": (f"C2: {a.docs} synthetic Zipf docs (V={a.vocab}, s=1.07), 100000 two-term "
                             "AND queries (gen_synthetic_log rule, seed 7), top-10, batches of 4096, "
                             "device-resident")})
    pmc = load_pmc("c2")
    if pmc:
        leg["roofline"].update(pmc)
    return leg


def end_to_end_leg(a, idx, qlog, local, threads):
    """The whole Search chain per batch of 4096, from query strings to results
    in host memory: term lookup (the reference's FindIteratorsSolid,
    vacuum_engine.h:209-219), upload, plan/segment/replay, result download
    (wsr_search_text).  `clients` host threads each submit whole batches back to
    back, so batches overlap on the device; latency = submit -> results on the
    host, per batch (every query of a batch completes with it), measured while
    all clients run."""
    import threading
    import wiser_amd as w
    from wiser_amd import _capi
    eng = w.VacuumEngine(idx, device=local, threads=threads, positions=False)
    eng.Load()
    lines = open(qlog).read().splitlines()
    texts = [("\n".join(lines[s:s + a.batch])).encode() for s in range(0, len(lines), a.batch)]
    out = {}
    for clients in (4, 8):
        lat, done, errs = [], [0], []
        lock = threading.Lock()
        stop_at = [0.0]

        def client(c):
            hits = (_capi.Hit * (a.batch * a.k))()
            nh = (C.c_int32 * a.batch)()
            nq = C.c_int32()
            i = c
            try:
                while time.perf_counter() < stop_at[0]:
                    t = texts[i % len(texts)]
                    t0 = time.perf_counter()
                    _capi.check(_capi.lib.wsr_search_text(eng._h, t, len(t), a.k, a.k, a.batch,
                                                           hits, nh, C.byref(nq)))
                    dt = (time.perf_counter() - t0) * 1e3
                    with lock:
                        lat.append(dt)
                        done[0] += nq.value
                    i += clients
            except Exception as e:   # noqa: BLE001 - reported below
                errs.append(e)

        # warm the per-handle batch pool
        stop_at[0] = time.perf_counter() + 0.3
        ts = [threading.Thread(target=client, args=(c,)) for c in range(clients)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        lat.clear()
        done[0] = 0
        t0 = time.perf_counter()
        stop_at[0] = t0 + 1.5
        ts = [threading.Thread(target=client, args=(c,)) for c in range(clients)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        el = time.perf_counter() - t0
        if errs:
            raise SystemExit(f"end-to-end leg failed: {errs[0]}")
        lat.sort()
        out[f"clients_{clients}"] = {
            "value": round(done[0] / el, 1), "unit": "queries/s", "batches": len(lat),
            "p50_ms": round(lat[len(lat) // 2], 3), "p99_ms": round(lat[min(len(lat) - 1, int(0.99 * len(lat)))], 3),
            "seconds": round(el, 2)}
    eng.close()
    best = max(out.values(), key=lambda x: x["value"])
    out.update({"value": best["value"], "unit": "queries/s", "p50_ms": best["p50_ms"], "p99_ms": best["p99_ms"],
                "workload": ("the headline log as text, batches of 4096: wsr_search_text = term lookup + upload + "
                             "run + results to host memory; client threads submit batches back to back, "
                             "latency submit -> host results per batch under that load")})
    return out


# Legs over the headline index: its log (in a.index_dir), what it is, whether
# the engine needs positions.  The single-term legs are the reference's
# run_exp.py:116-117 workloads (type_single.docfreq_high / _low,
# gen_synthetic_log.py:171-189); realistic_mix is its mixed log
# (query_pool.h:363-375, run_exp.py:119 "type_realistic"): 10 % phrases among
# the 1-5-term AND mix in the same batches.
LEG_LOGS = {
    "c4_mixed_1to5": ("mixed_{tag}_20000.log", "w.gen_mixed_log({idx!r}, {log!r}, n_queries=20000, seed=7)",
                      False, "{tag}: 20000 AND queries of 1-5 terms (AOL term-count shares, gen_synthetic_log "
                             "group rule, seed 7), top-10"),
    "c5_phrase": ("phrase_{tag}_10000.log", "w.gen_phrase_log({idx!r}, {log!r}, n_queries=10000, seed=7)",
                  True, "{tag}: 10000 two-term phrase queries from the corpus's phrase pool "
                        "(gen_synthetic_log.py:216-265), top-10"),
    "single_high": ("single_high_{tag}_20000.log",
                    "w.gen_single_term_log({idx!r}, {log!r}, True, n_queries=20000, seed=7)",
                    False, "{tag}: 20000 single-term queries of the df >= 10^4 group (run_exp.py:116 "
                           "type_single.docfreq_high, gen_synthetic_log.py:171-189), top-10"),
    "single_low": ("single_low_{tag}_20000.log",
                   "w.gen_single_term_log({idx!r}, {log!r}, False, n_queries=20000, seed=7)",
                   False, "{tag}: 20000 single-term queries of the df < 10^4 group (run_exp.py:117 "
                          "type_single.docfreq_low), top-10"),
    "realistic_mix": ("realistic_{tag}_20000.log",
                      "w.gen_realistic_log({idx!r}, {log!r}, n_queries=20000, phrase_share=0.1, seed=7)",
                      True, "{tag}: 20000 queries, 10 % two-term phrases among the 1-5-term AND mix in the "
                            "same batches (query_pool.h:363-375 format), top-10"),
}


def leg_items(a, idx, name):
    """-> (items [(terms, is_phrase)], workload text, positions) of a LEG_LOGS leg
    (its log written first when missing, in a child process)."""
    import wiser_amd as w
    fname, gen, positions, what = LEG_LOGS[name]
    tag = os.path.basename(idx.rstrip("/"))
    log = os.path.join(a.index_dir, fname.format(tag=tag))
    if not os.path.exists(log):
        in_child(gen.format(idx=idx, log=log) + "\nprint('{}')")
    return w.read_query_log(log), what.format(tag=tag), positions


def extra_legs(a, idx, qlog, local, threads):
    """The other legs of one N = 1 run: C2 (configs[1]) as a leg of its own,
    then over the headline index: the whole Search chain from strings
    (end_to_end), mixed 1-5 term AND (configs[3]'s query mix), two-term
    phrases (configs[4]; on the headline index when it has a phrase pool, else
    on C2), single-query serving, and C1 with snippets (configs[0])."""
    import wiser_amd as w
    legs = {}
    chosen = set(x for x in a.legs.split(",") if x)

    def want(name):
        return not chosen or name in chosen

    c2_idx = None
    # serving in a process of its own, as a server runs: its closed loop of host
    # threads is the leg most sensitive to what the timed loops before it left in
    # this process (the same points ran 20-40 % faster in a fresh process,
    # profiles/r04m_bench.json and r04f1/ against r04n/serve_points.jsonl)
    if want("serving"):
        legs["serving"] = in_child(
            "import bench\nfrom types import SimpleNamespace\n"
            f"out = bench.serving_leg(SimpleNamespace(batch={a.batch}, k={a.k}), {idx!r}, {qlog!r}, "
            f"{local}, {threads})\nprint(json.dumps(out))")
    if want("c2_synthetic_1m") and not (a.workload == "c2" and not (a.vacuum_dir or a.linedoc)):
        legs["c2_synthetic_1m"] = c2_leg(a, local, threads)
    if want("end_to_end"):
        legs["end_to_end"] = end_to_end_leg(a, idx, qlog, local, threads)
    synthetic = a.workload == "c3" and not (a.vacuum_dir or a.linedoc)
    has_pool = os.path.exists(os.path.join(idx, "phrases.txt"))
    engines = {}

    def engine(positions):   # one engine per positions setting, shared by the legs
        if positions not in engines:
            e = w.VacuumEngine(idx, device=local, threads=threads, positions=positions)
            t = time.time()
            e.Load()
            engines[positions] = (e, round(time.time() - t, 1))
        return engines[positions]

    for name in ("c4_mixed_1to5", "single_high", "single_low", "c5_phrase", "realistic_mix"):
        if not want(name) or (LEG_LOGS[name][2] and not has_pool and name == "realistic_mix"):
            continue
        lidx = idx
        if name == "c5_phrase" and not has_pool:   # (the pool of a synthetic corpus)
            lidx = c2_idx = ensure_c2(a)[0]
        items, what, positions = leg_items(a, lidx, name)
        if lidx == idx:
            eng, load_s = engine(positions)
        else:
            eng = w.VacuumEngine(lidx, device=local, threads=threads, positions=positions)
            t = time.time()
            eng.Load()
            load_s = round(time.time() - t, 1)
        mixed = name == "realistic_mix"
        leg = run_leg(eng, lidx, items, a.k, a.batch, 4, a.check, 0 if a.no_cpu else a.cpu_seconds / 4,
                      class_form=mixed)
        leg["workload"] = what
        if leg["batches_resident"] > leg["distinct_batches"]:
            leg["workload"] += (f"; {leg['distinct_batches']} distinct batches, each run in full, resident as "
                                f"{leg['batches_resident']} (copies)")
        if mixed:
            # the value: batches cut by the engine's batch former (wsr_class_order:
            # class-pure batches); the log's own order (phrases inside every
            # batch) beside it
            leg["workload"] += ("; batches cut by the engine's batch former (wsr_class_order: the log's "
                                "conjunctive queries, then its phrases, each class in batches of 4096)")
            inter = run_leg(eng, lidx, items, a.k, a.batch, 4, 0, 0)
            leg["interleaved"] = {"value": inter["value"], "ms_per_batch": inter["ms_per_batch"],
                                  "note": "the same log cut in log order: ~10 % phrases in every batch"}
        if positions:
            leg["load_s"] = load_s
            leg["image"] = eng.image_info()
        pmc = load_pmc(name) if (lidx == idx and synthetic) else None
        if pmc:
            leg["roofline"].update(pmc)
        if lidx != idx:
            eng.close()
        legs[name] = leg
    if "realistic_mix" in legs and "c4_mixed_1to5" in legs and "c5_phrase" in legs:
        # the share-weighted pure legs: the time per query of 90 % AND mix and 10 % phrases
        items, _, _ = leg_items(a, idx, "realistic_mix")
        f = sum(1 for _, ph in items if ph) / len(items)
        exp = 1.0 / ((1 - f) / legs["c4_mixed_1to5"]["value"] + f / legs["c5_phrase"]["value"])
        legs["realistic_mix"]["weighted_pure_legs"] = round(exp, 1)
        legs["realistic_mix"]["vs_weighted_pure_legs"] = round(legs["realistic_mix"]["value"] / exp, 3)
    for e, _ in engines.values():
        e.close()
    if want("c3_topics") and a.workload == "c3" and not (a.vacuum_dir or a.linedoc):
        legs["c3_topics"] = topics_leg(a, local, threads)
    if want("c1_snippets"):
        legs["c1_snippets"] = snippet_leg(a, local, threads)
    del c2_idx
    return legs


TOPICS = dict(topics=128, topics_per_term=2, affinity=0.6)


def ensure_c3_topics(a):
    """The topic-clustered C3 stand-in (the same df histogram; doc ids in 128
    contiguous topic ranges, every term under N/16 postings draws 60 % of its
    docs from two home topics) and its 100k two-term log."""
    d = os.path.join(a.index_dir, f"c3_topics_{a.c3_docs}_{a.c3_term_scale:g}")
    qlog = os.path.join(d, "two_term_100000.log")
    if not os.path.exists(os.path.join(d, "READY")):
        os.makedirs(d, exist_ok=True)
        info = in_child(
            f"t = time.time()\n"
            f"st = w.build_wiki_standin({d!r}, n_docs={a.c3_docs}, term_scale={a.c3_term_scale!r}, "
            f"threads={HOST_THREADS}, **{TOPICS!r})\n"
            f"w.gen_two_term_log({d!r}, {qlog!r}, n_queries=100000, seed=7)\n"
            f"print(json.dumps({{'docs': st.n_docs, 'terms': st.n_terms, 'postings': st.n_postings, "
            f"'build_s': round(time.time() - t, 1)}}))")
        open(os.path.join(d, "READY"), "w").write("ok")
        log(f"C3 topic-clustered stand-in built: {info}")
    return d, qlog


def topics_leg(a, local, threads):
    """the headline workload on the topic-clustered stand-in
    (ensure_c3_topics), whose terms co-occur by topic as a real corpus's do,
    and its high x high class alone (both terms df >= 10k, the first 4096)."""
    import wiser_amd as w
    idx, qlog = ensure_c3_topics(a)
    t = time.time()
    eng = w.VacuumEngine(idx, device=local, threads=threads, positions=False)
    eng.Load()
    load_s = round(time.time() - t, 1)
    lines = [l.split() for l in open(qlog).read().splitlines()]
    out = run_leg(eng, idx, [(q, False) for q in lines], a.k, a.batch, 4, a.check,
                  0 if a.no_cpu else a.cpu_seconds / 8)
    hh = [q for q in lines if all(eng.lookup(x)[1] >= 10000 for x in q)][:a.batch]
    out["high_high"] = run_leg(eng, idx, [(q, False) for q in hh], a.k, a.batch, 4, a.check, 0)
    out.update({"load_s": load_s, "image": eng.image_info(),
                "workload": (f"C3 stand-in with topic-clustered doc ids ({TOPICS}), the same df "
                             "histogram, its 100000 two-term AND log (gen_synthetic_log rule, seed 7), "
                             "top-10, batches of 4096, device-resident; high_high: its first 4096 queries "
                             "whose two terms both have df >= 10k")})
    eng.close()
    return out


def snippet_leg(a, local, threads):
    """configs[0] ("C1"): the reference's own 10k-doc TOKEN_ONLY linedoc
    (src/testdata/test_doc_tokenized), single-term BM25 top-10 over every
    distinct token plus 10k tokens sampled with seed 1, here with
    SearchQuery::return_snippets (3 passages): GPU top-k, then the host snippet
    stage over the box's CPU share (wsr_snippets_batch).  Checked against the
    oracle's VacuumEngine::Search + GenerateSnippet, which is also the CPU
    baseline (1 thread)."""
    import random
    import wiser_amd as w
    from oracle.oracle import OracleVacuum
    src = os.path.join(ROOT, "tests", "golden", "data", "test_doc_tokenized")
    d = os.path.join(a.index_dir, "c1_test_doc_tokenized")
    if not os.path.exists(os.path.join(d, "READY")):
        os.makedirs(d, exist_ok=True)
        w.build_from_linedoc(src, d, "TOKEN_ONLY")
        open(os.path.join(d, "READY"), "w").write("ok")
    toks = set()
    with open(src) as f:
        next(f)
        for line in f:
            toks.update(line.rstrip("\n").split("\t")[2].split())
    distinct = sorted(toks)
    rng = random.Random(1)
    terms = distinct + [rng.choice(distinct) for _ in range(10000)]
    eng = w.VacuumEngine(d, device=local, threads=threads, positions=False)
    eng.Load()
    eng.snippet_threads = HOST_THREADS
    from wiser_amd import _capi
    # native path timed: the batch's GPU top-k (wsr_search_batch), then the
    # snippet stage of its entries on HOST_THREADS threads (wsr_snippets_batch)
    batches = []
    for i in range(0, len(terms), a.batch):
        chunk = terms[i:i + a.batch]
        arr = (_capi.Query * len(chunk))(*[eng.resolve(w.SearchQuery([t], n_results=a.k))[0]
                                           for t in chunk])
        batches.append((arr, len(chunk)))
    cap = 64 << 20
    sbuf = C.create_string_buffer(cap)
    ends = (C.c_uint64 * (a.batch * a.k))()
    total = C.c_uint64()
    def run(snip):
        t_topk = t_snip = 0.0
        n = 0
        for arr, nq in batches:
            hits = (_capi.Hit * (nq * a.k))()
            nh = (C.c_int32 * nq)()
            t0 = time.perf_counter()
            _capi.check(_capi.lib.wsr_search_batch(eng._h, arr, nq, a.k, hits, nh))
            t1 = time.perf_counter()
            if snip:
                _capi.check(_capi.lib.wsr_snippets_batch(eng._h, arr, nq, hits, nh, a.k, 3, HOST_THREADS,
                                                         sbuf, cap, ends, C.byref(total)))
                n += sum(nh)
            t_topk += t1 - t0
            t_snip += time.perf_counter() - t1
        return t_topk, t_snip, n
    run(True)   # warm (and fills the skip-row cache)
    t_topk, t_snip, n_snip = run(True)
    el = t_topk + t_snip
    # Python mirror, for parity: SearchBatch with return_snippets
    res = eng.SearchBatch([w.SearchQuery([t], n_results=a.k, return_snippets=True)
                           for t in terms[: a.check]])
    got = [[(e.doc_id, e.doc_score, e.snippet) for e in r.entries] for r in res]
    out = {"value": round(len(terms) / el, 1), "unit": "queries/s", "queries": len(terms),
           "snippets": n_snip, "snippets_per_s": round(n_snip / t_snip, 1), "snippet_threads": HOST_THREADS,
           "topk_ms_per_batch": round(1e3 * t_topk / len(batches), 3),
           "snippet_ms_per_batch": round(1e3 * t_snip / len(batches), 3),
           "parity_checked_queries": 0,
           "workload": ("C1: the reference's 10k-doc TOKEN_ONLY linedoc, single-term top-10 over every "
                        f"distinct token ({len(distinct)}) + 10000 sampled (seed 1), return_snippets, "
                        "3 passages; per batch of 4096: GPU top-k (wsr_search_batch, host arrays in and "
                        "out) then the snippet stage (wsr_snippets_batch)")}
    # the top-k alone (no snippets): the GPU path against config 1's own CPU
    # engine, QqMemEngineDelta over varint postings (oracle restatement)
    t_topk_only, _, _ = run(False)
    out["topk_only"] = {"value": round(len(terms) / t_topk_only, 1), "unit": "queries/s",
                        "note": "wsr_search_batch per 4096 (host arrays in and out), no snippets"}
    eng.close()

    def deferred():   # oracle work, after every timed loop of the run (see snapshot)
        orc = OracleVacuum(d)
        bad = 0
        for t, g in zip(terms[: a.check], got):
            bad += g != orc.search_snippets([t], a.k)
        if bad:
            raise SystemExit(f"c1 snippet leg: {bad} queries differ from the oracle")
        out["parity_checked_queries"] = len(got)
        if not a.no_cpu:
            t0, n, i = time.time(), 0, 0
            while time.time() - t0 < 2.0:
                orc.search_snippets([terms[i % len(terms)]], a.k)
                n += 1
                i += 1
            out["cpu_baseline"] = {"value": round(n / (time.time() - t0), 1), "cores": 1, "kind": "port",
                                   "sample": f"{n} queries of the leg's list, oracle Search + GenerateSnippet, 2s"}
            from oracle.oracle import OracleQqMem
            qq = OracleQqMem(src, "TOKEN_ONLY")
            t0, n, i = time.time(), 0, 0
            while time.time() - t0 < 2.0:
                qq.search([terms[i % len(terms)]], a.k)
                n += 1
                i += 1
            out["topk_only"]["cpu_baseline"] = {
                "value": round(n / (time.time() - t0), 1), "cores": 1, "kind": "port",
                "sample": f"{n} single-term top-{a.k} queries of the leg's list through the oracle's "
                          "QqMemEngineDelta (varint PostingListDelta, skip span 100), 2s"}
            qq.close()
        orc.close()
    DEFERRED.append(deferred)
    return out


def serving_leg(a, idx, qlog, local, threads):
    """Single-query serving through the micro-batcher (wsr_server_*): client
    threads keep 512-768 (or 64) queries each in flight (the reference client's
    threads, grpc_client_impl.h:557-620) over the headline log; latency = submit ->
    result.  The clients share the box's 16-core CPU share with the dispatcher,
    so few client threads with deep windows load it best."""
    import wiser_amd as w
    from wiser_amd import _capi
    eng = w.VacuumEngine(idx, device=local, threads=threads, positions=False)
    eng.Load()
    lines = [l.split() for l in open(qlog).read().splitlines()]
    arr = (_capi.Query * len(lines))()
    for i, t in enumerate(lines):
        arr[i] = eng.resolve(w.SearchQuery(t, n_results=a.k))[0]
    out = {}
    # (7 x 704, 6 x 768, 5 x 960 and 8 x 640 in flight: around the best points
    # of the sweeps on the box's 16-core share, profiles/r04n/serve_points.jsonl:
    # 6.1 / 5.2 / 5.1 M q/s at p50 0.85 / 0.88 / 0.94 ms; more client threads
    # oversubscribe the share beside the dispatcher, the completer and HIP's)
    # (a first, unrecorded second of load: the first server of a process ran
    # its first point 20 % below the same point later, profiles/r04s2/)
    srv = w.Server(eng, max_batch=a.batch, window_us=1000)
    srv.bench(arr, n_clients=7, depth=704, seconds=1.0)
    srv.close()
    for clients, depth, window in ((7, 704, 1000), (6, 768, 1000), (5, 960, 1000), (8, 640, 1000), (4, 64, 100)):
        srv = w.Server(eng, max_batch=a.batch, window_us=window)
        st = srv.bench(arr, n_clients=clients, depth=depth, seconds=3.0)
        srv.close()
        out[f"in_flight_{clients * depth}"] = {
            "value": round(st.qps, 1), "unit": "queries/s", "p50_ms": round(st.p50_ms, 3),
            "p99_ms": round(st.p99_ms, 3), "mean_batch": round(st.mean_batch, 1),
            "window_us": window, "clients": clients, "depth": depth,
            "queue_ms": round(st.queue_ms, 3), "gpu_ms": round(st.gpu_ms, 3),
            "handoff_ms": round(st.handoff_ms, 3)}
    eng.close()
    return out


def timed_launch_stats(batches, steps):
    """Segment-phase launch durations of the timed region itself: the HIP
    events (recorded on each batch's own stream, fork -> join) of every batch's
    last run inside the timed loop, with consecutive batches overlapping as they
    ran there (the durations a rocprofv3 kernel trace of the same command
    averages).  With fewer steps than batches only the batches the timed loop
    ran count (the others last ran one at a time, before it)."""
    ran = batches[:min(steps, len(batches))]
    if not ran:
        return
    seg = [b.stats() for b in ran]
    DIAG["timed_seg_ms"] = sum(st.segment_ms for st in seg) / len(seg)
    DIAG["timed_lean_ms"] = sum(st.lean_ms for st in seg) / len(seg)


def kernel_accounting(eng, batches):
    """HIP-event kernel times + algorithmic bytes over one pass of the batches."""
    import wiser_amd as w
    acc = dict(seg=0.0, lean=0.0, plan=0.0, rep=0.0, algo=0, surv=0, dblk=0, oblk=0, items=0)
    for b in batches:
        b.run()
        w.sync(eng)
        st = b.stats()
        acc["seg"] += st.segment_ms
        acc["lean"] += st.lean_ms
        acc["plan"] += st.plan_ms
        acc["rep"] += st.replay_ms
        acc["algo"] += st.algo_bytes
        acc["surv"] += st.survivors
        acc["dblk"] += st.driver_blocks
        acc["oblk"] += st.other_blocks
        acc["items"] += st.work_items
    return acc


def staggered(dist, rank, world, fn, group=2):
    """fn() on every rank, `group` ranks at a time: a full-image load holds the
    host image (26.7 GB for the C3 stand-in) until its upload, so eight ranks
    loading at once would need eight host images at the same time."""
    if dist is None or world <= group:
        return fn()
    out = None
    for g in range(0, world, group):
        if g <= rank < g + group:
            out = fn()
        dist.barrier()
    return out


def open_full(idx, local, threads, rank, world, dist):
    import wiser_amd as w

    def load():
        e = w.VacuumEngine(idx, device=local, threads=threads, positions=False)
        e.Load()
        return e
    return staggered(dist, rank, world, load)


def open_shard_engine(a, idx, rank, world, local, dist, threads):
    """This rank's doc-range shard image with the engine's RCCL communicator
    (the full-index image the hybrid and replica forms also need is opened
    separately, open_full, after the pure doc-range form has run alone)."""
    from wiser_amd.shard import NativeShardedSearcher
    t = time.time()

    def share_id(x):   # rank 0's RCCL id to every rank, over the launcher's gloo group
        if dist is None:   # (one rank: --mode shard at N = 1, a rehearsal of this path)
            return x
        box = [x]
        dist.broadcast_object_list(box, src=0)
        return box[0]

    if a.exchange == "gloo" and dist is not None:
        from wiser_amd.shard import HostExchangeShardedSearcher
        S = HostExchangeShardedSearcher(idx, rank, world, device=local, threads=threads, positions=False)
    else:
        S = NativeShardedSearcher(idx, rank, world, share_id, device=local, threads=threads, positions=False)
    log(f"rank {rank}: shard {S.doc_range} loaded in {time.time()-t:.1f}s")
    return S


def run_shard(a, S, full, heavy_blocks, lines, rank, world, dist):
    """Doc-range shards.  Every rank holds the doc-id range
    [N*r/W, N*(r+1)/W) (S) and takes its own 4096 queries per step.  Heavy
    queries (driver list of >= heavy_blocks blocks, where the work is) run on
    every rank over its range: wsr_shard_step packs each owner's events into a
    fixed slot, one RCCL all-to-all moves counts and slots between all pairs,
    and the owner replays its queries; the rest run whole on the rank's
    full-index image (full) with no collective (heavy_blocks 0: every query is
    sharded, full unused).  Returns a dict of the run and its batches."""
    import torch
    import wiser_amd as w
    from wiser_amd.shard import slot_for_fill

    def barrier():
        if dist is not None:
            dist.barrier()

    B = a.batch
    per_rank = len(lines) // world
    nb = max(1, per_rank // B)
    df = {}

    def is_heavy(q):
        if heavy_blocks <= 0:
            return True
        ds = []
        for x in q:
            if x not in df:
                df[x] = S.engine.lookup(x)[1]   # global df, as every image keeps
            ds.append(df[x])
        return bool(ds) and min(ds) > 0 and min(math.ceil(d / 128) for d in ds) >= heavy_blocks

    # Heavy queries of `every` consecutive steps go through one sharded step (at
    # the first step of the group): a sharded step has a large fixed host cost
    # (its own plan and segment launches, the RCCL call, the owner replay), so
    # with few heavy queries per step (0.7 % of the log at N = 8) a step per
    # batch makes the loop host-bound (profiles/r02_sm_shard_every.txt: 0.22 ms
    # of host time per 0.15 ms step); grouped, heavy batches keep ~4096 queries
    # per rank (a whole batch; one-rank hybrid rehearsal, C3: 16.3 M q/s at
    # ~1024 per heavy batch, 18.0 M at ~4096, profiles/r04v/) and the light
    # batches run every step.
    def heavy_of(j, g):
        chunk = lines[g * per_rank + j * B: g * per_rank + (j + 1) * B]
        return [q for q in chunk if is_heavy(q)]
    every = a.shard_every
    if every <= 0:
        per_step = max(1, sum(len(heavy_of(j, rank)) for j in range(nb)) // nb)
        every = max(1, min(nb, -(-4096 // per_step)))
        if dist is not None:   # one cadence for every rank (the collective pairs up)
            ev = torch.tensor([float(every)])
            dist.all_reduce(ev, op=dist.ReduceOp.MAX)
            every = int(ev.item())
    every = max(1, min(every, nb))
    # every rank builds the same global heavy batches from the same log split
    # One shape for every heavy batch (q_per_owner = the largest heavy batch,
    # the rest padded with empty queries): --shard-group batches go through one
    # all-to-all only when their shapes agree (every rank computes the same
    # split of the same log, so the shape is common).
    heavy_parts = {j: [sum((heavy_of(jj, g) for jj in range(j, min(nb, j + every))), []) for g in range(world)]
                   for j in range(0, nb, every)}
    hq_all = max((len(p) for parts in heavy_parts.values() for p in parts), default=0)
    steps = []   # per batch index: (heavy ResidentBatch or None, q_per_owner, heavy chunk,
                 #                   cheap ResidentBatch or None, cheap chunk)
    for j in range(nb):
        hb, hq, hchunk = None, 0, []
        if j % every == 0:
            parts = heavy_parts[j]
            hq = hq_all if any(parts) else 0
            if hq:
                for p in parts:
                    hchunk += p + [[]] * (hq - len(p))   # (an empty query: an empty result)
                hb = w.ResidentBatch(S.engine, hq * world, a.k)
                hb.upload(resolve(S.engine, hchunk, a.k))
        mine = lines[rank * per_rank + j * B: rank * per_rank + (j + 1) * B]
        cheap = [q for q in mine if not is_heavy(q)]
        cb = None
        if cheap:
            cb = w.ResidentBatch(full, len(cheap), a.k)
            cb.upload(resolve(full, cheap, a.k))
        steps.append((hb, hq, hchunk, cb, cheap))
    # exchange slot: every heavy batch once with a generous slot, then twice the
    # largest fill any rank saw (wsr_shard_fill), agreed over the group
    fill = 0
    for hb, hq, _, _, _ in steps:
        if hb:
            S.step(hb, hq, 64 * hq)
            fill = max(fill, S.max_fill(hb))
    if dist is not None:
        mx = torch.tensor([float(fill)])
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        fill = int(mx.item())
    max_hq = max(1, max(st[1] for st in steps))
    slot = slot_for_fill(fill, max_hq)

    # heavy batches of up to --shard-group consecutive steps (of one shape)
    # go through one all-to-all: its host cost is paid once per group
    pend = []

    def flush():
        if pend:
            S.steps([x for x, _ in pend], pend[0][1], slot)
            pend.clear()

    def step(i, fetch=False):
        hb, hq, _, cb, _ = steps[i % nb]
        if cb:
            cb.run()
        if hb:
            if pend and (pend[0][1] != hq or any(x is hb for x, _ in pend)):
                flush()   # (a group holds one shape, and each batch once)
            pend.append((hb, hq))
            if fetch or len(pend) >= max(1, a.shard_group):
                flush()
        if fetch:
            return (S.fetch_owned(hb, hq) if hb else None), (cb.fetch() if cb else None)
        return None

    def sync_all():
        S.flush()   # (a host-exchange rehearsal's last exchange)
        w.sync(S.engine)
        if full:
            w.sync(full)

    lat = []   # one step at a time (p50_alone), every batch once before the clock
    for i in range(nb):
        barrier()
        t0 = time.perf_counter()
        step(i, fetch=True)
        lat.append((time.perf_counter() - t0) * 1e3)
    # the W warmup steps right before the clock
    for s_ in range(a.warmup):
        step(s_)
    flush()
    barrier()
    sync_all()
    cs0 = S.comm_stats() if hasattr(S, "comm_stats") else None
    t0 = time.perf_counter()
    for s_ in range(a.steps):
        step(s_)
    flush()
    host_ms = (time.perf_counter() - t0) / max(1, a.steps) * 1e3
    sync_all()
    el = time.perf_counter() - t0
    comm = None
    if cs0 is not None:   # what the timed loop's step groups really were
        cs1 = S.comm_stats()
        comm = {k: cs1[k] - cs0[k] for k in cs1}
        comm["mean_group"] = round(comm["steps"] / max(1, comm["groups"]), 3)
    snaps = []
    for i, (hb, hq, hchunk, cb, cheap) in enumerate(steps):   # error flags (a slot overflow among
        hres = S.fetch_owned(hb, hq) if hb else None         # them) of every last step
        cres = cb.fetch() if cb else None
        if i == 0 and a.check and rank == 0:   # step 0's last timed run, checked after the timed loops
            if hres:
                snaps.append(snapshot(S.engine.engine_dir_path, hchunk[:hq], hres[0], hres[1], a.k, a.check))
            if cres:
                snaps.append(snapshot(S.engine.engine_dir_path, cheap, cres[0], cres[1], a.k, a.check))
    # every rank completes its own 4096 queries per step (heavy owned + cheap)
    queries = sum(len(steps[s_ % nb][4]) + sum(1 for q in steps[s_ % nb][2][rank * steps[s_ % nb][1]:
                                                                          (rank + 1) * steps[s_ % nb][1]] if q)
                  for s_ in range(a.steps))
    share = sum(st[1] for st in steps) / max(1, nb * B)

    def close():
        for hb, _, _, cb, _ in steps:
            for x in (hb, cb):
                if x:
                    x.close()
    return {"queries": queries, "el": el, "p50": statistics.median(lat), "snaps": snaps,
            "slot": slot, "heavy_share": share, "heavy_blocks": heavy_blocks, "every": every,
            "host_ms": host_ms, "comm": comm,
            "batches": [st[3] for st in steps if st[3]] or [st[0] for st in steps if st[0]],
            "engine": full if (full and any(st[3] for st in steps)) else S.engine, "close": close}


def run_replica(a, eng, idx, lines, rank, world, dist):
    """Full index per GPU (eng); the log is split across ranks, 4096 queries
    per rank per step, consecutive batches in flight on per-batch streams."""
    import wiser_amd as w
    per_rank = (len(lines) + world - 1) // world
    mine = lines[rank * per_rank:(rank + 1) * per_rank] or lines[:a.batch]
    batches, chunks = [], []
    for s in range(0, len(mine), a.batch):
        chunk = mine[s:s + a.batch]
        b = w.ResidentBatch(eng, a.batch, a.k)
        if a.item_blocks:
            from wiser_amd._capi import check as _check, lib as _lib
            _check(_lib.wsr_batch_set_item_blocks(eng._h, b._b, a.item_blocks))
        b.upload(resolve(eng, chunk, a.k))
        batches.append(b)
        chunks.append(chunk)
    nb = len(batches)
    lat = []   # one batch at a time (p50_alone), every batch once before the clock
    for b in batches:
        t0 = time.perf_counter()
        b.run()
        b.fetch()
        lat.append((time.perf_counter() - t0) * 1e3)
    # the W warmup steps right before the clock (the device busy, as in the loop)
    for s in range(a.warmup):
        batches[s % nb].run()
    if dist:
        dist.barrier()
    w.sync(eng)
    K = a.max_inflight if a.max_inflight < nb else 0
    t0 = time.perf_counter()
    for s in range(a.steps):
        if K and s >= K:
            batches[(s - K) % nb].wait_ready()
        batches[s % nb].run()
    host_ms = (time.perf_counter() - t0) / max(1, a.steps) * 1e3
    w.sync(eng)
    el = time.perf_counter() - t0
    timed_launch_stats(batches, a.steps)
    # every batch's last run: the device error flags (capacity, limits) must be
    # clear, or the pass does not count (fetch raises on any flag)
    for b in batches[::-1]:
        hits, nh = b.fetch()
    snaps = []
    if a.check and rank == 0:   # batch 0's last timed run, checked after every timed loop
        snaps.append(snapshot(idx, chunks[0], hits, nh, a.k, a.check))
    queries = sum(batches[s % nb].nq for s in range(a.steps))

    def close():
        for b in batches:
            b.close()
    return {"queries": queries, "el": el, "p50": statistics.median(lat), "snaps": snaps,
            "host_ms": host_ms, "batches": batches, "engine": eng, "close": close}


def group_note(a, comm):
    """How the timed loop's sharded steps were exchanged, from the
    communicator's own counters (a group holds each batch once, so it can be
    smaller than --shard-group)."""
    if not comm:
        return f"one host exchange per sharded step (gloo rehearsal, --shard-group {a.shard_group} unused)"
    return (f"one ncclAllToAll per {comm['mean_group']} sharded steps on average ({comm['groups']} groups, "
            f"{comm['steps']} steps; --shard-group {a.shard_group} at most), owner replays: "
            f"{comm['replays_in_lean']} in later lean kernels, {comm['replays_on_stream']} on the exchange stream")


def reduce_timing(dist, el, queries, p50, on_gpu, summed):
    """Max wall time and p50 over ranks; queries summed (replicas) or as is."""
    import torch
    tt = torch.tensor([el, float(queries), p50], dtype=torch.float64)
    if on_gpu:
        tt = tt.cuda()
    mx = tt.clone()
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    sm = tt.clone()
    dist.all_reduce(sm, op=dist.ReduceOp.SUM)
    return mx[0].item(), (sm[1].item() if summed else queries), mx[2].item()


def load_pmc(workload):
    """Per-launch fabric bytes of the segment phase (lean_kernel +
    segment_kernel) from TCC_EA0 request counts by size (scripts/pmc_bytes.py;
    the formula is checked against known streaming kernels in the same
    profile run's calib_bytes file, where FETCH_SIZE reads half the bytes on
    gfx950), measured on this workload's replica leg."""
    name = PMC_PROFILES.get(workload)
    path = os.path.join(ROOT, "profiles", name) if name else None
    if not path or not os.path.exists(path):
        return None
    try:
        pm = json.load(open(path))
        here = src_sha()
        if pm.get("src_sha") != here:   # profiled on other kernel sources: not this build's bytes
            return {"traffic": None, "traffic_stale": name,
                    "traffic_note": f"profile of sources {pm.get('src_sha')}, running {here}"}
        out = {"traffic": pm["hbm_bytes_per_launch"], "traffic_source": name, "traffic_src_sha": here,
               "traffic_fetch_size_raw": pm["per_launch"].get("FETCH_SIZE", 0.0) * 1024}
        if "algo_bytes_per_launch" in pm:   # the profiled run's own algorithmic bytes
            out["traffic_over_algo"] = round(pm["hbm_bytes_per_launch"] / pm["algo_bytes_per_launch"], 3)
        return out
    except Exception:
        return None


def launcher_cmd(gpus, argv, port, script=None):
    """The child launcher `--gpus N > 1` runs when no launcher started this
    process: one rank per GPU on this node, rendezvous on 127.0.0.1."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr", "127.0.0.1", "--master-port", str(port),
            script or os.path.abspath(__file__), *argv]


def check_world(gpus, env):
    """-> 'spawn' | 'run', or raise SystemExit when the launcher's world size
    disagrees with --gpus: a multi-GPU measurement must never silently be a
    different N."""
    if gpus < 1:
        raise SystemExit(f"--gpus {gpus}: must be >= 1")
    ws = env.get("WORLD_SIZE")
    if ws is None:
        return "spawn" if gpus > 1 else "run"
    if int(ws) != gpus:
        raise SystemExit(f"WORLD_SIZE={ws} but --gpus {gpus}: refusing to measure a different "
                         f"number of ranks than asked for")
    return "run"


def spawn_ranks(gpus, argv, script=None):
    """Start `torch.distributed.run` as a child (never an exec: nothing in this
    process has touched the GPU yet, and it never will), pass its stdout and
    stderr through, and return its exit code."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = launcher_cmd(gpus, argv, port, script)
    log(f"--gpus {gpus} without a launcher: starting {gpus} ranks ({' '.join(cmd[1:6])} ...)")
    return subprocess.run(cmd, env=env, cwd=ROOT).returncode


def main():
    a = parse()
    # before any HIP call (runtime_info below is one): N > 1 without a launcher
    # spawns one, and a launcher whose world size is not N is refused
    if check_world(a.gpus, os.environ) == "spawn":
        sys.exit(spawn_ranks(a.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # (N = 1: replica, or --mode shard to rehearse the sharded path with one rank)
    mode = a.mode if world > 1 else ("shard" if a.mode == "shard" else "replica")
    # One HIP runtime per process, the same as the GPU test suite's: torch loads
    # first (it maps its libamdhip64 / librccl), then libwiser_hip.so binds to
    # those sonames; torch itself is only the launcher's rendezvous (N > 1)
    try:
        import torch
    except ImportError:
        torch = None
    import wiser_amd as w
    from wiser_amd import _capi
    runtime = _capi.runtime_info()
    if world > 1:
        import torch.distributed as dist
        # one GPU per rank; rehearsals with more ranks than GPUs share devices
        # (device_count does not initialise the GPU, torch never touches it)
        local = local % max(1, torch.cuda.device_count())
        # host-side group (gloo): rendezvous, the RCCL id, barriers and the
        # max-over-ranks timing; the data path is the engine's own RCCL exchange
        dist.init_process_group(a.dist_backend)

    idx, qlog, built = ensure_index(a, rank, dist)
    lines = [l.split() for l in open(qlog).read().splitlines()]
    threads = HOST_THREADS
    wkey = "dump" if (a.vacuum_dir or a.linedoc) else a.workload

    forms = {}      # N > 1: every form measured, reduced over ranks
    full = S = None
    t = time.time()
    def reduced(r):
        el, q, p50 = r["el"], r["queries"], r["p50"]
        if dist:
            el, q, p50 = reduce_timing(dist, el, q, p50, False, summed=True)
        return {"value": round(q / el, 1), "ms_per_step": round(el / a.steps * 1e3, 4),
                "p50_alone_ms": round(p50, 3), "queries": int(q), "seconds": round(el, 5)}

    shard_bytes = full_bytes = None
    if mode == "replica":
        full = open_full(idx, local, threads, rank, world, dist)
        log(f"rank {rank}: engine loaded in {time.time()-t:.1f}s")
    else:
        hb_default = max(64, 63 * world)
        S = open_shard_engine(a, idx, rank, world, local, dist, threads)
        shard_bytes = S.engine.image_info()["total_bytes"]
        if world > 1 and a.mode == "auto" and a.heavy_blocks != 0:
            # the pure doc-range form first, with only this rank's shard image
            # resident: the form an index larger than one GPU runs, and its own
            # HBM per rank
            r = run_shard(a, S, None, 0, lines, rank, world, dist)
            forms["docshard"] = {**reduced(r), "parallelism": f"docshard{world}", "slot_events": r["slot"],
                                 "shard_every": r["every"], "hbm_per_rank": shard_bytes, "comm": r["comm"],
                                 "note": "every query on every shard, only the rank's shard image resident; "
                                         + group_note(a, r["comm"])}
            r["close"]()
        if a.heavy_blocks != 0 or a.mode == "auto":
            full = open_full(idx, local, threads, rank, world, dist)
    load_s = round(time.time() - t, 1)
    if full is not None:
        full_bytes = full.image_info()["total_bytes"]

    if mode == "replica":
        main_run = run_replica(a, full, idx, lines, rank, world, dist)
        parallelism = f"replicas{world}"
    else:
        # the value: hybrid (--heavy-blocks default) or the form asked for
        hb = a.heavy_blocks if a.heavy_blocks >= 0 else hb_default
        main_run = run_shard(a, S, full, hb, lines, rank, world, dist)
        share = main_run["heavy_share"]
        parallelism = (f"docshard{world}" if hb == 0 else
                       f"hybrid-docshard{world} ({100 * share:.2f}% of queries sharded)")
    acc = kernel_accounting(main_run["engine"], main_run["batches"])
    image = main_run["engine"].image_info()
    nbk = len(main_run["batches"])
    iso_ms = acc["seg"] / nbk
    seg_avg_ms = DIAG.get("timed_seg_ms", iso_ms)
    seg_src = "timed region" if "timed_seg_ms" in DIAG else "one batch at a time"
    lean_avg_ms = DIAG.get("timed_lean_ms", acc["lean"] / nbk)
    mres = reduced(main_run)
    snaps = main_run["snaps"]
    host_ms = main_run["host_ms"]
    main_run["close"]()
    if world > 1 and a.mode == "auto":
        # the control, from the same full image: replicas (no collective)
        r = run_replica(a, full, idx, lines, rank, world, dist)
        forms["replica"] = {**reduced(r), "parallelism": f"replicas{world}", "hbm_per_rank": full_bytes,
                            "note": "control: the full index on every GPU, each rank its own 4096 "
                                    "queries, no collective"}
        r["close"]()
    if S is not None:
        S.close()
    if full is not None:
        full.close()

    extra = None
    if rank == 0 and world == 1 and not a.no_extra:
        extra = extra_legs(a, idx, qlog, local, threads)
    # oracle work only now, after every timed loop (see snapshot): parity of the
    # headline's and every leg's last timed run, then the CPU baselines
    checked = sum(verify_snapshot(sn) for sn in snaps)
    for fn in DEFERRED:
        fn()
    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu:
        cpu = cpu_baseline(idx, lines, a.k, a.cpu_seconds, "the headline workload's log")

    if rank == 0:
        # the dominant kernel, lean_kernel (its HIP events on the batch stream,
        # plan end -> lean end; the general segment_kernel runs beside it on a
        # second stream and is given with the fork -> join time below)
        roof = roofline_of(acc, nbk, lean_avg_ms, seg_src + ", lean_kernel (HIP events on its stream)",
                           "lean_kernel")
        roof.update({"traffic": None, "traffic_source": None})
        if mode == "replica":
            pmc = load_pmc(wkey)
            if pmc:
                roof.update(pmc)
        roof.update({
            # the same bytes over the pipelined step time (consecutive batches
            # overlap on the device; value's own clock)
            "achieved_per_step": round((acc["algo"] / nbk) / (mres["seconds"] / a.steps) / 1e9, 1),
            # the segment phase: lean_kernel with the general segment_kernel
            # beside it on a second stream (HIP events fork -> join on the
            # batch's stream; isolated: one batch at a time, nothing overlapping)
            "lean_kernel_ms": round(lean_avg_ms, 4),
            "fork_join_ms": round(seg_avg_ms, 4),
            "frac_fork_join": round((acc["algo"] / nbk) / (seg_avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "isolated_launch_ms": round(iso_ms, 4),
            "isolated_frac": round((acc["algo"] / nbk) / (iso_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "algo_bytes_rule": "SURVEY 8d: per query the docid+tf span bytes of every term's list "
                               "(wsr_list_bytes) + 1 B per survivor + 12 B per result"})
        out = {
            "metric": METRIC, "value": mres["value"], "unit": "queries/s", "n_gpus": world,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": mres["ms_per_step"],
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32/f64",
            "data": "synthetic",
            "config": {"workload": workload_text(a, idx, len(lines)), "global_batch": a.batch * world,
                       "parallelism": parallelism, "k": a.k},
            # p50 at the operating point: the end-to-end leg (strings in, results in host
            # memory, batches overlapped); p50_alone_ms: one resident batch by itself
            "p50_ms": (extra["end_to_end"]["p50_ms"] if extra and "end_to_end" in extra
                       else mres["p50_alone_ms"]),
            "p50_alone_ms": mres["p50_alone_ms"],
            "roofline": roof,
            "cpu_baseline": cpu,
            "kernel_ms_per_batch": {"plan": round(acc["plan"] / nbk, 4),
                                    "segment": round(iso_ms, 4),
                                    "replay": round(acc["rep"] / nbk, 4)},
            "per_batch": {"survivors": int(acc["surv"] / nbk), "driver_blocks": int(acc["dblk"] / nbk),
                          "other_blocks": int(acc["oblk"] / nbk), "work_items": int(acc["items"] / nbk)},
            "parity_checked_queries": checked,
        }
        out["runtime"] = runtime
        out["image"] = image   # HBM bytes of the engine image the value ran on
        out["load_s"] = load_s
        if built:
            out["index_build"] = built
        # host time to enqueue the timed steps: close to ms_per_step = launch-bound
        out["host_enqueue_ms_per_step"] = round(host_ms, 4)
        if mode != "replica":
            kind = ("ncclAllToAll of per-owner regions ({count, offset} pairs + fixed event slot) over "
                    "xGMI per step group (wsr_shard_steps), no host round trip inside a step: "
                    + group_note(a, main_run["comm"]))
            if a.exchange == "gloo" and world > 1:
                kind = ("REHEARSAL: fused emit / owner replay with the slots moved by gloo through "
                        "host memory (not the RCCL path's speed)")
            out["exchange"] = {"kind": kind, "slot_events": main_run["slot"],
                               "heavy_blocks": main_run["heavy_blocks"],
                               "shard_every": main_run["every"], "shard_group": a.shard_group,
                               "comm": main_run["comm"],
                               "heavy_query_share": round(main_run["heavy_share"], 4)}
            out["hbm_per_rank"] = {"shard_image_bytes": shard_bytes, "full_image_bytes": full_bytes,
                                   "total_bytes": (shard_bytes or 0) + (full_bytes or 0),
                                   "note": "the value's form; forms.*.hbm_per_rank: each form's own"}
        if forms:
            out["forms"] = forms
        if extra:
            out["legs"] = extra
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
