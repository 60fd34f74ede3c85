"""One secondary leg of bench.py alone (for rocprofv3 runs of its kernels):
c4 = the C3 stand-in's 20k mixed 1-5-term AND log, c5 = its 10k two-term
phrase log (positions on), c3 = the headline's two-term log through the same
loop.  Builds the stand-in and the leg's log first when missing (outside the
timed loop), then runs bench.run_leg with no oracle work and prints one JSON
line with the leg's roofline (algo_bytes_per_launch) and workload, the form
scripts/pmc_bytes.py reads.

usage: leg_run.py {c3,c4,c5} [PASSES]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import bench
    leg = sys.argv[1]
    passes = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    sys.argv = [sys.argv[0], "--no-cpu"]
    a = bench.parse()
    import wiser_amd as w
    idx, qlog, _ = bench.ensure_c3(a)
    tag = os.path.basename(idx.rstrip("/"))
    if leg == "c4":
        log = os.path.join(a.index_dir, f"mixed_{tag}_20000.log")
        if not os.path.exists(log):
            bench.in_child(f"w.gen_mixed_log({idx!r}, {log!r}, n_queries=20000, seed=7)\nprint('{{}}')")
        items = [(l.split(), False) for l in open(log).read().splitlines()]
        what = f"{tag}: 20000 AND queries of 1-5 terms (bench leg c4_mixed_1to5), top-10"
    elif leg == "c5":
        log = os.path.join(a.index_dir, f"phrase_{tag}_10000.log")
        if not os.path.exists(log):
            bench.in_child(f"w.gen_phrase_log({idx!r}, {log!r}, n_queries=10000, seed=7)\nprint('{{}}')")
        items = w.read_query_log(log)
        what = f"{tag}: 10000 two-term phrase queries (bench leg c5_phrase), top-10"
    else:
        items = [(l.split(), False) for l in open(qlog).read().splitlines()]
        what = f"{tag}: the headline's 100000 two-term AND queries through the leg loop, top-10"
    eng = w.VacuumEngine(idx, device=0, threads=bench.HOST_THREADS, positions=(leg == "c5"))
    eng.Load()
    out = bench.run_leg(eng, idx, items, a.k, a.batch, passes, 0, 0)
    out["config"] = {"workload": what}
    eng.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
