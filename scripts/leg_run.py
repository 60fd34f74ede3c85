"""One bench.py leg alone (for rocprofv3 runs of its kernels): c3 = the
headline's two-term log through the leg loop, c2 = configs[1]'s 1 M-doc Zipf
index and its 100k two-term log, or any bench.LEG_LOGS leg over the C3
stand-in (c4_mixed_1to5, single_high, single_low, c5_phrase, realistic_mix;
c4 / c5 are accepted for the first two).  Builds the index and the leg's log
first when missing (outside the timed loop), then runs bench.run_leg with no
oracle work and prints one JSON line with the leg's roofline
(algo_bytes_per_launch), workload and the sources' hash, the form
scripts/pmc_bytes.py reads.

usage: leg_run.py LEG [PASSES]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
ALIASES = {"c4": "c4_mixed_1to5", "c5": "c5_phrase"}


def main():
    import bench
    leg = ALIASES.get(sys.argv[1], sys.argv[1])
    passes = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    sys.argv = [sys.argv[0], "--no-cpu"]
    a = bench.parse()
    import wiser_amd as w
    positions = False
    if leg == "c2":
        idx, qlog = bench.ensure_c2(a)
        items = [(l.split(), False) for l in open(qlog).read().splitlines()]
        what = "C2: the 1M-doc Zipf index's 100000 two-term AND queries through the leg loop, top-10"
    else:
        idx, qlog, _ = bench.ensure_c3(a)
        if leg == "c3":
            items = [(l.split(), False) for l in open(qlog).read().splitlines()]
            what = (f"{os.path.basename(idx.rstrip('/'))}: the headline's 100000 two-term AND queries "
                    "through the leg loop, top-10")
        else:
            items, what, positions = bench.leg_items(a, idx, leg)
    eng = w.VacuumEngine(idx, device=0, threads=bench.HOST_THREADS, positions=positions)
    eng.Load()
    # (realistic_mix: batches cut by the engine's batch former, as in bench.py)
    out = bench.run_leg(eng, idx, items, a.k, a.batch, passes, 0, 0, class_form=leg == "realistic_mix")
    out["config"] = {"workload": what}
    out["src_sha"] = bench.src_sha()
    eng.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
