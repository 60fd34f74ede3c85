#!/usr/bin/env python3
"""Fabric bytes per dispatch from the raw TCC_EA0 request counters, by request
size, instead of rocprofv3's derived FETCH_SIZE (whose gfx950 expression counts
a 128-byte request as 64 bytes: it adds TCC_BUBBLE, the gfx942 128-byte count,
not TCC_EA0_RDREQ_128B).  read = 128 x RDREQ_128B + 32 x RDREQ_32B + 64 x the
rest; write = 64 x WRREQ_64B + 32 x the rest.  scripts/calib_ea.hip checks the
formula on known byte counts (stream) and gives bytes per line of the engine's
gather shapes.

Usage: pmc_bytes.py PMC_DIR [KERNEL[,KERNEL...] OUT_JSON [BENCH_JSON]]
Without kernels: prints every kernel's per-dispatch averages.  BENCH_JSON: the
bench line of a profiled pass; its workload and algorithmic bytes per launch
are recorded beside the counter bytes.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def load(pmc_dir):
    rows = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(f"{pmc_dir}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0].strip()
            short = name.split("<")[0].split("::")[-1]
            tmpl = name[len(name.split("<")[0]):]
            rows[short + tmpl][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return rows


def bytes_of(c):
    out = {}
    if "TCC_EA0_RDREQ_sum" in c:
        rd, r128 = c["TCC_EA0_RDREQ_sum"], c.get("TCC_EA0_RDREQ_128B_sum", 0.0)
        r32 = c.get("TCC_EA0_RDREQ_32B_sum", 0.0)
        out["read_bytes"] = 128 * r128 + 32 * r32 + 64 * (rd - r128 - r32)
    if "TCC_EA0_WRREQ_sum" in c:
        wr, w64 = c["TCC_EA0_WRREQ_sum"], c.get("TCC_EA0_WRREQ_64B_sum", 0.0)
        out["write_bytes"] = 64 * w64 + 32 * (wr - w64)
    return out


def averages(rows):
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in rows.items()}


if __name__ == "__main__":
    avg = averages(load(sys.argv[1]))
    if len(sys.argv) < 4:
        for k, c in sorted(avg.items()):
            print(k, json.dumps({**c, **bytes_of(c)}))
        sys.exit(0)
    kernels = sys.argv[2].split(",")
    tot = defaultdict(float)
    per = {}
    for k, c in avg.items():
        if k.split("<")[0] in kernels:
            per[k] = {**c, **bytes_of(c)}
            for x, v in per[k].items():
                tot[x] += v
    res = {"kernels": per, "per_launch": dict(tot),
           "hbm_bytes_per_launch": tot.get("read_bytes", 0.0) + tot.get("write_bytes", 0.0),
           "src_sha": __import__("bench").src_sha(),   # the profiled sources (bench.load_pmc checks it)
           "formula": "read = 128*RDREQ_128B + 32*RDREQ_32B + 64*(RDREQ - both); "
                      "write = 64*WRREQ_64B + 32*(WRREQ - WRREQ_64B) (TCC_EA0, all channels)"}
    if len(sys.argv) > 4:
        try:
            b = json.loads(open(sys.argv[4]).read().strip().splitlines()[-1])
            res["algo_bytes_per_launch"] = b["roofline"]["algo_bytes_per_launch"]
            res["workload"] = b["config"]["workload"]
            res["traffic_over_algo"] = res["hbm_bytes_per_launch"] / res["algo_bytes_per_launch"]
        except (OSError, ValueError, KeyError, IndexError):
            pass
    json.dump(res, open(sys.argv[3], "w"), indent=1)
    print(json.dumps(res, indent=1))
