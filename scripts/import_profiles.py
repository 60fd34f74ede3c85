#!/usr/bin/env python3
"""Copy a profiling run's summaries from gpurun_out/TAG into profiles/DEST and
stamp the counter profiles (*_pmc_segment.json) with the tree they describe:
the git HEAD at import and whether the profiled sources (their src_sha, from
scripts/pmc_bytes.py) are the tree's (bench.py attaches a profile's traffic
only when they are).  Refuses a counter profile whose sources
differ from the tree's, so that no stale traffic is committed.

usage: import_profiles.py TAG DEST"""
import glob
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    tag, dest = sys.argv[1], sys.argv[2]
    src = os.path.join(ROOT, "gpurun_out", tag)
    out = os.path.join(ROOT, "profiles", dest)
    os.makedirs(out, exist_ok=True)
    here = bench.src_sha()
    head = subprocess.run(["git", "-C", ROOT, "rev-parse", "--short", "HEAD"], capture_output=True,
                          text=True).stdout.strip()
    dirty = bool(subprocess.run(["git", "-C", ROOT, "status", "--porcelain", "--"] + list(bench.PMC_SRC),
                                capture_output=True, text=True).stdout.strip())
    for f in sorted(glob.glob(os.path.join(src, "*"))):
        name = os.path.basename(f)
        if name.endswith((".err", ".log")) and not name.startswith("pytest"):
            continue
        if name.endswith("_pmc_segment.json"):
            d = json.load(open(f))
            if d.get("src_sha") != here:
                sys.exit(f"{name}: profiled sources {d.get('src_sha')} are not the tree's {here}")
            d["git_head"] = head + ("+" if dirty else "")
            d["git_head_note"] = ("the commit the profiled sources belong to ('+': the tree had uncommitted "
                                  "changes to them at import, the src_sha is authoritative)")
            json.dump(d, open(os.path.join(out, name), "w"), indent=1)
        elif os.path.isfile(f):
            shutil.copy(f, os.path.join(out, name))
    print(out)


if __name__ == "__main__":
    main()
