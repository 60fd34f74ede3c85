#!/usr/bin/env python3
"""Index a large linedoc with the streaming writer in a child process and
record wall time, peak RSS (the child's ru_maxrss) and the index shape.

usage: writer_scale.py LINEDOC OUT_DIR FORMAT [bloom] [threads] [chunk_docs] > result.json"""
import json
import os
import resource
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ld, out, fmt = sys.argv[1], sys.argv[2], sys.argv[3]
    bloom = len(sys.argv) > 4 and sys.argv[4] == "bloom"
    threads = sys.argv[5] if len(sys.argv) > 5 else ""
    chunk = sys.argv[6] if len(sys.argv) > 6 else ""
    env = dict(os.environ)
    if threads:
        env["WSR_WRITER_THREADS"] = threads
    if chunk:
        env["WSR_WRITER_CHUNK_DOCS"] = chunk
    code = ("import json, sys; sys.path.insert(0, %r); import wiser_amd as w; "
            "st = w.build_from_linedoc(%r, %r, %r, bloom=%s); "
            "print(json.dumps({'n_docs': st.n_docs, 'n_terms': st.n_terms, 'n_postings': st.n_postings, "
            "'vacuum_bytes': st.vacuum_bytes, 'avg_length': st.avg_length}))"
            % (ROOT, ld, out, fmt, "(0.0009, 5)" if bloom else "None"))
    t = time.time()
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True)
    el = time.time() - t
    if r.returncode:
        sys.stderr.write(r.stderr)
        raise SystemExit(r.returncode)
    st = json.loads(r.stdout.strip().splitlines()[-1])
    rss_kb = resource.getrusage(resource.RUSAGE_CHILDREN).ru_maxrss
    files = {f: os.path.getsize(os.path.join(out, f)) for f in sorted(os.listdir(out))}
    print(json.dumps({"linedoc": os.path.basename(ld), "linedoc_bytes": os.path.getsize(ld), "format": fmt,
                      "bloom": "ratio 0.0009, 5 entries" if bloom else None,
                      "threads": threads or "default (min(cpus, 16))", "chunk_docs": chunk or "default (8192)",
                      "wall_s": round(el, 1), "peak_rss_mib": round(rss_kb / 1024, 1),
                      "host_cpus": os.cpu_count(), "index": st, "files": files}, indent=1))


if __name__ == "__main__":
    main()
