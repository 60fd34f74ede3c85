"""A corpus whose lists exercise the offset buckets (engine_types.h): 70k
docs; "g" every 56th doc (64-doc buckets of ~1.1 postings) plus crowded
stretches -- 20 consecutive docs from 6400 (a walk past the offset window), 9
from 19200 and 7 from 12800 (inside the window), 5 from 25600 (just past the
entry's four); "s" every 45th doc; "z" in docs 0-9, 500-519 and the last (one
bucket of ten in a list of 31: crowded, so a bitmap); "y" every other doc (a
bitmap); "u0".."u999" every 1000th doc (drivers)."""
N_DOCS = 70000


def build_bucket_index(root):
    import wiser_amd as w
    ld = root / "b.linedoc"
    n = N_DOCS
    crowd = set(range(6400, 6420)) | set(range(19200, 19209)) | set(range(12800, 12807)) | set(range(25600, 25605))
    with open(ld, "w") as f:
        f.write("FIELDS_HEADER_INDICATOR###\tdoctitle\tbody\ttokenized\n")
        for i in range(n):
            toks = [f"u{i % 1000}"]
            if i % 56 == 3 or i in crowd:
                toks += ["g"] * (1 + i % 3)
            if i < 10 or 500 <= i < 520 or i == n - 1:
                toks.append("z")
            if i % 45 == 7:
                toks.append("s")
            if i % 2:
                toks.append("y")
            f.write(f"t\t{' '.join(toks)}\t{' '.join(toks)}\n")
    d = root / "idx"
    d.mkdir()
    w.build_from_linedoc(str(ld), str(d), "TOKEN_ONLY")
    return str(d)
