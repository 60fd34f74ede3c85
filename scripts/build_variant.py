#!/usr/bin/env python3
"""Build a variant of libwiser_hip.so for an on-GPU A/B without touching the
tree's sources: copy wiser_amd/csrc to a scratch directory, apply literal
substitutions, compile with the Makefile's flags into
wiser_amd/_lib/variants/NAME.so (git-ignored, travels to the GPU box).
Select it at run time with WISER_HIP_LIB=wiser_amd/_lib/variants/NAME.so.

usage: build_variant.py NAME FILE OLD NEW [FILE OLD NEW ...]
(each OLD must occur exactly once in FILE, a path under wiser_amd/csrc/)
"""
import os
import shutil
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRCS = ["writer.cc", "index.cc", "engine.cc", "server.cc", "docstore.cc", "snippet.cc", "kernels.hip"]
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-Wall",
         "-Wno-unused-function"]


def main():
    name, subs = sys.argv[1], sys.argv[2:]
    if not subs or len(subs) % 3:
        sys.exit(__doc__)
    tmp = tempfile.mkdtemp(prefix=f"wsr_var_{name}_")
    src = os.path.join(tmp, "wiser_amd", "csrc")   # (sources include ../../include/)
    shutil.copytree(os.path.join(R, "wiser_amd", "csrc"), src)
    os.symlink(os.path.join(R, "include"), os.path.join(tmp, "include"))
    for i in range(0, len(subs), 3):
        f, old, new = subs[i:i + 3]
        p = os.path.join(src, f)
        s = open(p).read()
        if s.count(old) != 1:
            sys.exit(f"{f}: {old!r} occurs {s.count(old)} times")
        open(p, "w").write(s.replace(old, new))
    hipcc = "/opt/rocm/bin/hipcc"

    def obj(f):
        o = os.path.join(tmp, f + ".o")
        subprocess.run([hipcc, *FLAGS, "-c", os.path.join(src, f), "-o", o], check=True)
        return o

    with ThreadPoolExecutor(4) as ex:
        objs = list(ex.map(obj, SRCS))
    out_dir = os.path.join(R, "wiser_amd", "_lib", "variants")
    os.makedirs(out_dir, exist_ok=True)
    out = os.path.join(out_dir, name + ".so")
    subprocess.run([hipcc, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out, *objs, "-lpthread",
                    "-l:liblz4.so.1", "-lrccl"], check=True)
    shutil.rmtree(tmp)
    print(out)


if __name__ == "__main__":
    main()
