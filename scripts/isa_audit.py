#!/usr/bin/env python3
"""Audit the gfx950 ISA of kernels.hip for the round-4 hang pattern.

The hang: a `__noinline__` callee claimed work with
    for (;;) { qi = 0; if (lane == 0) qi = atomicAdd(claim, 1); qi = readfirstlane(qi);
               if (qi >= nq) break; ...}
Its arguments arrive in VGPRs, so the exit test was divergent to the compiler;
the loop-invariant `lane == 0` test was threaded into the back edge, and lanes
1..63 re-entered the readfirstlane block through a divergent latch
(`s_andn2_b64 exec, exec, ...` then into the header) with qi = 0 while lane 0
waited in the outer loop: readfirstlane read lane 1's 0 and the loop never ended.

The audit flags every `v_readfirstlane` that is the first exec-sensitive
instruction of a block entered by a divergent loop latch -- the only shape in
which the "first active lane" can be a lane other than the one that produced
the value.  Usage: isa_audit.py FILE.s  (exit 1 when something is flagged).
Produce FILE.s with
    hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off --save-temps -c kernels.hip
"""
import re
import sys

LABEL = re.compile(r"^(\.LBB\d+_\d+|[A-Za-z_][\w.$]*):")
FUNC_END = re.compile(r"^\s*\.size\s+(\S+),")


def blocks_of(lines):
    """(label, [instruction lines]) in order, one list per function."""
    funcs, cur, name, blk, body = [], [], None, None, []
    for ln in lines:
        m = LABEL.match(ln)
        if m:
            if blk is not None:
                cur.append((blk, body))
            blk, body = m.group(1), []
            if not blk.startswith(".LBB"):
                name = blk
            continue
        if FUNC_END.match(ln):
            if blk is not None:
                cur.append((blk, body))
            if cur:
                funcs.append((name, cur))
            cur, blk, body = [], None, []
            continue
        s = ln.split(";")[0].strip()
        if s and not s.startswith("."):
            body.append(s)
    return funcs


def audit(path):
    lines = open(path).read().splitlines()
    flagged = []
    for fname, blks in blocks_of(lines):
        order = [b for b, _ in blks]
        # blocks entered by a divergent latch: the predecessor ends with
        # `s_andn2_b64 exec, exec, X` followed by s_cbranch_execnz L (or a
        # fall-through into L after s_cbranch_execz elsewhere)
        div_targets = set()
        for i, (b, body) in enumerate(blks):
            for j, ins in enumerate(body):
                if not ins.startswith("s_andn2_b64 exec, exec"):
                    continue
                rest = body[j + 1:]
                for r in rest:
                    m = re.match(r"s_cbranch_execnz\s+(\S+)", r)
                    if m:
                        div_targets.add(m.group(1))
                        break
                    if r.startswith("s_cbranch_execz") and r is rest[-1] and i + 1 < len(order):
                        div_targets.add(order[i + 1])   # falls through into the next block
                        break
        for b, body in blks:
            if b not in div_targets:
                continue
            for ins in body:
                if ins.startswith("v_readfirstlane"):
                    flagged.append((fname, b, ins))
                    break
                if "exec" in ins or ins.startswith(("v_", "global_", "flat_", "buffer_", "ds_")):
                    break   # something exec-masked came first
    return flagged


if __name__ == "__main__":
    bad = audit(sys.argv[1])
    for f, b, ins in bad:
        print(f"{f}: {b}: {ins}")
    print(f"{len(bad)} flagged")
    sys.exit(1 if bad else 0)
