"""ISA audit of the round-4 lean-kernel hang (scripts/isa_audit.py).

The fixture is the gfx950 ISA of `owner_replay_tail` as built at 6b27ba1 (the
lane-0 atomicAdd claim loop that never ended on the GPU): the audit must flag
its readfirstlane behind the divergent latch, and must find no such
readfirstlane in the current kernels.hip.
"""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import isa_audit  # noqa: E402

HIPCC = "/opt/rocm/bin/hipcc"


def test_audit_flags_the_round4_claim_loop():
    bad = isa_audit.audit(os.path.join(ROOT, "tests", "golden", "isa", "owner_replay_tail_6b27ba1.s"))
    assert len(bad) == 1
    fname, block, ins = bad[0]
    assert "owner_replay_tail" in fname and ins.startswith("v_readfirstlane_b32")


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_current_kernels_have_no_divergent_latch_readfirstlane(tmp_path):
    out = tmp_path / "kernels.s"
    subprocess.check_call([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                           "-Wno-unused-function", "--cuda-device-only", "-S",
                           os.path.join(ROOT, "wiser_amd", "csrc", "kernels.hip"), "-o", str(out)],
                          stderr=subprocess.DEVNULL)
    bad = isa_audit.audit(str(out))
    assert bad == [], bad
