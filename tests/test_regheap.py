"""RegHeap (wiser_amd/csrc/regheap.h: the register-resident restatement of the
reference's MinPointerHeap for k <= 16, used by the replay) compiled for the
host with g++ and checked against libstdc++'s own std::priority_queue with the
reference comparator, RankDoc and SortHeap, on tie-heavy random streams."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_regheap_equals_libstdcxx(tmp_path):
    exe = str(tmp_path / "regheap_check")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "wiser_amd", "csrc"),
                           os.path.join(ROOT, "tests", "cpp", "regheap_check.cc"), "-o", exe])
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("ok "), r.stdout
