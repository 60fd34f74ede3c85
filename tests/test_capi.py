"""The C-ABI library loads, exports every symbol include/wiser_hip.h declares,
and fails loudly (no CPU fallback) when there is no HIP device.  CPU only."""
import ctypes as C
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_exports_every_declared_symbol(built):
    from wiser_amd import _capi
    names = _capi.header_symbols()
    assert len(names) >= 20
    missing = [n for n in names if not hasattr(_capi.lib, n)]
    assert not missing, missing


def test_version_and_error_string(built):
    from wiser_amd import _capi
    assert b"gfx950" in _capi.lib.wsr_version()
    h = C.c_void_p()
    rc = _capi.lib.wsr_open(b"/nonexistent/index", None, C.byref(h))
    assert rc == -2 and not h.value
    assert b"my.doc_length" in _capi.lib.wsr_last_error()


def test_no_cpu_fallback(built, indexes):
    """On a machine without a HIP device the engine refuses to load."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    import wiser_amd as w
    from wiser_amd._capi import WiserError
    d = indexes["three"][0]
    e = w.VacuumEngine(d)
    with pytest.raises(WiserError) as ei:
        e.Load()
    assert ei.value.code == -3 and "no CPU fallback" in str(ei.value)


def test_null_arguments_are_errors(built):
    from wiser_amd import _capi
    assert _capi.lib.wsr_open(None, None, None) == -1
    assert _capi.lib.wsr_term_count(None, None) == -1
    assert _capi.lib.wsr_search_batch(None, None, 1, 1, None, None) == -1
    _capi.lib.wsr_close(None)  # no-op


def test_struct_layouts(built, tmp_path):
    """ctypes mirrors agree with include/wiser_hip.h as compiled by gcc."""
    import subprocess
    from wiser_amd import _capi
    src = tmp_path / "sz.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "wiser_hip.h"\n'
                   'int main(void){printf("%zu %zu %zu %zu %zu %zu %zu %zu\\n", sizeof(wsr_query),'
                   ' offsetof(wsr_query, flags), offsetof(wsr_query, more_ids), sizeof(wsr_hit),'
                   ' sizeof(wsr_open_opts),'
                   ' offsetof(wsr_open_opts, positions), sizeof(wsr_batch_stats),'
                   ' sizeof(wsr_build_stats)); return 0;}\n')
    exe = tmp_path / "sz"
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)])
    got = [int(x) for x in subprocess.check_output([str(exe)]).split()]
    assert got == [C.sizeof(_capi.Query), _capi.Query.flags.offset, _capi.Query.more_ids.offset,
                   C.sizeof(_capi.Hit),
                   C.sizeof(_capi.OpenOpts), _capi.OpenOpts.positions.offset,
                   C.sizeof(_capi.BatchStats), C.sizeof(_capi.BuildStats)]
    assert C.sizeof(_capi.Query) == 88 and C.sizeof(_capi.Hit) == 16


def test_class_order_is_stable_and_class_pure(built):
    from wiser_amd import _capi
    """wsr_class_order (the engine's batch former): conjunctive queries first
    (a one-term phrase counts as a single-term query), then phrases of two or
    more terms, each class in its input order; class_batches cuts each class
    on its own."""
    import random
    import wiser_amd as w
    rng = random.Random(5)
    n = 1000
    arr = (_capi.Query * n)()
    kinds = []
    for i in range(n):
        nt = rng.choice([1, 2, 2, 3])
        ph = rng.random() < 0.15
        arr[i].n_terms = nt
        arr[i].flags = 1 if ph else 0
        kinds.append(ph and nt > 1)
    order, nc = w.class_order(arr)
    assert sorted(order) == list(range(n))
    assert nc == kinds.count(False)
    assert order[:nc] == [i for i in range(n) if not kinds[i]]
    assert order[nc:] == [i for i in range(n) if kinds[i]]
    bs = w.class_batches(arr, 128)
    assert [i for b in bs for i in b] == order
    assert all(len(b) <= 128 and len({kinds[i] for i in b}) == 1 for b in bs)
    assert _capi.lib.wsr_class_order(None, 3, None, None) == -1
