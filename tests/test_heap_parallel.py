"""The wave-parallel heap restatement of the device (WaveHeap, kernels.hip)
against the serial libstdc++ __push_heap / __adjust_heap restatement
(heapmodel.Heap): identical arrays after every insertion (RankDoc) and an
identical SortHeap order, on streams with many tied scores."""
import random

from heapmodel import Heap, WaveHeapModel


def run(heap_cls, items, k):
    h, states = heap_cls(), []
    for s, d in items:
        if len(h.v) < k:
            h.push((s, d))
        elif s > h.v[0][0]:
            h.pop()
            h.push((s, d))
        states.append(list(h.v))
    out = []
    while h.v:
        out.append(h.v[0])
        h.pop()
        states.append(list(h.v))
    return states, out[::-1]


def test_wave_heap_equals_libstdcxx():
    rng = random.Random(2026)
    for trial in range(1500):
        k = rng.choice([1, 2, 3, 5, 8, 10, 16, 31, 32, 33, 63, 64])
        n = rng.randint(0, 400)
        alphabet = rng.choice([2, 3, 5, 20, 1000])
        items = [(float(rng.randint(1, alphabet)), d) for d in range(n)]
        assert run(WaveHeapModel, items, k) == run(Heap, items, k), (trial, k, alphabet)
