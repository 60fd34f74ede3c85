"""Test helper: pure-Python model of the reference ranking (used only to check
the doc-range shard exchange on CPU).  BM25 in IEEE double with the reference's
operation order (scoring.h:21-25,65-69,85-90,124-145) and the libstdc++
push_heap/pop_heap restated with comparator a.score > b.score
(query_processing.h:510-524,551-562,588-603)."""
import math


def char4_decode(c):
    mant, sh = c & 7, (c >> 3) - 1
    return mant if sh < 0 else ((mant | 8) << sh) & 0xFFFFFFFF


def idf(n, df):
    return math.log(1 + (n - df + 0.5) / (df + 0.5))


def norm(c4, avg):
    return 1.2 * (1 - 0.75 + 0.75 * char4_decode(c4) / avg)


def tfn(tf, nrm):
    return (tf * (1.2 + 1)) / (tf + nrm)


class Heap:
    def __init__(self):
        self.v = []

    def _push_hole(self, hole, top, val):
        parent = (hole - 1) // 2
        while hole > top and self.v[parent][0] > val[0]:
            self.v[hole] = self.v[parent]
            hole = parent
            parent = (hole - 1) // 2
        self.v[hole] = val

    def push(self, val):
        self.v.append(val)
        self._push_hole(len(self.v) - 1, 0, val)

    def pop(self):
        if len(self.v) > 1:
            ln = len(self.v) - 1
            val = self.v[ln]
            self.v[ln] = self.v[0]
            hole, child = 0, 0
            while child < (ln - 1) // 2:
                child = 2 * (child + 1)
                if self.v[child][0] > self.v[child - 1][0]:
                    child -= 1
                self.v[hole] = self.v[child]
                hole = child
            if (ln & 1) == 0 and child == (ln - 2) // 2:
                child = 2 * (child + 1)
                self.v[hole] = self.v[child - 1]
                hole = child - 1
            self._push_hole(hole, 0, val)
        self.v.pop()


def rank_stream(items, k):
    """RankDoc over (score, doc) items in doc order -> (SortHeap result, insertions)."""
    h, ins = Heap(), []
    for s, d in items:
        if len(h.v) < k:
            h.push((s, d)); ins.append((s, d))
        elif s > h.v[0][0]:
            h.pop(); h.push((s, d)); ins.append((s, d))
    out = []
    while h.v and len(out) < k:
        out.append(h.v[0]); h.pop()
    return out[::-1], ins


class WaveHeapModel:
    """The device's wave-parallel restatement of the same heap (kernels.hip
    WaveHeap): entry i in lane i; a sift up moves, in one step, every ancestor
    whose score is > the value one level down (they are the deepest part of the
    chain, since scores never decrease going down); a pop first shifts the
    root-to-hole path of 'second children' up one level, then sifts the old last
    entry up from the hole.  Must leave the array exactly as Heap does."""

    def __init__(self):
        self.v = []

    def _sift_up(self, hole, anc, val):
        L = [x for x in anc if self.v[x][0] > val[0]]
        if not L:
            self.v[hole] = val
            return
        old = list(self.v)
        chain = set(anc) | {hole}
        for y in chain:
            if y != 0 and (y - 1) // 2 in L:
                self.v[y] = old[(y - 1) // 2]
        self.v[min(L)] = val

    @staticmethod
    def _ancestors(h):
        out = []
        while h > 0:
            h = (h - 1) // 2
            out.append(h)
        return out

    def push(self, val):
        self.v.append(None)
        h = len(self.v) - 1
        self._sift_up(h, self._ancestors(h), val)

    def pop(self):
        n = len(self.v)
        if n > 1:
            ln = n - 1
            val = self.v[ln]
            old = list(self.v)

            def nxt(i):   # __adjust_heap's choice: the right child unless it is > the left
                return 2 * i + 1 if old[2 * i + 2][0] > old[2 * i + 1][0] else 2 * i + 2
            path, h = [0], 0
            while h < (ln - 1) // 2:
                h = nxt(h)
                path.append(h)
            if (ln & 1) == 0 and h == (ln - 2) // 2:
                h = 2 * h + 1
                path.append(h)
            for a, b in zip(path, path[1:]):
                self.v[a] = old[b]
            self._sift_up(h, path[:-1], val)
        self.v.pop()
