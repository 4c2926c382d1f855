"""The multi-rank stress loop's inputs and its wrong-element classifier
(tests/test_gpu_multirank.py's worker imports this; tests/test_stress_records.py
checks the classifier against the wrong results recorded in rounds 3-4,
DESIGN.md §2).

Every input element carries a per-(call, rank) signature, so a wrong element
names where its bytes came from: zero, a missing or stale contribution of one
rank, an earlier call's result, the readback sentinel, or this rank's own input
shifted by a few elements (a host buffer the device-to-host copy left unwritten
keeps what the allocator's previous user stored there)."""
import numpy as np

SENT_HOST = 0xA5                      # the pageable readback's prefill byte


def ivec(it, r, n):
    # the high term differs per (call, rank), so a wrong value names its source
    hi = (((it * 2654435761) ^ (r * 40503)) % 4093) << 17
    return ((np.arange(n, dtype=np.int64) * 7 + it * 31 + r * 1009) % 100003 + hi).astype(np.int32)


def stress_n(it):
    return (1 << 18) if it % 50 == 49 else (1, 5, 64, 1000, 4096, 65536, 100003, 300001)[it % 8]


def stress_input(it, r, p):
    # what rank r sent in iteration `it` (the reduce_scatter_block calls send p blocks)
    n = stress_n(it)
    return ivec(it, r, n * p if it % 9 == 4 and it % 7 != 3 else n)


def classify(it, n, e, got_e, tot_e, p, rank, back=24):
    """Hypotheses that explain the wrong elements at indices `e` (values
    `got_e`, expected `tot_e`); a hypothesis explaining only part of them is
    reported with its count.  Wrapping int32 arithmetic."""
    e = np.asarray(e)
    g, t = np.asarray(got_e).astype(np.int64), np.asarray(tot_e).astype(np.int64)
    w = lambda v: (np.asarray(v).astype(np.int64) & 0xFFFFFFFF)
    hyp = []

    def note(name, ok):
        k = int(np.count_nonzero(ok))
        if k == e.size:
            hyp.append(name)
        elif k:
            hyp.append(f"{name} ({k} of {e.size})")

    note("zero", g == 0)
    note("readback sentinel", w(g) == SENT_HOST * 0x01010101)
    mine = ivec(it, rank, n)
    for s in range(-16, 17):
        if 0 <= e.min() + s and e.max() + s < n:
            note(f"own input {s:+d}", g == mine[e + s])
    for r in range(p):
        x = ivec(it, r, n)[e].astype(np.int64)
        note(f"missing r{r}", w(t - x) == w(g))
        for b in range(1, back + 1):
            i2 = it - b
            if i2 < 0:
                break
            old = stress_input(i2, r, p)
            if e.max() < old.size:
                note(f"stale r{r} from it{i2}", w(t - x + old[e]) == w(g))
    for b in range(1, back + 1):
        i2 = it - b
        n2 = stress_n(i2) if i2 >= 0 else 0
        if i2 >= 0 and e.max() < n2:
            t2 = sum(ivec(i2, r, n2)[e].astype(np.int64) for r in range(p))
            note(f"result of it{i2}", w(t2) == w(g))
    return hyp
