"""Kernel unit tests, each stage run alone on host-made input and
compared with a plain Python reference of the same step:

* stable compaction of the compat map's fixed [line * 20 + k] slots (replaces
  thrust::partition, reference main.cu:411) -- random live masks, order preserved;
* boundary mark + head compaction + adjacent difference over sorted keys (kernFindUniqBool /
  partition #3 / kernGetCount, main.cu:161-238,462) on both the LDS and the global path;
* radix sort up to 10^7 keys.

Sizes span < 1 tile, exactly 32,768 and 32,769 (the reference's 128 x 256 launch silently
drops element 32,768: bug B3) and several tiles."""
import random

import pytest

import locust_amd as lc

pytestmark = pytest.mark.gpu

E = 20  # EMITS_PER_LINE


def runs_reference(keys):
    """(key, val, count) of each run of a sorted list: val = index of the run's first key."""
    out = []
    for i, k in enumerate(keys):
        if i == 0 or k != keys[i - 1]:
            out.append([k, i, 0])
        out[-1][2] += 1
    return [tuple(e) for e in out]


@pytest.mark.parametrize("num_lines,density", [(1, 1.0), (13, 0.5), (1638, 1.0), (1639, 1.0),
                                               (1639, 0.3), (5000, 0.05), (20000, 0.7)])
def test_compact_slots_stable(num_lines, density):
    """1,638 full lines = 32,760 live slots; 1,639 = 32,780 (crosses 32,768)."""
    rng = random.Random(num_lines * 7 + int(density * 10))
    counts = [E if density == 1.0 else sum(rng.random() < density for _ in range(E))
              for _ in range(num_lines)]
    # live slots carry unique keys; dead slots carry junk that must not leak through
    slots = [b"l%dk%d" % (l, k) if k < counts[l] else b"dead"
             for l in range(num_lines) for k in range(E)]
    eng = lc.Engine(lc.make_config("gpu", map_path="compat"), num_lines * 64, num_lines)
    dense = eng.compact_slots(counts, slots)
    want = [slots[l * E + k] for l in range(num_lines) for k in range(counts[l])]
    assert dense == want


def test_compact_slots_all_empty_lines():
    eng = lc.Engine(lc.make_config("gpu", map_path="compat"), 1 << 16, 1000)
    assert eng.compact_slots([0] * 1000, [b""] * (1000 * E)) == []


def sorted_keys(n, nuniq, seed):
    rng = random.Random(seed)
    pool = sorted({bytes(rng.choice(b"abcdefghij\x80\xfe") for _ in range(rng.randint(1, 29)))
                   for _ in range(nuniq)})
    return sorted(rng.choice(pool) for _ in range(n))


@pytest.mark.parametrize("reduce_path", ["lds", "global"])
@pytest.mark.parametrize("n,nuniq", [(1, 1), (255, 40), (256, 256), (257, 3), (2048, 1),
                                     (32768, 5000), (32769, 5000), (32769, 32769),
                                     (250000, 20000)])
def test_reduce_sorted_mark_and_diff(n, nuniq, reduce_path):
    keys = sorted_keys(n, nuniq, n + nuniq)
    eng = lc.Engine(lc.make_config("gpu", reduce_path=reduce_path, sort="radix"),
                    max(n, 1) * 4, max(n // 8, 1))
    r = eng.reduce_sorted(keys)
    assert r.entries() == runs_reference(keys)
    assert r.num_unique == len(set(keys))


def test_reduce_sorted_run_across_tile_edges():
    """A run that starts in one tile and ends several tiles later, and one-key runs at every
    tile edge of the LDS variant (2,048 keys per tile)."""
    keys = []
    for t in range(6):
        keys += [b"a%02d" % t] * 2047 + [b"b%02d" % t]
    keys = sorted(keys + [b"zz"] * 5000)
    for path in ("lds", "global"):
        eng = lc.Engine(lc.make_config("gpu", reduce_path=path, sort="radix"), 1 << 20, 1 << 12)
        assert eng.reduce_sorted(keys).entries() == runs_reference(keys)


@pytest.mark.timeout(600)
def test_radix_sort_ten_million():
    """10^7 keys through the onesweep passes (planned on the host)."""
    n = 10_000_000
    rng = random.Random(7)
    pool = [b"%x" % rng.getrandbits(rng.randint(4, 60)) for _ in range(1 << 16)]
    keys = [pool[rng.getrandbits(16)] for _ in range(n)]
    eng = lc.Engine(lc.make_config("gpu", sort="radix"), 1 << 25, 1 << 20)
    s, perm = eng.sort_keys(keys)
    want = sorted(keys)
    assert s == want
    del want
    # the permutation is a stable one: equal keys keep input order
    assert all(keys[a] < keys[b] or (keys[a] == keys[b] and a < b)
               for a, b in zip(perm[:200000], perm[1:200001]))


def merge_reference(runs):
    """Python reference of the root merge: sum counts per key over all runs, sort, and
    val = total count of the smaller keys."""
    tot = {}
    for run in runs:
        for k, c in run:
            tot[k] = tot.get(k, 0) + c
    out, at = [], 0
    for k in sorted(tot):
        out.append((k, at, tot[k]))
        at += tot[k]
    return out


def _random_runs(rng, nruns, vocab, per_run):
    # keys sharing 8- and 16-byte prefixes exercise the later key words of the compare
    words = ([b"w%d" % i for i in range(vocab // 2)] +
             [b"abcdefgh%05d" % i for i in range(vocab // 4)] +
             [b"abcdefghijklmnop%03d" % i for i in range(vocab - vocab // 2 - vocab // 4)])
    runs = []
    for _ in range(nruns):
        n = rng.randint(0, per_run)
        ks = sorted(rng.sample(words, min(n, len(words))))
        runs.append([(k, rng.randint(1, 1000)) for k in ks])
    return runs


@pytest.mark.parametrize("nruns,vocab,per_run", [(1, 50, 50), (2, 100, 80), (3, 5000, 4000),
                                                 (8, 8000, 5608), (9, 3000, 3000),
                                                 (17, 2000, 300), (64, 400, 100)])
def test_merge_sorted_runs(nruns, vocab, per_run):
    """Gather-strategy root merge (lock-step binary search + look-back scan) against the
    Python reference: overlapping, disjoint and empty runs, up to 64 runs, > 1 scan tile."""
    rng = random.Random(nruns * 1000 + vocab)
    runs = _random_runs(rng, nruns, vocab, per_run)
    eng = lc.Engine(lc.make_config("gpu"), 1 << 20, 1 << 16)
    res = eng.merge_runs(runs)
    want = merge_reference(runs)
    assert res.entries() == want
    assert res.num_unique == len(want)
    assert res.num_tokens == sum(c for run in runs for _, c in run)


def test_merge_sorted_runs_skewed():
    """Runs whose key ranges barely overlap: disjoint blocks, one dense run packed between two
    neighbouring keys of a sparse one, and a run holding every key."""
    rng = random.Random(7)
    runs = [[(b"%02d-%05d" % (r, i), rng.randint(1, 9)) for i in range(r * 300)]
            for r in range(6)]
    runs.append([(b"m%07d" % (i * 1000), 1) for i in range(3000)])   # sparse
    runs.append([(b"m%07d" % i, 2) for i in range(1, 999)])          # inside one gap
    runs.append([(k, 3) for k in sorted({k for run in runs for k, _ in run})])
    eng = lc.Engine(lc.make_config("gpu"), 1 << 20, 1 << 16)
    res = eng.merge_runs(runs)
    want = merge_reference(runs)
    assert res.entries() == want
    assert res.num_tokens == sum(c for run in runs for _, c in run)


def test_merge_sorted_runs_empty():
    eng = lc.Engine(lc.make_config("gpu"), 1 << 16, 1 << 10)
    res = eng.merge_runs([[], []])
    assert res.entries() == [] and res.num_unique == 0
