"""Partition map of the ordered dictionary build (locust/partmap.hpp): order-preserving
2-byte-prefix ranges balanced by work, checked on the host (no GPU)."""
import collections

import locust_amd as lc
from locust_amd.utils import oracle


def _weights(entries):
    w = collections.Counter()
    for k, _v, c in entries:
        b = (k + b"\0\0")[:2]
        w[b[0] << 8 | b[1]] += c + 3
    return w


def test_balanced_map_is_monotone_and_covers(hamlet):
    ent = oracle.wordcount(hamlet)[0]
    m = lc._C.part_map_build([(k, c) for k, _v, c in ent])
    part = m["part"]
    assert all(part[b] <= part[b + 1] for b in range(65535)), "not order-preserving"
    assert part[0] == 0 and part[65535] <= 255
    lo = m["lo"]
    for p in range(257):
        if p <= part[65535]:
            assert part[lo[p]] == p and (lo[p] == 0 or part[lo[p] - 1] < p)
        else:
            assert lo[p] == 65536
    # every row uses at most 8 thresholds, and the lookup formula reproduces `part`
    for c in range(256):
        thr = [(m["thr"][c] >> (8 * i)) & 0xFF for i in range(8)]
        for d in range(256):
            assert part[c << 8 | d] == m["base"][c] + sum(1 for t in thr if t and t <= d)
    # balance: far below the first-letter map's largest partition
    w = _weights(ent)
    first = collections.Counter()
    for b, x in w.items():
        first[b >> 8] += x
    by_part = collections.Counter()
    for b, x in w.items():
        by_part[part[b]] += x
    assert max(by_part.values()) == m["predicted_max"]
    # 't' (4,555) and 's' split; the largest partition is the unsplittable 'th' prefix
    hot = max(w.values())
    assert m["predicted_max"] < max(first.values()) and m["predicted_max"] == hot
    # every other partition is at most ~8 x the ideal share (8 thresholds per first byte)
    second = sorted(by_part.values())[-2]
    assert second <= 8 * sum(w.values()) // 256


def test_default_map_for_empty_input():
    m = lc._C.part_map_build([])
    assert m["part"][0x7468] == 0x74 and m["predicted_max"] == 0
