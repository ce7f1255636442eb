"""The fast map's XCD-ordered tiles (csrc/kernels/map_tile.hpp xcd_tile): block b of a
G-block launch maps tile x * q + min(x, r) + k (x = b % 8, k = b // 8, q, r = divmod(G, 8)).
Every tile must be mapped exactly once whatever G, and the kernel must use the mapping
only as a permutation (part_off rows and traces are indexed by tile, not by block)."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def xcd_tile(b: int, g: int) -> int:
    q, r = divmod(g, 8)
    x, k = b % 8, b // 8
    return x * q + min(x, r) + k


def test_xcd_tile_is_a_bijection():
    for g in list(range(1, 300)) + [1023, 1024, 1025, 4096, 4099]:
        tiles = sorted(xcd_tile(b, g) for b in range(g))
        assert tiles == list(range(g)), g


def test_each_xcd_takes_a_contiguous_run():
    g = 188  # whole Hamlet in 1 KiB tiles
    for x in range(8):
        mine = [xcd_tile(b, g) for b in range(x, g, 8)]
        assert mine == list(range(mine[0], mine[0] + len(mine)))


def test_device_formula_matches():
    src = open(os.path.join(ROOT, "csrc", "kernels", "map_tile.hpp")).read()
    body = src[src.index("__device__ __forceinline__ u32 xcd_tile("):]
    body = body[:body.index("}") + 1]
    assert "x * q + (x < r ? x : r) + k" in body
    assert re.search(r"q = G / kXcds, r = G % kXcds, x = b % kXcds, k = b / kXcds", body)
    tok = open(os.path.join(ROOT, "csrc", "kernels", "tokenize.hip")).read()
    assert "xcd_tile(blockIdx.x, gridDim.x)" in tok
