"""The small-pass route (csrc/engine/pipeline.hip shape_arena): an engine for
at most LOCUST_SMALL_PASS_KB (default 1024) KiB whose worst-case token count passes
kPartBuildMaxTokens (2^18) keeps the one-kernel ordered build and its in-job plan.
Inputs of 0.5-1 MiB -- 3x and 5x Hamlet, one repeated key, all-distinct random keys, one
crowded partition -- each checked against the independent oracle with the route on and
off (LOCUST_SMALL_PASS_KB=0: the two-kernel large build), job after job (the first job
plans in-job, later ones run on the retuned map), and the HBM-table fallbacks counted."""
import random

import pytest

import locust_amd as lc
from locust_amd.utils import oracle

pytestmark = pytest.mark.gpu


def _inputs(hamlet: bytes):
    rng = random.Random(17)
    yield "hamlet3x", hamlet * 3
    yield "hamlet5x", hamlet * 5
    yield "one_key", b"\n".join(b" ".join([b"the"] * 10) for _ in range(20_000)) + b"\n"
    alpha = b"abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ"
    words = {bytes(rng.choice(alpha) for _ in range(rng.randrange(4, 12))) for _ in range(90_000)}
    words = sorted(words)
    rng.shuffle(words)
    yield "random_distinct", b"\n".join(b" ".join(words[i:i + 4]) for i in range(0, len(words), 4)) + b"\n"
    crowd = [b"w%06d" % i for i in range(120_000)]  # every key in one starting-map partition
    yield "crowded", b"\n".join(b" ".join(crowd[i:i + 5]) for i in range(0, len(crowd), 5)) + b"\n"


@pytest.mark.parametrize("small_pass_kb", [None, "0"])
def test_small_pass_route_matches_oracle(hamlet, monkeypatch, small_pass_kb):
    if small_pass_kb is None:
        monkeypatch.delenv("LOCUST_SMALL_PASS_KB", raising=False)
    else:
        monkeypatch.setenv("LOCUST_SMALL_PASS_KB", small_pass_kb)
    for name, text in _inputs(hamlet):
        assert (1 << 19) <= len(text) <= (1 << 20), (name, len(text))
        ent, ntok, _ = oracle.wordcount(text)
        eng = lc._C.GpuEngine(lc.make_config("gpu", reduce_path="lds"), len(text),
                              text.count(b"\n") + 1)
        assert eng.capacity > (1 << 18), name  # past kPartBuildMaxTokens: the route applies
        for j in range(3):
            r = eng.run(text)
            assert r.num_tokens == ntok, (name, j)
            assert r.entries() == ent, f"{name} job {j}: entries differ from the oracle"
        st = eng.stats()
        # a fallback redoes the job on the HBM table (still exact, above).  Hamlet never
        # needs one.  One key repeated 200,000 times: on the small-pass route it is one
        # partition past the LDS token window in every job, whatever the plan (all its
        # quantile cuts are the same key); the large build's per-tile combining folds it
        # into one record per tile first, so it never falls back
        if name.startswith("hamlet"):
            assert st["fallbacks"] == 0, (name, st)
        if name == "one_key":
            assert st["fallbacks"] == (3 if small_pass_kb is None else 0), (name, st)
