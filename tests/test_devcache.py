"""Process-wide device block cache (csrc/include/locust/devcache.hpp): an engine's arena
goes back to the cache when the engine is destroyed and the next engine of the same shape
reuses it (no hipMalloc, no new physical placement); results stay identical."""
import pytest


@pytest.mark.gpu
def test_engine_arena_is_reused_and_results_match(hamlet):
    import locust_amd as lc

    lc._C.dev_cache_trim()
    cfg = lc.make_config("gpu", reduce_path="lds")
    text = hamlet
    nl = text.count(b"\n") + 1
    eng = lc._C.GpuEngine(cfg, len(text), nl)
    first = eng.run(text).entries()
    del eng
    st = lc._C.dev_cache_stats()
    assert st["blocks"] >= 1 and st["bytes"] > 0
    eng = lc._C.GpuEngine(cfg, len(text), nl)
    assert lc._C.dev_cache_stats()["blocks"] == st["blocks"] - 1  # the arena came back out
    assert eng.run(text).entries() == first
    del eng
    lc._C.dev_cache_trim()
    assert lc._C.dev_cache_stats() == {"blocks": 0, "bytes": 0}
