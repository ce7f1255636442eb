"""Job configuration helpers (runtime replacements for the reference's #defines).

Reference: /root/reference/MapReduce/src/main.cu:18-37 (GPU_IMPLEMENTATION, SHARE_MEMORY,
EMITS_PER_LINE, GRID_SIZE, ...).  Every switch is a field of the native ``JobConfig``;
``LOCUST_*`` environment variables override the defaults.
"""
from __future__ import annotations

import os

from ._native import load

_C = load()

_REDUCE = {"lds": _C.ReducePath.lds, "global": _C.ReducePath.global_}
_MAP = {"compat": _C.MapPath.compat, "fast": _C.MapPath.fast}
_SORT = {"radix": _C.SortPath.radix, "dict": _C.SortPath.dict}
_BACKEND = {"gpu": _C.Backend.gpu, "cpu": _C.Backend.cpu}


def make_config(
    backend: str = "gpu",
    *,
    device: int = 0,
    reduce_path: str | None = None,
    map_path: str | None = None,
    sort: str | None = None,
    emits_per_line: int = 20,
    max_key_len: int = 29,
    delimiters: str | None = None,
    ref_compat: bool = False,
    combine: bool = False,
    check: bool | None = None,
    sync_plan: bool = True,
    chunk_bytes: int | None = None,
    zero_copy_text: int | None = None,
    graph: int | None = None,
    ref_timers: bool = False,
):
    """Build a native ``JobConfig``.  ``None`` means: environment override or default."""
    cfg = _C.JobConfig()
    cfg.backend = _BACKEND[backend]
    cfg.device = device
    reduce_path = reduce_path or os.environ.get("LOCUST_REDUCE_PATH", "lds")
    map_path = map_path or os.environ.get("LOCUST_MAP_PATH", "fast")
    sort = sort or os.environ.get("LOCUST_SORT", "dict")
    cfg.reduce_path = _REDUCE[reduce_path]
    cfg.map_path = _MAP[map_path]
    cfg.sort_path = _SORT[sort]
    cfg.emits_per_line = emits_per_line
    cfg.max_key_len = max_key_len
    if delimiters is not None:
        cfg.delimiters = delimiters
    cfg.ref_compat = ref_compat
    cfg.combine = combine
    if check is None:
        check = os.environ.get("LOCUST_CHECK", "0") not in ("", "0")
    cfg.check = check
    cfg.sync_plan = sync_plan
    if chunk_bytes is None:
        chunk_bytes = int(os.environ.get("LOCUST_CHUNK_MB", "0")) << 20
    cfg.chunk_bytes = chunk_bytes
    if zero_copy_text is None:
        zero_copy_text = int(os.environ.get("LOCUST_ZERO_COPY", "-1"))
    cfg.zero_copy_text = zero_copy_text
    if graph is None:
        graph = int(os.environ.get("LOCUST_GRAPH", "-1"))
    cfg.graph = graph
    cfg.ref_timers = ref_timers
    return cfg


_STRATEGY = {"auto": _C.DistStrategy.auto, "shuffle": _C.DistStrategy.shuffle,
             "gather": _C.DistStrategy.gather}


def make_dist_config(world: int, job=None, *, samples_per_rank: int = 64, gather: bool = True,
                     strategy: str | None = None, gather_max_records: int | None = None,
                     **job_kwargs):
    """Distributed job config.  ``strategy``: auto (default, or ``LOCUST_DIST_STRATEGY``),
    shuffle (sample-sort all-to-all) or gather (combined records straight to rank 0)."""
    d = _C.DistConfig()
    d.strategy = _STRATEGY[strategy or os.environ.get("LOCUST_DIST_STRATEGY", "auto")]
    if gather_max_records is not None:
        d.gather_max_records = gather_max_records
    d.job = job if job is not None else make_config(**job_kwargs)
    d.world = world
    d.samples_per_rank = samples_per_rank
    d.gather = gather
    return d
