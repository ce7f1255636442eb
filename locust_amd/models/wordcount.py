"""WordCount -- the reference's one job (README.md:26-62), as a reusable job object.

``Engine`` keeps a preallocated device pipeline (HBM arena, pinned staging, stream,
events) alive across runs, so repeated jobs pay no allocation.  ``WordCount`` is the
user-facing job: load a file or a text window, run on one GPU, many GPUs (loopback in
one process) or the CPU reference path, and format the reference's output.
"""
from __future__ import annotations

from dataclasses import dataclass, field

from .._native import load
from ..config import make_config, make_dist_config

_C = load()


class Engine:
    """Single-device engine with fixed capacity (bytes, lines)."""

    def __init__(self, cfg=None, max_bytes: int = 1 << 20, max_lines: int = 1 << 15):
        self.cfg = cfg if cfg is not None else make_config()
        self.cpu = self.cfg.backend == _C.Backend.cpu
        self._eng = None if self.cpu else _C.GpuEngine(self.cfg, max_bytes, max_lines)

    @property
    def capacity(self) -> int:
        return 0 if self.cpu else self._eng.capacity

    def run(self, text: bytes):
        if self.cpu:
            return _C.cpu_run(self.cfg, text)
        return self._eng.run(text)

    def map_stage(self, text: bytes) -> list[bytes]:
        """Map + sort only (stage 1): the sorted token list of ``text``."""
        if self.cpu:
            return _C.cpu_map_stage(self.cfg, text)
        return self._eng.map_stage(text)

    def reduce_stage(self, keys: list[bytes]):
        """Reduce only (stage 2) over tokens in any order."""
        if self.cpu:
            text = b"\n".join(keys)
            return _C.cpu_run(self.cfg, text)
        return self._eng.reduce_stage(keys)

    def sort_keys(self, keys: list[bytes]):
        """Device radix sort of byte-string keys: (sorted keys, permutation)."""
        if self.cpu:
            perm = sorted(range(len(keys)), key=lambda i: keys[i])
            return [keys[i] for i in perm], perm
        return self._eng.sort_keys(keys)

    def compact_slots(self, line_counts: list[int], slot_keys: list[bytes]) -> list[bytes]:
        """Stable compaction of fixed [line * emits_per_line + k] slots (compat engine):
        the first ``line_counts[l]`` slots of each line, in order."""
        return self._eng.compact_slots(line_counts, slot_keys)

    def reduce_sorted(self, keys: list[bytes]):
        """Boundary mark + head compaction + adjacent difference over sorted keys."""
        return self._eng.reduce_sorted(keys)

    def merge_runs(self, runs: list[list[tuple[bytes, int]]]):
        """Root merge of the gather strategy: runs of (key, count), each sorted with
        distinct keys -> merged (key, val, count) entries."""
        return self._eng.merge_runs(runs)


def wordcount_text(text: bytes, backend: str = "gpu", cfg=None, **kw):
    cfg = cfg if cfg is not None else make_config(backend, **kw)
    nlines = text.count(b"\n") + (1 if text and not text.endswith(b"\n") else 0)
    return Engine(cfg, max(len(text), 1), max(nlines, 1)).run(text)


def wordcount_file(path: str, line_start: int = -1, line_end: int = -1, backend: str = "gpu",
                   cfg=None, **kw):
    cfg = cfg if cfg is not None else make_config(backend, **kw)
    text, nlines, _first, _total = _C.load_lines(path, line_start, line_end, cfg.ref_compat)
    return Engine(cfg, max(len(text), 1), max(nlines, 1)).run(text)


def map_stage(path: str, spill: str, line_start: int = -1, line_end: int = -1,
              backend: str = "gpu", fmt: str = "binary", cfg=None, **kw) -> dict:
    """Stage 1 of the reference's split job (main.cu:421-433), count-carrying: the line
    window's combined (key, count) records -> ``spill`` (+ ``spill + ".idx"``); returns
    the counts, spill size and stage times.  ``fmt``: text | binary | kiv."""
    cfg = cfg if cfg is not None else make_config(backend, **kw)
    return _C.map_stage(cfg, path, line_start, line_end, spill, fmt)


def reduce_stage(spills: list[str], reducer: int = 0, reducers: int = 1,
                 backend: str = "gpu", cfg=None, **kw):
    """Stage 2: key range ``reducer`` of ``reducers`` over the spills, merged with counts
    summed (the device merge on the GPU); returns (result, stats).  The result's entries
    carry the global val; concatenating reducers 0..R-1 gives the single-stage result."""
    cfg = cfg if cfg is not None else make_config(backend, **kw)
    return _C.reduce_spills(cfg, list(spills), reducer, reducers)


def run_multi(text: bytes, world: int, backend: str = "gpu", combine: bool = True,
              samples_per_rank: int = 64, strategy: str | None = None, comm: str = "auto",
              **kw):
    """Multi-rank WordCount in this process, one thread per rank.  comm="auto" (and
    "loopback"): the loopback communicator -- ranks exchange by peer-to-peer device copies
    (over xGMI when the ranks' GPUs differ; rehearses N ranks on fewer GPUs).  comm="rccl":
    an RCCL clique (ncclCommInitAll), one GPU per rank -- opt-in until a run with real RCCL
    peers has been recorded (csrc/engine/dist_runner.hip resolve_local_comm)."""
    dcfg = make_dist_config(world, make_config(backend, combine=combine, **kw),
                            samples_per_rank=samples_per_rank, strategy=strategy)
    return _C.run_multi(text, dcfg, comm)


@dataclass
class WordCount:
    """A WordCount job description (the reference's only job)."""

    path: str | None = None
    line_start: int = -1
    line_end: int = -1
    backend: str = "gpu"
    gpus: int = 1
    options: dict = field(default_factory=dict)

    def load(self):
        cfg = make_config(self.backend, **self.options)
        return _C.load_lines(self.path, self.line_start, self.line_end, cfg.ref_compat)

    def run(self):
        text, _n, _first, _total = self.load()
        if self.gpus > 1:
            return run_multi(text, self.gpus, self.backend, **self.options)
        return wordcount_text(text, self.backend, **self.options)
