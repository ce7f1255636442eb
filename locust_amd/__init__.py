"""Locust-MI355X: a GPU MapReduce engine for AMD Instinct MI355X (gfx950).

Capabilities of wuyan33/Locust (GPU WordCount MapReduce with a CPU reference path and a
socket-based distributor), re-designed MI355X-first:

* Map / Process / Reduce are hand-written HIP kernels for CDNA4 wave64 (device strtok_r,
  byte-parallel tokenizer, decoupled look-back scans, LSD radix sort on packed keys,
  LDS-staged boundary-mark / adjacent-difference reduce) -- see ``csrc/kernels``.
* Multi-GPU runs shard the input by bytes, range-partition with sample-sort splitters and
  exchange 40-byte (key, count) records over xGMI (``csrc/comm``): a first job sizes the
  exchange from an all-gathered count matrix (grouped ``ncclSend``/``ncclRecv`` with exact
  sizes, two host syncs), later jobs use one fixed-slot ``ncclAllToAll`` (every bucket
  padded to the previous job's largest bucket + 1/8, one host sync).  Every rank writes its
  key range straight into one shared host output (a POSIX shm segment each rank registers
  with HIP) at its global offset -- no gather to rank 0.  Small combined outputs of
  repeated jobs go to rank 0 in one ``ncclAllGather`` of device-written slots.
* The reference's ``./MapReduce <file> [start end] [node stage]`` CLI and output format are
  kept byte-for-byte (``build/MapReduce``).

Quick start::

    import locust_amd as lc
    res = lc.wordcount_file("data/hamlet.txt", 0, 700)          # GPU
    print(res.format().decode()[:200])
    res_cpu = lc.wordcount_file("data/hamlet.txt", 0, 700, backend="cpu")
"""
from __future__ import annotations

import os as _os

# Captured RCCL collectives (the gather-slot job replays map + all-gather + merge as one
# hipGraph) stay on RCCL's own connection buffers instead of IPC-registering ours.  Set
# once, at import, before any RCCL communicator or engine thread exists; a user's explicit
# setting wins.
_os.environ.setdefault("NCCL_GRAPH_REGISTER", "0")
# Code objects: the engines load this library's own kernel files at construction (see
# warm_kernel_modules in csrc/include/locust/kernels.hpp), so a fresh process's first job
# does not pay lazy loading inside it -- without HIP_ENABLE_DEFERRED_LOADING=0, which would
# also load RCCL's 573 MB of device code into every process (+1.3 GB of host memory).

from ._native import REPO_ROOT, build, cli_path, load  # noqa: E402

_C = load()

from .config import make_config, make_dist_config  # noqa: E402
from .models.wordcount import (  # noqa: E402
    Engine,
    WordCount,
    map_stage,
    reduce_stage,
    run_multi,
    wordcount_file,
    wordcount_text,
)

JobConfig = _C.JobConfig
DistConfig = _C.DistConfig
LocustError = _C.LocustError
HostText = _C.HostText
gen_text = _C.gen_text  # synthetic Hamlet-shaped text (csrc/io/gen.cpp)

__all__ = [
    "REPO_ROOT",
    "build",
    "cli_path",
    "make_config",
    "make_dist_config",
    "Engine",
    "WordCount",
    "map_stage",
    "reduce_stage",
    "run_multi",
    "wordcount_file",
    "wordcount_text",
    "JobConfig",
    "DistConfig",
    "LocustError",
    "HostText",
    "gen_text",
]
__version__ = "0.1.0"
