// Process-wide cache of large device blocks (engine arenas, streamed-chunk buffers).
//
// Engines come and go inside one process (the bench's cold probe, the CLI's stage engines,
// the Python API, distributed ranks adding engines).  Returning every arena to the driver
// and asking for a new one made a later engine's 256 MiB chunk copies run at ~30 GB/s
// instead of ~57 (tools/s10g_probe.py, profiles/r3_s4/), and costs a hipMalloc of several
// GB per engine.  Freed blocks are kept per device and handed to the next request that
// fits (best fit, at most 5/4 of the request), like a caching allocator; on an allocation
// failure the cache is emptied and the allocation retried.  LOCUST_DEV_CACHE=0 switches
// it off (every block goes straight back to hipFree), LOCUST_DEV_CACHE_GB caps what is
// kept (default 64 GB of the 288 GB per MI355X).
#pragma once

#include <cstddef>

namespace locust {

// A device block of at least `bytes` on the current device (whole 2 MiB pages).  Its
// size is written to *got.  Throws locust::Error when the device is out of memory.
void* dev_block_alloc(size_t bytes, size_t* got);
// Give a block back: the caller's work on it must be complete (the engines synchronise
// their streams first).  Kept for reuse unless the cache is off or full.
void dev_block_free(void* p, size_t bytes);
// hipFree every cached block (all devices).
void dev_block_trim();
// Cached blocks / bytes (tests, logs).
size_t dev_block_cached(size_t* bytes = nullptr);

// Pinned host memory (hipHostMalloc with `flags`) for `what`, logged at LOCUST_LOG=debug
// when >= 1 MiB with the process's running total of pinned allocations: where a
// multi-rank run's host memory goes.  Throws locust::Error on failure.
// A buffer of >= 4 MiB (read rings, chunk staging, one-pass text, key downloads, the
// mapped result buffers) is instead anonymous memory advised to transparent huge pages,
// first-touched here and hipHostRegister'ed (mapped; registered memory is fine-grained
// unless asked otherwise, like a coherent hipHostMalloc): page-locking 64 MiB took 8-12 ms through
// hipHostMalloc -- the 4 KiB page faults -- and 3.7 ms this way (tools/micro/pin_probe.hip;
// LOCUST_HUGE_PIN=0: hipHostMalloc for everything).  Free with pinned_free.
void* pinned_alloc(size_t bytes, unsigned flags, const char* what);
// Frees a pinned_alloc buffer (hipHostUnregister + munmap, or hipHostFree).  Null: no-op.
void pinned_free(void* p);

}  // namespace locust
