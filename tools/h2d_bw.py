"""H2D bandwidth probe: one large pinned copy vs piecewise copies on one or two streams."""
import torch

N = 43 << 20
h = torch.empty(N, dtype=torch.uint8).pin_memory()
h.fill_(7)
d = torch.empty(N, dtype=torch.uint8, device="cuda")
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def one():
    d.copy_(h, non_blocking=True)


def pieces(p, streams):
    def f():
        cur = torch.cuda.current_stream()
        ev = torch.cuda.Event()
        ev.record(cur)
        for s in streams:
            s.wait_event(ev)
        for k, o in enumerate(range(0, N, p)):
            s = streams[k % len(streams)]
            with torch.cuda.stream(s):
                d[o:o + p].copy_(h[o:o + p], non_blocking=True)
        for s in streams:
            cur.wait_stream(s)
    return f


for name, fn in [("one 43MiB", one), ("4MiB x1", pieces(4 << 20, [s1])),
                 ("4MiB x2", pieces(4 << 20, [s1, s2])), ("1MiB x1", pieces(1 << 20, [s1])),
                 ("8MiB x2", pieces(8 << 20, [s1, s2]))]:
    ms = timeit(fn)
    print(f"{name:12s} {ms:.3f} ms  {N / ms / 1e6:.1f} GB/s")

# D2H: one 9.7 MB copy (the synth1m output size) from device memory into pinned memory
M = 9728 << 10
dh = torch.empty(M, dtype=torch.uint8).pin_memory()
dd = torch.empty(M, dtype=torch.uint8, device="cuda")
ms = timeit(lambda: dh.copy_(dd, non_blocking=True))
print(f"D2H 9.5MiB   {ms:.3f} ms  {M / ms / 1e6:.1f} GB/s")
