"""Debug helper: per-run distinct counts of the large ordered path vs the CPU engine."""
import sys
import locust_amd as lc

lines = int(sys.argv[1]) if len(sys.argv) > 1 else 220000
h = lc._C.HostText.generate(lines=lines, seed=3)
want = lc._C.cpu_run(lc.make_config("cpu"), h.to_bytes()).entries()
print("cpu unique", len(want), "tokens", sum(c for _k, _v, c in want))
eng = lc._C.GpuEngine(lc.make_config("gpu", graph=0), h.size, h.size)
for i in range(4):
    r = eng.run_text(h)
    e = r.entries()
    print(i, "gpu unique", r.num_unique, "tokens", r.num_tokens, "sum", sum(c for _k, _v, c in e), "match", e == want)
