"""The 1/2/4/8-GPU table of a scaling run.

    python tools/scale_report.py SCALE_r05.json [more.json ...] [--md OUT.md]   ("-": stdin)

Takes the driver's SCALE_r*.json (or any file holding bench.py result lines: a JSON
document at any nesting, JSON lines, or text with the lines inside) and prints, per GPU
count N:

* the headline (whole Hamlet, weak scaling: every rank maps its own copy) and its weak
  efficiency T(1) / T(N);
* the synth1m point (1M synthetic lines in total, strong scaling: 1/N per rank) with its
  throughput and strong efficiency T(1) / (N x T(N)) against the N = 1 synth1m point;
* from the line's scale_diag (N > 1): the min / max over ranks of the map, exchange,
  merge and emit stages, the bytes each rank sent (max over ranks), whether every pair of
  GPUs had direct access, the RCCL transports seen, and the largest per-rank peak RSS;
* the exchange strategy of the headline and of synth1m ("local" at N = 1), the largest
  per-rank engine device memory (HBM plan);
* a run that failed ("status": "failed", the watchdog's line): its reason and every rank's
  last stage instead of the numbers.
"""
from __future__ import annotations

import argparse
import json
import sys


def bench_lines(obj) -> list[dict]:
    """Every bench.py result line inside obj (dicts with "metric" and "n_gpus")."""
    out = []
    if isinstance(obj, dict):
        if "metric" in obj and "n_gpus" in obj and "value" in obj:
            out.append(obj)
        else:
            for v in obj.values():
                out += bench_lines(v)
    elif isinstance(obj, list):
        for v in obj:
            out += bench_lines(v)
    elif isinstance(obj, str) and '"metric"' in obj:
        for ln in obj.splitlines():
            ln = ln.strip()
            if ln.startswith("{") and '"metric"' in ln:
                try:
                    out += bench_lines(json.loads(ln))
                except ValueError:
                    pass
    return out


def load(paths: list[str]) -> list[dict]:
    lines = []
    for p in paths:
        text = sys.stdin.read() if p == "-" else open(p, errors="replace").read()
        try:
            lines += bench_lines(json.loads(text))
        except ValueError:
            lines += bench_lines(text)
    best: dict[int, dict] = {}
    for ln in lines:  # one line per N: the last one seen
        best[int(ln["n_gpus"])] = ln
    return [best[n] for n in sorted(best)]


def _mm(v) -> str:
    return "-" if not v else f"{v[0]:.3f}-{v[1]:.3f}"


def table(lines: list[dict]) -> str:
    if not lines:
        return "no bench.py result lines found\n"
    one = next((ln for ln in lines if ln["n_gpus"] == 1), None)
    t1 = one["value"] if one else None
    s1 = (one.get("synth1m") or {}).get("ms_per_step") if one else None
    rows = ["| N | headline ms | weak eff | synth1m ms | GB/s | strong eff | map ms | exchange ms | "
            "merge ms | emit ms | max sent MB | all pairs direct | transports | max RSS MB |",
            "|---:|---:|---:|---:|---:|---:|---|---|---|---|---:|---|---|---:|"]
    fails = []
    for ln in lines:
        n = ln["n_gpus"]
        if ln.get("status") == "failed" or ln.get("value") is None:
            prog = ln.get("progress") or {}
            stages = ", ".join(f"r{r}: {v.get('stage', '?')}" if isinstance(v, dict) else f"r{r}: {v}"
                               for r, v in sorted(prog.items(), key=lambda kv: str(kv[0])))
            fails.append(f"N={n}: failed ({ln.get('reason', '?')}); last stages: {stages or '-'}")
            rows.append(f"| {n} | failed | - | - | - | - | - | - | - | - | - | - | - | - |")
            continue
        sy = ln.get("synth1m") or {}
        sms = sy.get("ms_per_step")
        weak = f"{t1 / ln['value']:.2f}" if t1 else "-"
        strong = f"{s1 / (n * sms):.2f}" if s1 and sms else "-"
        d = ln.get("scale_diag") or {}
        st = d.get("stages_ms_min_max") or {}
        ranks = d.get("ranks") or []
        sent = max((sum(r.get("sent_to") or []) for r in ranks), default=0)
        acc = [a for r in ranks for a in (r.get("peer_access") or []) if a is not None]
        direct = "-" if not acc else ("yes" if all(acc) else f"{sum(acc)}/{len(acc)}")
        tr = sorted({t for r in ranks for v in (r.get("transport") or {}).values() for t in v})
        rss = d.get("peak_rss_kb_max")
        rows.append(
            f"| {n} | {ln['value']:.4f} | {weak} | {sms if sms is not None else '-'} | "
            f"{sy.get('GB_per_s', '-')} | {strong} | {_mm(st.get('map'))} | "
            f"{_mm(st.get('exchange'))} | {_mm(st.get('merge'))} | {_mm(st.get('emit'))} | "
            f"{sent / 1e6:.2f} | {direct} | {', '.join(tr) or '-'} | "
            f"{rss / 1024:.0f} |" if rss else
            f"| {n} | {ln['value']:.4f} | {weak} | {sms if sms is not None else '-'} | "
            f"{sy.get('GB_per_s', '-')} | {strong} | {_mm(st.get('map'))} | "
            f"{_mm(st.get('exchange'))} | {_mm(st.get('merge'))} | {_mm(st.get('emit'))} | "
            f"{sent / 1e6:.2f} | {direct} | {', '.join(tr) or '-'} | - |")
    extra = []
    for ln in lines:
        if ln.get("value") is None:
            continue
        d = ln.get("scale_diag") or {}
        hbm = d.get("hbm_device_bytes_max")
        extra.append(f"N={ln['n_gpus']}: strategy {ln.get('strategy') or '-'} (headline), "
                     f"{(ln.get('synth1m') or {}).get('strategy', '-')} (synth1m)"
                     + (f"; engine device memory max {hbm / 2**30:.2f} GiB per rank" if hbm else ""))
    note = ("\nweak eff = T(1) / T(N) of the headline (per-rank work fixed); strong eff = "
            "T(1) / (N x T(N)) of synth1m (total work fixed), against the N = 1 synth1m point.\n")
    tail = "".join(f"\n{x}" for x in extra + fails)
    return "\n".join(rows) + "\n" + note + (tail + "\n" if tail else "")


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("files", nargs="+")
    ap.add_argument("--md", default="")
    a = ap.parse_args(argv)
    txt = table(load(a.files))
    sys.stdout.write(txt)
    if a.md:
        with open(a.md, "w") as f:
            f.write(txt)
    return 0


if __name__ == "__main__":
    sys.exit(main())
