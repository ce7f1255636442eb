"""Per-window timeline of one streamed job from rocprofv3 --kernel-trace --memory-copy-trace
CSVs: for every map window, its H2D copies (bytes, time), the map kernel and the dictionary
insert, and where the job's time went (copies busy, kernels busy, neither) -- what bounds a
stage-1 map process's run (maps read at ~15-20 GB/s, the single stage
at ~33).

    python tools/stream_windows.py kernel_trace.csv memory_copy_trace.csv [--first N]
"""
import argparse
import csv


def spans(rows, name_key):
    out = []
    for r in rows:
        out.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get(name_key, ""), r))
    out.sort()
    return out


def busy(iv):
    """Total length of the union of [s, e) intervals."""
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("kernels")
    ap.add_argument("copies")
    ap.add_argument("--first", type=int, default=6)
    a = ap.parse_args()
    ks = spans(list(csv.DictReader(open(a.kernels))), "Kernel_Name")
    cs = spans(list(csv.DictReader(open(a.copies))), "Direction")
    h2d = [c for c in cs if "HOST_TO_DEVICE" in c[2].upper() or "H2D" in c[2].upper()]
    maps = [k for k in ks if "map_fast" in k[2]]
    ins = [k for k in ks if "insert" in k[2]]
    if not maps:
        print("no map kernels in the trace")
        return 1
    t0 = min(x[0] for x in ks + cs)
    t1 = max(x[1] for x in ks + cs)
    print(f"job span {(t1 - t0) / 1e6:.2f} ms: {len(maps)} map windows, {len(h2d)} H2D copies "
          f"({sum(int(c[3].get('Size', c[3].get('Bytes', 0)) or 0) for c in h2d) / 1e9:.2f} GB)")
    kb = busy([(s, e) for s, e, _n, _r in ks])
    cb = busy([(s, e) for s, e, _n, _r in h2d])
    both = busy([(s, e) for s, e, _n, _r in ks + h2d])
    print(f"kernels busy {kb / 1e6:.2f} ms, H2D busy {cb / 1e6:.2f} ms, either {both / 1e6:.2f} ms, "
          f"neither {(t1 - t0 - both) / 1e6:.2f} ms")
    durs = sorted((e - s) / 1e3 for s, e, _n, _r in maps)
    idur = sorted((e - s) / 1e3 for s, e, _n, _r in ins)
    print(f"map kernel us: median {durs[len(durs) // 2]:.1f}, min {durs[0]:.1f}, max {durs[-1]:.1f}; "
          f"insert us: median {idur[len(idur) // 2] if idur else 0:.1f}, max {idur[-1] if idur else 0:.1f}")
    if h2d:
        rates = []
        for s, e, _n, r in h2d:
            b = int(r.get("Size", r.get("Bytes", 0)) or 0)
            if e > s and b:
                rates.append(b / (e - s))
        rates.sort()
        if rates:
            print(f"H2D GB/s per copy: median {rates[len(rates) // 2]:.1f}, min {rates[0]:.1f}")
    cd = [(e - s) / 1e3 for s, e, _n, _r in h2d]
    if cd:
        sc = sorted(cd)
        print(f"H2D copy us: median {sc[len(sc) // 2]:.1f}, min {sc[0]:.1f}, max {sc[-1]:.1f}; "
              f"first copies {', '.join('%.0f' % x for x in cd[:6])}; last {', '.join('%.0f' % x for x in cd[-4:])}")
        print(f"first H2D at {(h2d[0][0] - t0) / 1e6:.2f} ms, first map at {(maps[0][0] - t0) / 1e6:.2f} ms, "
              f"last map ends {(maps[-1][1] - t0) / 1e6:.2f} ms, first activity: "
              f"{min(ks + cs)[2][:40]}")
        gaps = [(h2d[i + 1][0] - h2d[i][1]) / 1e3 for i in range(len(h2d) - 1)]
        if gaps:
            sg = sorted(gaps)
            print(f"gap between H2D copies us: median {sg[len(sg) // 2]:.1f}, max {sg[-1]:.1f}")
    print(f"first {a.first} windows (ms from job start):")
    for i, (s, e, _n, _r) in enumerate(maps[:a.first]):
        nxt = [x for x in ins if x[0] >= e][:1]
        ie = f", insert {(nxt[0][1] - nxt[0][0]) / 1e3:.1f} us" if nxt else ""
        print(f"  window {i}: map at {(s - t0) / 1e6:7.2f} for {(e - s) / 1e3:7.1f} us{ie}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
