"""The starting partition map on text it was not fitted to.

The one-shot CLI's first job partitions the ordered build with a data-independent starting
map (csrc/engine/partmap.cpp): the letters split on their second byte.  Round 5 had added
third-byte cuts at 'th' / 'the' / 'tho' / 'co' words chosen by measuring Hamlet -- the
benchmark fixture itself; this tool's first run (profiles/r6/partmap/heldout.md) timed
them against the plain letters map on inputs none of the maps was fitted to, they did not
help there, and round 6 removed them.  Every map is timed untuned (LOCUST_PART_TUNE=0:
every job starts from the map, as a one-job process does) on:

  * synthetic text of Hamlet's size with other seeds, vocabularies and Zipf exponents
    (the native generator: English-like word lengths, Zipf-distributed ranks);
  * English prose the maps never saw: this repository's top-level documents (SURVEY.md,
    VERDICT.md, README.md), concatenated to Hamlet's size;
  * a different distribution altogether: the repository's Python sources.

Variants (one fresh process each, alternating, tools/ab_procs.py): the default (letters)
map and LOCUST_PART_DEFAULT=byte (first byte only).  Writes a table (markdown) to --out.

    python tools/partmap_heldout.py --out profiles/r6/partmap/heldout.md [--rounds 3]
"""
import argparse
import glob
import os
import re
import statistics
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

HAMLET = 191_734
VARIANTS = {"letters (default)": "LOCUST_PART_TUNE=0",
            "first byte": "LOCUST_PART_TUNE=0,LOCUST_PART_DEFAULT=byte"}


def inputs(d: str) -> dict:
    import locust_amd as lc

    out = {}
    for name, kw in (("gen seed 2", dict(seed=2)),
                     ("gen seed 3, vocab 2,000", dict(seed=3, vocab=2000)),
                     ("gen seed 4, vocab 200,000", dict(seed=4, vocab=200_000)),
                     ("gen seed 5, Zipf s=0.8", dict(seed=5, zipf_s=0.8)),
                     ("gen seed 6, Zipf s=1.3", dict(seed=6, zipf_s=1.3))):
        out[name] = lc._C.gen_text(bytes=HAMLET, **kw)
    prose = b"".join(open(os.path.join(ROOT, f), "rb").read()
                     for f in ("SURVEY.md", "VERDICT.md", "README.md", "BASELINE.md")
                     if os.path.exists(os.path.join(ROOT, f)))
    out["English prose (repo docs)"] = (prose * (HAMLET // max(len(prose), 1) + 1))[:HAMLET]
    code = b"".join(open(p, "rb").read() for p in sorted(glob.glob(os.path.join(ROOT, "locust_amd", "**", "*.py"),
                                                                   recursive=True)))
    code += b"".join(open(p, "rb").read() for p in sorted(glob.glob(os.path.join(ROOT, "tests", "*.py"))))
    out["Python sources"] = (code * (HAMLET // max(len(code), 1) + 1))[:HAMLET]
    out["hamlet (the benchmark fixture)"] = open(os.path.join(ROOT, "data", "hamlet.txt"), "rb").read()
    paths = {}
    for name, text in out.items():
        cut = text.rfind(b"\n")
        text = text[:cut + 1] if cut > 0 else text
        p = os.path.join(d, re.sub(r"[^a-z0-9]+", "_", name.lower()) + ".txt")
        with open(p, "wb") as f:
            f.write(text)
        paths[name] = p
    return paths


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=30)
    a = ap.parse_args()
    rows = []
    with tempfile.TemporaryDirectory() as d:
        for name, path in inputs(d).items():
            p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "ab_procs.py"),
                                *VARIANTS.values(), "--config", "file:" + path, "--rounds",
                                str(a.rounds), "--steps", str(a.steps), "--warmup", str(a.warmup)],
                               capture_output=True, text=True, timeout=900)
            if p.returncode:
                print(p.stderr[-3000:], file=sys.stderr)
                return 1
            med = {}
            for line in p.stdout.splitlines():
                m = re.match(r"(.*): ms/job median ([0-9.]+) .*first job median ([0-9.]+)", line)
                if m:
                    med[m.group(1)] = (float(m.group(2)), float(m.group(3)))
            vals = [med[v] for v in VARIANTS.values()]
            rows.append((name, os.path.getsize(path), vals))
            print(name, vals, flush=True)
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as f:
        f.write("# Starting partition maps on held-out text (untuned jobs, LOCUST_PART_TUNE=0)\n\n")
        f.write(f"Median ms per job over {a.rounds} fresh processes per variant ({a.steps} jobs "
                f"each after {a.warmup} warm-up jobs); first = a fresh engine's first job.  "
                "`tools/partmap_heldout.py`.\n\n")
        f.write("| input | bytes | " + " | ".join(VARIANTS) + " | letters vs first byte |\n")
        f.write("|---|---:|" + "---:|" * len(VARIANTS) + "---:|\n")
        for name, size, vals in rows:
            cells = " | ".join(f"{ms:.4f} (first {fj:.4f})" for ms, fj in vals)
            f.write(f"| {name} | {size} | {cells} | {vals[0][0] / vals[1][0]:.3f} |\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
