"""One process of tests/test_switches.py: runs a fixed set of WordCount jobs under the
LOCUST_* environment it was started with and checks every result against the oracle.

    python tests/switch_worker.py single|stream|dist|merge|cli

Exit status 0 = every job matched; the failure is printed otherwise.  A separate process
per setting because many switches are read once per process (or per engine)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import locust_amd as lc  # noqa: E402
from locust_amd.utils import oracle  # noqa: E402


def check(res, text, what):
    ent, ntok, _ = oracle.wordcount(text)
    assert res.num_tokens == ntok, (what, res.num_tokens, ntok)
    assert res.entries() == ent, f"{what}: entries differ from the oracle"


def main(kind: str) -> None:
    hamlet = open(os.path.join(ROOT, "data", "hamlet.txt"), "rb").read()
    # ~2.6 MB of synthetic text: a one-pass "large" input (piecewise upload, partials build)
    synth = lc.gen_text(lines=60_000, seed=7)
    if kind == "single":
        # 5x Hamlet (~0.94 MiB): past 2^18 worst-case tokens, within LOCUST_SMALL_PASS_KB --
        # the small-pass route (or, with it off, the large build) of the one-pass engine
        for text, what in ((hamlet, "hamlet"), (oracle.window(hamlet, 0, 700), "hamlet700"),
                           (hamlet * 5, "hamlet5x"), (synth, "synth")):
            eng = lc.Engine(lc.make_config("gpu"), len(text), text.count(b"\n") + 1)
            for j in range(3):  # first job, retuned job, steady job
                check(eng.run(text), text, f"{what} job {j}")
    elif kind == "stream":
        eng = lc.Engine(lc.make_config("gpu", chunk_bytes=1 << 20), len(synth),
                        synth.count(b"\n") + 1)
        for j in range(2):
            check(eng.run(synth), synth, f"streamed job {j}")
    elif kind == "dist":
        for world in (1, 2, 3):
            for strategy in ("shuffle", "auto"):
                res = lc.run_multi(synth, world, strategy=strategy, comm="loopback")
                check(res, synth, f"loopback {world} {strategy}")
    elif kind == "merge":
        # stage 2 on the device over 70 spills (rounds of 64 runs) of the synthetic text's
        # line windows; a low LOCUST_MERGE_MAX_RECORDS also splits merges by key range
        import tempfile

        lines = synth.split(b"\n")
        with tempfile.TemporaryDirectory() as d:
            files = []
            for k in range(70):
                part = b"\n".join(lines[k::70]) + b"\n"
                recs = [(key, c) for key, _v, c in oracle.wordcount(part)[0]]
                files.append(os.path.join(d, f"out.{k}.kv"))
                lc._C.write_spill(files[-1], recs, "binary")
            for reducers in (1, 3):
                got = []
                for r in range(reducers):
                    res, _st = lc._C.reduce_spills(lc.make_config("gpu"), files, r, reducers)
                    got += res.entries()
                ent = oracle.wordcount(synth)[0]
                assert got == ent, f"device merge of 70 spills, {reducers} reducers"
    elif kind == "cli":
        # the one-shot CLI twice on one file: the second run starts from the partition map
        # the first one tuned (unless LOCUST_PART_CACHE=0); the output never changes
        import json
        import subprocess
        import tempfile

        with tempfile.TemporaryDirectory() as d:
            env = dict(os.environ)
            if env.get("LOCUST_CACHE_DIR", None) == "":
                env["LOCUST_CACHE_DIR"] = os.path.join(d, "cache")
            f = os.path.join(d, "h.txt")
            with open(f, "wb") as fh:
                fh.write(hamlet)
            maps = []
            for _ in range(2):
                j = os.path.join(d, "r.json")
                p = subprocess.run([lc.cli_path(), f, "--json", j], capture_output=True,
                                   env=env, timeout=120)
                assert p.returncode == 0, p.stderr.decode()[-2000:]
                got = b"".join(l + b"\n" for l in p.stdout.split(b"\n") if l.startswith(b"print key:"))
                assert got == oracle.format_gpu(oracle.wordcount(hamlet)[0]), "CLI output"
                maps.append(json.load(open(j))["part_map"])
            off = os.environ.get("LOCUST_PART_CACHE") == "0"
            assert maps == (["default", "default"] if off else ["default", "cache"]), maps
    else:
        raise SystemExit(f"unknown kind {kind}")
    print("switch worker ok:", kind, {k: v for k, v in os.environ.items()
                                      if k.startswith("LOCUST_")})


if __name__ == "__main__":
    main(sys.argv[1])
