"""Back-to-back lean jobs on one engine with the inputs changing every job: the host reads
each job's results the moment the ordered kernel's last workgroup stores the completion
word (a relaxed system-scope store, every workgroup having released its records before
its done count -- dict.hip self-clean tail), so a record or counter still in flight would
show up here as a job whose output is another job's or a mix.  Every output is compared
byte for byte with its text's oracle-checked output."""
import random

import pytest

import locust_amd as lc
from locust_amd.utils import oracle

pytestmark = pytest.mark.gpu


def test_lean_jobs_back_to_back_change_inputs(hamlet):
    rng = random.Random(11)
    words = hamlet.split()
    texts = [
        hamlet,
        oracle.window(hamlet, 0, 700),
        oracle.window(hamlet, 1200, 1500),
        oracle.window(hamlet, 3000, 4463),
        b"\n".join(b" ".join(rng.choice(words) for _ in range(12)) for _ in range(3000)) + b"\n",
        b"\n".join(b" ".join(rng.choice(words)[::-1] for _ in range(9)) for _ in range(800)),
    ]
    eng = lc._C.GpuEngine(lc.make_config("gpu"), max(len(t) for t in texts) + 1, 1 << 16)
    want = []
    for t in texts:  # each text's output, checked against the oracle once
        r = eng.run(t)
        assert r.entries() == oracle.wordcount(t)[0]
        want.append(r.format())
    assert r.times()["graph"] is False  # the lean job: the kernel signals the host itself
    order = [rng.randrange(len(texts)) for _ in range(4000)]
    for i, k in enumerate(order):
        got = eng.run(texts[k]).format()
        assert got == want[k], f"job {i}: text {k} came back as another job's output"
