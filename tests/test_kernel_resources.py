"""Register / LDS / scratch budgets of the product kernels, from the compiler's own
resource report (hipcc -Rpass-analysis=kernel-resource-usage; gfx950 cross-compiles on the
CPU box).  Round 4 found three silent regressions this way: a by-value struct copy in a
device function promoted to 32 KB of LDS in map_fast_kernel<1, 1024> (its 1 KiB tiles took
20 us instead of 13), a struct copy through private memory in every ordered kernel, and a
dynamically indexed record array in merge_emit_compact_kernel -- scratch (private memory)
in a hot kernel costs its setup at every launch and memory traffic per access."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"
FILES = ["tokenize", "dict", "merge", "exchange", "psort", "radix_sort", "reduce", "map",
         "partplan", "shuffle", "signal"]
# diagnostics-only kernels allowed to use scratch
SCRATCH_OK = {"string_selftest_kernel"}
# LDS ceilings (bytes) of kernels whose LDS is part of their design
LDS_MAX = {"map_fast_kernelILi1ELi1024": 8192, "map_fast_kernelILi16ELi256": 20480,
           "map_ordered_kernel": 160 * 1024}


def resources(src):
    p = subprocess.run([HIPCC, "-std=c++17", "-fPIC", "-I" + os.path.join(ROOT, "csrc/include"),
                        "-O3", "--offload-arch=gfx950", "-munsafe-fp-atomics", "-c", src, "-o",
                        os.devnull, "-Rpass-analysis=kernel-resource-usage"],
                       capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    out, name = {}, None
    for ln in p.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", ln)
        if m:
            name = m.group(1)
            out[name] = {}
            continue
        m = re.search(r"remark:\s+([\w ]+?)(?: \[[^\]]*\])?: (\d+)", ln)
        if m and name:
            out[name][m.group(1).strip()] = int(m.group(2))
    return out


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="no hipcc")
@pytest.mark.parametrize("stem", FILES)
def test_no_scratch_and_lds_budgets(stem):
    res = resources(os.path.join(ROOT, "csrc", "kernels", stem + ".hip"))
    assert res, "no kernels reported"
    for name, r in res.items():
        if not any(ok in name for ok in SCRATCH_OK):
            assert r.get("ScratchSize", 0) == 0, (name, r)
            assert r.get("VGPRs Spill", 0) == 0, (name, r)
        for key, cap in LDS_MAX.items():
            if key in name:
                assert r["LDS Size"] <= cap, (name, r["LDS Size"], cap)
