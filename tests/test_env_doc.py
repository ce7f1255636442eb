"""docs/ENVIRONMENT.md names every LOCUST_* variable the native code reads."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_every_native_switch_is_documented():
    used = set()
    for d, _, files in os.walk(os.path.join(ROOT, "csrc")):
        for f in files:
            if f.endswith((".cpp", ".hpp", ".hip")):
                used |= set(re.findall(r'getenv\("(LOCUST_[A-Z0-9_]+)"',
                                       open(os.path.join(d, f), errors="replace").read()))
    doc = open(os.path.join(ROOT, "docs", "ENVIRONMENT.md")).read()
    assert used and not sorted(v for v in used if f"`{v}`" not in doc)
