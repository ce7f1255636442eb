"""Loopback ranks on one GPU (all ranks' kernels on this device): repeated whole-Hamlet
jobs at WORLD ranks, for kernel profiles of the distributed kernels at that run count
(e.g. the root merge of 8 slots).   python tools/loopback_prof.py [world] [jobs]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import locust_amd as lc  # noqa: E402

world = int(sys.argv[1]) if len(sys.argv) > 1 else 8
jobs = int(sys.argv[2]) if len(sys.argv) > 2 else 20
text = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                         "data", "hamlet.txt"), "rb").read()
job = lc.make_config("gpu", combine=True)
cfgs = [lc.make_dist_config(world, job, strategy="gather") for _ in range(jobs)]
out = lc._C.run_multi_schedule(text, cfgs)
print("jobs", len(out), "strategy", out[-1][1]["strategy"], "unique", out[-1][0].num_unique)
