"""TaskWorker (csrc/include/locust/worker.hpp), the engine's retune thread:
a submit over a busy worker is refused loudly instead of replacing the task, and a task's
exception is kept and rethrown on the caller's thread (never std::terminate)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PROG = r'''
#include <chrono>
#include <cstdio>
#include <stdexcept>
#include <string>
#include <thread>
#include "locust/worker.hpp"
int main() {
  locust::TaskWorker w;
  w.start();
  std::atomic<bool> go{false};
  w.submit([&] { while (!go) std::this_thread::sleep_for(std::chrono::milliseconds(1)); });
  bool refused = false;
  try { w.submit([] {}); } catch (const std::logic_error&) { refused = true; }
  go = true;
  w.wait_idle();
  w.rethrow_error();  // nothing to rethrow
  w.submit([] { throw std::runtime_error("task failed"); });
  w.wait_idle();
  bool rethrown = false;
  try { w.rethrow_error(); } catch (const std::runtime_error& e) { rethrown = std::string(e.what()) == "task failed"; }
  w.rethrow_error();  // cleared
  w.submit([] {});  // usable after a failure
  w.wait_idle();
  std::printf("%d %d %d\n", refused ? 1 : 0, rethrown ? 1 : 0, w.idle() ? 1 : 0);
  return 0;
}
'''


def test_task_worker_refuses_busy_submit_and_rethrows(tmp_path):
    src = tmp_path / "w.cpp"
    src.write_text(PROG)
    exe = tmp_path / "w"
    subprocess.run(["g++", "-std=c++17", "-O1", "-pthread", "-I", os.path.join(ROOT, "csrc", "include"),
                    str(src), "-o", str(exe)], check=True, capture_output=True, timeout=120)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stderr
    assert out.stdout.split() == ["1", "1", "1"]
