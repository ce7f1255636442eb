// One persistent host thread that runs one task at a time off the caller's path.
//
// The engine hands it the partition map's retune after a job (a pass over the job's output
// that took ~0.15 ms of a small first job's wall time when done inline, and ~2 ms for a
// 200K-key output) so the job returns as soon as its results are in host memory.  The
// thread is made once (engine construction), not per task: a std::async per job cost a
// thread creation inside the job.
#pragma once

#include <atomic>
#include <condition_variable>
#include <exception>
#include <functional>
#include <mutex>
#include <stdexcept>
#include <thread>
#include <utility>

namespace locust {

class TaskWorker {
 public:
  TaskWorker() = default;
  ~TaskWorker() { stop(); }
  TaskWorker(const TaskWorker&) = delete;
  TaskWorker& operator=(const TaskWorker&) = delete;

  // Makes the thread (idempotent).
  void start() {
    std::lock_guard<std::mutex> lk(mu_);
    if (!th_.joinable() && !stop_) th_ = std::thread([this] { loop(); });
  }
  // No task queued or running (never blocks).
  bool idle() const { return !busy_.load(std::memory_order_acquire); }
  // Runs f on the worker thread.  The worker must be idle (one task at a time): a submit
  // over a queued or running task is refused loudly instead of replacing it.
  void submit(std::function<void()> f) {
    start();
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (busy_.load(std::memory_order_acquire) || task_)
        throw std::logic_error("TaskWorker::submit: the worker is still busy with a task");
      task_ = std::move(f);
      busy_.store(true, std::memory_order_release);
    }
    cv_.notify_one();
  }
  void wait_idle() {
    std::unique_lock<std::mutex> lk(mu_);
    idle_cv_.wait(lk, [&] { return !busy_.load(std::memory_order_acquire); });
  }
  // The exception the last task threw (cleared), rethrown on the caller's thread -- a task
  // never takes the process down with std::terminate on the worker thread.
  void rethrow_error() {
    std::exception_ptr e;
    {
      std::lock_guard<std::mutex> lk(mu_);
      std::swap(e, error_);
    }
    if (e) std::rethrow_exception(e);
  }
  // Finishes the running task, then ends the thread.
  void stop() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_one();
    if (th_.joinable()) th_.join();
  }

 private:
  void loop() {
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      cv_.wait(lk, [&] { return stop_ || task_; });
      if (task_) {
        std::function<void()> f = std::move(task_);
        task_ = nullptr;
        lk.unlock();
        std::exception_ptr err;
        try {
          f();
        } catch (...) {
          err = std::current_exception();
        }
        f = nullptr;  // captured state is released before the worker reports idle
        lk.lock();
        if (err) error_ = err;
        busy_.store(false, std::memory_order_release);
        idle_cv_.notify_all();
        continue;
      }
      if (stop_) return;
    }
  }
  std::thread th_;
  std::mutex mu_;
  std::condition_variable cv_, idle_cv_;
  std::function<void()> task_;
  std::exception_ptr error_;
  std::atomic<bool> busy_{false};
  bool stop_ = false;
};

}  // namespace locust
