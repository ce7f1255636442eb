// roctx ranges around the engine's stages (the reference has host timers
// only).  Under `rocprofv3 --marker-trace` the ranges ("locust:map", "locust:process",
// "locust:shuffle", ...) line up with the kernel trace; without a tool attached a push /
// pop is a cheap call into the roctx stub.  LOCUST_ROCTX=0 turns them off entirely.
#pragma once

namespace locust {

bool roctx_enabled();
void roctx_push(const char* name);
void roctx_pop();

class TraceRange {
 public:
  explicit TraceRange(const char* name) : on_(roctx_enabled()) {
    if (on_) roctx_push(name);
  }
  ~TraceRange() {
    if (on_) roctx_pop();
  }
  TraceRange(const TraceRange&) = delete;
  TraceRange& operator=(const TraceRange&) = delete;

 private:
  bool on_;
};

}  // namespace locust
