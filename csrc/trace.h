// roctx ranges for rocprofv3 (--marker-trace) timelines of the host-side pipeline.
//
// Reference parity: psana-ray has no tracing at all (the closest thing is a per-event
// INFO log, psana_ray/producer.py:103).  The library is dlopen'ed on first use, so the extension
// has no link-time dependency on the profiler SDK; without it (or with PSANA_RAY_ROCTX=0) every
// call is a predictable branch.
#pragma once

namespace pr {
namespace trace {

bool enabled();
void push(const char* name);
void pop();
void mark(const char* name);

struct Range {
  explicit Range(const char* name) : on_(enabled()) {
    if (on_) push(name);
  }
  ~Range() {
    if (on_) pop();
  }
  Range(const Range&) = delete;
  Range& operator=(const Range&) = delete;

 private:
  bool on_;
};

}  // namespace trace
}  // namespace pr
