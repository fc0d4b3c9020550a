#include "trace.h"

#include <dlfcn.h>
#include <stdlib.h>

#include <mutex>

namespace pr {
namespace trace {
namespace {

using push_fn = int (*)(const char*);
using pop_fn = int (*)();
using mark_fn = void (*)(const char*);

struct Api {
  push_fn push = nullptr;
  pop_fn pop = nullptr;
  mark_fn mark = nullptr;
  bool on = false;
};

const Api& api() {
  static Api a;
  static std::once_flag once;
  std::call_once(once, [] {
    const char* e = getenv("PSANA_RAY_ROCTX");
    if (e != nullptr && e[0] == '0') return;
    const char* names[] = {"librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so",
                           "/opt/rocm/lib/librocprofiler-sdk-roctx.so.1"};
    void* h = nullptr;
    for (const char* n : names)
      if ((h = dlopen(n, RTLD_NOW | RTLD_LOCAL)) != nullptr) break;
    if (h == nullptr) return;
    a.push = reinterpret_cast<push_fn>(dlsym(h, "roctxRangePushA"));
    a.pop = reinterpret_cast<pop_fn>(dlsym(h, "roctxRangePop"));
    a.mark = reinterpret_cast<mark_fn>(dlsym(h, "roctxMarkA"));
    a.on = a.push != nullptr && a.pop != nullptr && a.mark != nullptr;
  });
  return a;
}

}  // namespace

bool enabled() { return api().on; }
void push(const char* name) {
  if (api().on) api().push(name);
}
void pop() {
  if (api().on) api().pop();
}
void mark(const char* name) {
  if (api().on) api().mark(name);
}

}  // namespace trace
}  // namespace pr
