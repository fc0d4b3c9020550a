#include "lifecycle.h"

#include <map>
#include <mutex>

namespace pr {

namespace {
// leaked on purpose: used from atexit and from destructors that may run during static teardown
std::mutex& reg_mu() {
  static std::mutex* m = new std::mutex();
  return *m;
}
std::map<const void*, std::function<void()>>& reg() {
  static auto* r = new std::map<const void*, std::function<void()>>();
  return *r;
}
}  // namespace

void register_native_thread_owner(const void* owner, std::function<void()> halt) {
  std::lock_guard<std::mutex> lk(reg_mu());
  reg()[owner] = std::move(halt);
}

void unregister_native_thread_owner(const void* owner) {
  std::lock_guard<std::mutex> lk(reg_mu());
  reg().erase(owner);
}

void halt_native_threads() {
  // under the lock: an owner being destroyed meanwhile waits in unregister (its own destructor
  // then finds the thread already joined)
  std::lock_guard<std::mutex> lk(reg_mu());
  for (auto& kv : reg()) kv.second();
}

}  // namespace pr
