// Native threads that must not outlive the HIP runtime.
//
// The queue fabric's progress thread and the producer engine's thread call HIP.  An object that is
// still alive when the process exits (leaked by a caller, held by a reference cycle) would keep its
// thread calling HIP while the runtime's static destructors tear it down -- a crash AFTER the
// program's work is done (seen as a segfault at interpreter exit).  Every such object registers a
// halt callback here; the extension's loader registers halt_native_threads() with Python's atexit,
// which runs before module teardown and before any C++ static destructor.
#pragma once

#include <functional>

namespace pr {

void register_native_thread_owner(const void* owner, std::function<void()> halt);
void unregister_native_thread_owner(const void* owner);   // blocks while a halt is running
void halt_native_threads();                               // idempotent

}  // namespace pr
