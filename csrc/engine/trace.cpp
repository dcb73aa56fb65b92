// trace.cpp — lazy roctx binding (see trace.hpp).
#include "pga/trace.hpp"

#include <dlfcn.h>

#include <atomic>
#include <cstdlib>
#include <mutex>

namespace pga {

namespace {
using push_fn = int (*)(const char*);
using pop_fn = int (*)();
using mark_fn = void (*)(const char*);

struct Roctx {
  push_fn push = nullptr;
  pop_fn pop = nullptr;
  mark_fn mark = nullptr;
  int level = 0;
};

Roctx& roctx() {
  static Roctx r;
  static std::once_flag once;
  std::call_once(once, [] {
    const char* e = std::getenv("PGA_TRACE");
    r.level = e ? std::atoi(e) : 0;
    if (r.level <= 0) return;
    void* h = dlopen("librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
      r.level = 0;
      return;
    }
    r.push = (push_fn)dlsym(h, "roctxRangePushA");
    r.pop = (pop_fn)dlsym(h, "roctxRangePop");
    r.mark = (mark_fn)dlsym(h, "roctxMarkA");
    if (!r.push || !r.pop) r.level = 0;
  });
  return r;
}
}  // namespace

int trace_level() { return roctx().level; }

void trace_push(const char* name) {
  Roctx& r = roctx();
  if (r.level > 0) r.push(name);
}

void trace_pop() {
  Roctx& r = roctx();
  if (r.level > 0) r.pop();
}

void trace_mark(const char* name) {
  Roctx& r = roctx();
  if (r.level > 0 && r.mark) r.mark(name);
}

}  // namespace pga
