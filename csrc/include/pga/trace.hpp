// trace.hpp — roctx ranges around engine stages (the
// reference has no tracing at all).
//
// Off by default.  PGA_TRACE=1 marks every engine call (run, evaluate, top-k,
// migration gather/scatter, checkpoint); PGA_TRACE=2 adds one range per
// generation.  Ranges go to librocprofiler-sdk-roctx (loaded lazily with
// dlopen, so the engine has no link-time dependency on the profiler), where
// `rocprofv3 --marker-trace` picks them up.
#pragma once

namespace pga {

int trace_level();                 // PGA_TRACE, read once
void trace_push(const char* name);  // no-op unless tracing is on
void trace_pop();
void trace_mark(const char* name);

struct TraceRange {
  bool on;
  explicit TraceRange(const char* name, int level = 1) : on(trace_level() >= level) {
    if (on) trace_push(name);
  }
  ~TraceRange() {
    if (on) trace_pop();
  }
  TraceRange(const TraceRange&) = delete;
  TraceRange& operator=(const TraceRange&) = delete;
};

}  // namespace pga
