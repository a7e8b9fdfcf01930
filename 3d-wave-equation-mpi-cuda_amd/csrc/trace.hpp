// roctx ranges for rocprofv3 --marker-trace (the reference has only hand-rolled
// timers). Host-side scopes around the solver phases; a no-op unless a tool is attached.
#pragma once

#include <rocprofiler-sdk-roctx/roctx.h>

namespace wave3d {

struct TraceRange {
    explicit TraceRange(const char* name) { roctxRangePushA(name); }
    ~TraceRange() { roctxRangePop(); }
    TraceRange(const TraceRange&) = delete;
    TraceRange& operator=(const TraceRange&) = delete;
};

inline void trace_mark(const char* name) { roctxMarkA(name); }

}  // namespace wave3d
