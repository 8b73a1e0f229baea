// capi_internal.h — helpers shared by the C-ABI translation units (not part of the C-ABI).
#pragma once
#include <rocprofiler-sdk-roctx/roctx.h>

#include <string>

namespace gjkepa_internal {
// roctx range over one API call (rocprofv3 --marker-trace shows it beside the kernels it enqueued):
// the chain, the record all-gather, the host-buffer round trips (SURVEY.md §5 tracing)
struct Range {
    explicit Range(const char* what) { roctxRangePushA(what); }
    ~Range() { roctxRangePop(); }
    Range(const Range&) = delete;
    Range& operator=(const Range&) = delete;
};
// record `msg` as the calling thread's gjkepa_last_error() and return `code`
int set_error(int code, const std::string& msg);
}  // namespace gjkepa_internal
