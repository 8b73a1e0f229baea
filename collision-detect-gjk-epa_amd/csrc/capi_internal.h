// capi_internal.h — helpers shared by the C-ABI translation units (not part of the C-ABI).
#pragma once
#include <string>

namespace gjkepa_internal {
// record `msg` as the calling thread's gjkepa_last_error() and return `code`
int set_error(int code, const std::string& msg);
}  // namespace gjkepa_internal
