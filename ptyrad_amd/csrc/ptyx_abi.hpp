// ptyx_abi.hpp — error-reporting helpers shared by the translation units of libptyx.so
// (the thread-local message behind ptyx_last_error lives in ptyx_kernels.hip).
#pragma once
#include <string>

namespace ptyx {
namespace abi {
void clear_error();
int fail(int code, const std::string& msg);
int launch_status(const char* what);   // hipGetLastError → PTYX_EHIP with a message
}  // namespace abi
}  // namespace ptyx
