// fdlp_error.h -- thread-local last-error string behind fdlp_last_error().
#pragma once
#include <string>

namespace fdlp {
std::string& last_error_slot();
inline int fail(int code, const std::string& msg) {
  last_error_slot() = msg;
  return code;
}
}  // namespace fdlp
