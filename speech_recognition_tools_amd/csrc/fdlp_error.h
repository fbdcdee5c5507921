// fdlp_error.h -- thread-local last-error string behind fdlp_last_error().
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <string>

typedef struct fdlp_ark_writer fdlp_ark_writer;

namespace fdlp {
std::string& last_error_slot();
inline int fail(int code, const std::string& msg) {
  last_error_slot() = msg;
  return code;
}
// Appends n utterances to an open ark/scp writer with one writev per 512 utterances (header and rows of
// utterance i: rows[i] .. rows[i+1] of the row-major float32 matrix at base, cols wide).  Same bytes as n
// fdlp_ark_write calls (fdlp_host.cpp).
struct ArkItem {
  const char* id;
  const float* data;
  int32_t rows;
};
int ark_write_batch(fdlp_ark_writer* w, const ArkItem* items, size_t n, int32_t cols);
// n int16 ark codes -> the float32 ark values (fdlp_q_widen on the calling thread, table lookups)
void q_widen_span(const int16_t* q, int64_t n, int32_t decimals, float* out);
}  // namespace fdlp
