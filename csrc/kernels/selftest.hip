// Device-side self-test of the string library (run each case on
// host AND device).  One thread per string: strlen, strcmp with the next string, a
// bounded copy into a 30-byte key field, strtok_r over the string (token count and the
// byte offsets of the first 8 tokens) and itoa of an integer -- the Python test compares
// every field with the host build of the same header and with Python references.
#include "locust/dstring.hpp"
#include "locust/hip_check.hpp"
#include "locust/kernels.hpp"

namespace locust {
namespace {

__global__ void string_selftest_kernel(const char* __restrict__ blob, const u32* __restrict__ off,
                                       u32 n, const char* __restrict__ delims,
                                       const int* __restrict__ ints, StringTestOut* __restrict__ out) {
  const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const char* s = blob + off[i];
  StringTestOut o{};
  o.len = d_strlen(s);
  o.cmp_next = i + 1 < n ? d_strcmp(s, blob + off[i + 1]) : 0;
  o.copy_len = d_strcpy_bounded(o.copy, s, (int)sizeof(o.copy));
  char buf[kStringTestMax];
  int k = 0;
  for (; k + 1 < kStringTestMax && s[k]; ++k) buf[k] = s[k];
  buf[k] = 0;
  char* save = nullptr;
  o.ntok = 0;
  for (char* t = d_strtok_r(buf, delims, &save); t; t = d_strtok_r(nullptr, delims, &save)) {
    if (o.ntok < 8) o.tok_off[o.ntok] = (int)(t - buf);
    ++o.ntok;
  }
  d_itoa(ints[i], o.itoa_buf, 10);
  out[i] = o;
}

}  // namespace

void launch_string_selftest(const char* blob, const u32* off, u32 n, const char* delims,
                            const int* ints, StringTestOut* out, hipStream_t s) {
  if (!n) return;
  string_selftest_kernel<<<dim3((n + 63) / 64), dim3(64), 0, s>>>(blob, off, n, delims, ints, out);
  LOCUST_HIP_LAUNCH_CHECK();
}

}  // namespace locust
