// Device-side self-test of the string library (run each case on
// host AND device).  One thread per string: strlen, strcmp with the next string, a
// bounded copy into a 30-byte key field, strtok_r over the string (token count and the
// byte offsets of the first 8 tokens) and itoa of an integer -- the Python test compares
// every field with the host build of the same header and with Python references.
#include <string>
#include <vector>

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

namespace locust {

std::vector<StringTestOut> run_string_selftest(const std::vector<std::string>& strings,
                                               const std::vector<int>& ints,
                                               const std::string& delims, int device) {
  LOCUST_CHECK_ARG(ints.size() == strings.size(), "one integer per string");
  LOCUST_HIP_CHECK(hipSetDevice(device));
  std::string blob;
  std::vector<u32> off;
  for (const auto& x : strings) {
    LOCUST_CHECK_ARG(x.size() < (size_t)kStringTestMax, "self-test strings are < 128 bytes");
    off.push_back((u32)blob.size());
    blob += x;
    blob.push_back('\0');
  }
  const u32 n = (u32)strings.size();
  std::vector<StringTestOut> out(n);
  if (!n) return out;
  char *d_blob = nullptr, *d_delims = nullptr;
  u32* d_off = nullptr;
  int* d_ints = nullptr;
  StringTestOut* d_out = nullptr;
  LOCUST_HIP_CHECK(hipMalloc(&d_blob, blob.size()));
  LOCUST_HIP_CHECK(hipMalloc(&d_delims, delims.size() + 1));
  LOCUST_HIP_CHECK(hipMalloc(&d_off, n * sizeof(u32)));
  LOCUST_HIP_CHECK(hipMalloc(&d_ints, n * sizeof(int)));
  LOCUST_HIP_CHECK(hipMalloc(&d_out, n * sizeof(StringTestOut)));
  LOCUST_HIP_CHECK(hipMemcpy(d_blob, blob.data(), blob.size(), hipMemcpyHostToDevice));
  LOCUST_HIP_CHECK(hipMemcpy(d_delims, delims.c_str(), delims.size() + 1, hipMemcpyHostToDevice));
  LOCUST_HIP_CHECK(hipMemcpy(d_off, off.data(), n * sizeof(u32), hipMemcpyHostToDevice));
  LOCUST_HIP_CHECK(hipMemcpy(d_ints, ints.data(), n * sizeof(int), hipMemcpyHostToDevice));
  launch_string_selftest(d_blob, d_off, n, d_delims, d_ints, d_out, nullptr);
  LOCUST_HIP_CHECK(hipMemcpy(out.data(), d_out, n * sizeof(StringTestOut), hipMemcpyDeviceToHost));
  for (void* p : {(void*)d_blob, (void*)d_delims, (void*)d_off, (void*)d_ints, (void*)d_out})
    (void)hipFree(p);
  return out;
}

}  // namespace locust
