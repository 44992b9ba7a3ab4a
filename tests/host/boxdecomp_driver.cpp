// Host driver for sanitizer builds of csrc/boxdecomp.cpp (AddressSanitizer +
// UndefinedBehaviorSanitizer, ThreadSanitizer): random point sets through
// bo_nd_partition_host on 8 worker threads, the result compared with a
// one-thread run (bit-equal) and checked for cell sanity (lo <= hi, finite
// except +inf upper bounds of unbounded cells).  Test code only.
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdint>
#include <random>
#include <vector>

#include "../../include/botorch_amd.h"

void bo_set_error(const char* fmt, ...) {  // the library's error slot (gpu-side file) for this driver
  va_list ap;
  va_start(ap, fmt);
  std::vfprintf(stderr, fmt, ap);
  va_end(ap);
  std::fputc('\n', stderr);
}

static int run(int64_t S, int64_t n, int m, unsigned seed) {
  std::mt19937_64 g(seed);
  std::normal_distribution<double> nd(0.0, 1.0);
  std::vector<double> Y((size_t)(S * n * m)), ref((size_t)m, -3.0);
  for (auto& y : Y) y = nd(g);
  for (int64_t s = 0; n >= 2 && s < S; s += 7)  // duplicate points
    for (int j = 0; j < m; ++j) Y[(size_t)(s * n * m + j)] = Y[(size_t)(s * n * m + m + j)];
  int64_t K8 = 0, K1 = 0;
  if (bo_nd_partition_host(Y.data(), S, n, m, ref.data(), 0, &K8, nullptr, nullptr, 8)) return 1;
  std::vector<double> lo8((size_t)(S * K8 * m)), hi8(lo8.size()), lo1(lo8.size()), hi1(lo8.size());
  if (bo_nd_partition_host(Y.data(), S, n, m, ref.data(), K8, &K8, lo8.data(), hi8.data(), 8)) return 2;
  if (bo_nd_partition_host(Y.data(), S, n, m, ref.data(), K8, &K1, lo1.data(), hi1.data(), 1)) return 3;
  if (K1 != K8) return 4;
  for (size_t e = 0; e < lo8.size(); ++e) {
    if (!(lo8[e] == lo1[e] && (hi8[e] == hi1[e] || (std::isinf(hi8[e]) && std::isinf(hi1[e])))))
      return 5;
    if (!(lo8[e] <= hi8[e]) || std::isnan(lo8[e])) return 6;
  }
  std::printf("S=%lld n=%lld m=%d K=%lld ok\n", (long long)S, (long long)n, m, (long long)K8);
  return 0;
}

int main() {
  int rc = 0;
  rc |= run(96, 40, 3, 1);
  rc |= run(64, 60, 2, 2);
  rc |= run(32, 24, 4, 3);
  rc |= run(1, 0, 3, 4);  // empty set
  return rc;
}
