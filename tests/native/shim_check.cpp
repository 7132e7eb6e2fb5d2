// Pins lego-loam_amd/csrc/lego_numerics.h (the libm restatement shared by the
// oracle and the gfx950 kernels) against THIS host's glibc, bit for bit.
//   shim_check <stride> <pairs>
// sinf/cosf (and the fused lego_sincosf)/atanf/asinf over every `stride`-th float bit pattern (stride 1 =
// exhaustive), atan2f over `pairs` random bit-pattern pairs plus `pairs`
// uniform pairs in [-100,100]^2.  Prints mismatch counts; exit 1 on any.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>
#include <atomic>
#include "../../lego-loam_amd/csrc/lego_numerics.h"
using namespace lego;
static uint64_t sm(uint64_t& s) { uint64_t z = (s += 0x9e3779b97f4a7c15ULL); z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL; z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL; return z ^ (z >> 31); }
static bool same(float a, float b) { return f2u(a) == f2u(b) || (std::isnan(a) && std::isnan(b)); }
int main(int argc, char** argv) {
  const uint64_t stride = argc > 1 ? strtoull(argv[1], 0, 10) : 97;
  const long pairs = argc > 2 ? atol(argv[2]) : 2000000;
  std::atomic<long> bs{0}, bc{0}, ba{0}, bt{0}, n{0};
  std::vector<std::thread> th;
  const int T = 8;
  for (int t = 0; t < T; t++) th.emplace_back([&, t] {
    long s_ = 0, c_ = 0, a_ = 0, t_ = 0, n_ = 0;
    for (uint64_t u = (uint64_t)t * stride; u < (1ULL << 32); u += (uint64_t)T * stride) {
      float x = u2f((uint32_t)u);
      if (std::isnan(x)) continue;
      ++n_;
      if (!same(sinf(x), lego_sinf(x))) s_++;
      if (!same(cosf(x), lego_cosf(x))) c_++;
      float fs, fc;  // the fused form must equal both (and so glibc)
      lego_sincosf(x, &fs, &fc);
      if (!same(fs, lego_sinf(x))) s_++;
      if (!same(fc, lego_cosf(x))) c_++;
      if (!same(asinf(x), lego_asinf(x))) a_++;
      if (!same(atanf(x), lego_atanf(x))) t_++;
    }
    bs += s_; bc += c_; ba += a_; bt += t_; n += n_;
  });
  for (auto& x : th) x.join();
  uint64_t s = 1;
  long m1 = 0, m2 = 0;
  for (long i = 0; i < pairs; i++) {
    float y = u2f((uint32_t)sm(s)), x = u2f((uint32_t)sm(s));
    if (std::isnan(x) || std::isnan(y)) continue;
    if (!same(atan2f(y, x), lego_atan2f(y, x))) m1++;
  }
  for (long i = 0; i < pairs; i++) {
    float y = (float)((double)(sm(s) >> 11) / 9007199254740992.0 * 200 - 100);
    float x = (float)((double)(sm(s) >> 11) / 9007199254740992.0 * 200 - 100);
    if (!same(atan2f(y, x), lego_atan2f(y, x))) m2++;
  }
  printf("floats %ld sinf %ld cosf %ld asinf %ld atanf %ld atan2f_bits %ld atan2f_uniform %ld\n",
         (long)n, (long)bs, (long)bc, (long)ba, (long)bt, m1, m2);
  return (bs + bc + ba + bt + m1 + m2) ? 1 : 0;
}
