// Pins seg_edge_fast (lego_seg.h: the segmentation angle test decided from
// the quotient away from the threshold) against the reference expression
// atan2f(d2 sin(alpha), d1 - d2 cos(alpha)) > theta, on the sensor presets'
// alphas: random range pairs, pairs placed on the threshold (the angle within
// 1e-4 rad of theta, found by bisection on the second range), and corner
// cases (equal ranges, tiny / huge ranges, d1 - d2 cos(alpha) <= 0).
// Test infrastructure; built and run by tests/test_seg_edge.py.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <random>

#include "lego_seg.h"

using namespace lego;

int main() {
  const float theta = (float)(60.0 / 180.0 * M_PI);
  const float alphas[] = {(float)(0.2 / 180.0 * M_PI), (float)(2.0 / 180.0 * M_PI),     // VLP-16
                          (float)(0.1728 / 180.0 * M_PI), (float)(0.427 / 180.0 * M_PI),  // HDL-64E
                          (float)(0.2 / 180.0 * M_PI), (float)(0.3125 / 180.0 * M_PI)};   // VLS-128
  std::mt19937_64 rng(12345);
  std::uniform_real_distribution<float> U(0.05f, 120.f);
  long n = 0, bad = 0, band = 0;
  auto check = [&](float ra, float rb, float sa, float ca, float th, const TanBand& tb) {
    const bool f = seg_edge_fast(ra, rb, sa, ca, th, tb), r = seg_edge_ref(ra, rb, sa, ca, th);
    ++n;
    if (f != r) {
      if (bad < 10) std::printf("MISMATCH ra=%a rb=%a sa=%a ca=%a\n", ra, rb, sa, ca);
      ++bad;
    }
  };
  for (float th : {theta, (float)(10.0 / 180.0 * M_PI), (float)(80.0 / 180.0 * M_PI), (float)(100.0 / 180.0 * M_PI)}) {
    const TanBand tb = seg_tan_band_host(th);
    for (float al : alphas) {
      const float sa = lego_sinf(al), ca = lego_cosf(al);
      for (int i = 0; i < 400000; ++i) check(U(rng), U(rng), sa, ca, th, tb);
      // on the threshold: for ra, the rb < ra whose angle is theta, by bisection in float
      for (int i = 0; i < 20000; ++i) {
        const float ra = U(rng);
        float lo = 0.f, hi = ra;  // angle increases as rb (= d2) grows towards ra
        for (int it = 0; it < 60; ++it) {
          const float mid = 0.5f * (lo + hi);
          if (seg_edge_ref(ra, mid, sa, ca, th)) hi = mid;
          else lo = mid;
        }
        for (int d = -64; d <= 64; ++d) {
          float x = hi;
          for (int k = 0; k < (d < 0 ? -d : d); ++k) x = std::nextafterf(x, d < 0 ? 0.f : 1e30f);
          check(ra, x, sa, ca, th, tb);
          check(x, ra, sa, ca, th, tb);
          const float y = std::fmin(x, ra) * sa, xx = std::fmax(x, ra) - std::fmin(x, ra) * ca;
          if (xx > 0.f) {
            const double q = (double)(y / xx);
            band += (q >= tb.lo && q <= tb.hi) ? 1 : 0;
          }
        }
      }
      const float edge[] = {0.f, 1e-30f, 1e-6f, 0.05f, 1.f, 100.f, 1e6f, 3e38f};
      for (float a : edge)
        for (float b : edge) check(a, b, sa, ca, th, tb);
    }
  }
  std::printf("seg_edge_fast: %ld cases, %ld in the atan2f band, %ld mismatches\n", n, band, bad);
  return bad == 0 ? 0 : 1;
}
