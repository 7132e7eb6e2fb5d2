// lego_seg.h — the segmentation angle test of labelComponents
// (imageProjection.cpp:421-423): with d1 / d2 the larger / smaller of two
// neighbouring ranges, the pixels join when
//     atan2f(d2 sin(alpha), d1 - d2 cos(alpha)) > theta.
// seg_edge_fast returns that verdict without atan2f away from the threshold:
// for x > 0, y >= 0 the angle is atan(y / x), and a quotient beyond
// tan(theta -+ 1e-5) puts the angle 1e-5 rad from theta — far outside
// atan2f's 2-ulp error plus the quotient's rounding (< 4e-7 rad together);
// for x <= 0 < y the angle is at least pi / 2 > theta.  Everything else, and
// every quotient inside the band, takes atan2f itself, so the verdict is the
// reference's bit for bit (tests/native/seg_edge_check.cpp pins it against
// atan2f on random and near-threshold pairs).
#pragma once
#include <cmath>

#include "lego_numerics.h"

namespace lego {

struct TanBand {
  double lo, hi;  // tan(theta - 1e-5), tan(theta + 1e-5)
  bool quad1;     // theta < pi / 2 - 1e-3: the x <= 0 shortcut holds
};

// host side (DevCfg carries the three values to the kernels)
inline TanBand seg_tan_band_host(float theta) {
  return TanBand{std::tan((double)theta - 1e-5), std::tan((double)theta + 1e-5),
                 (double)theta < M_PI / 2 - 1e-3};
}

LEGO_HD bool seg_edge_fast(float ra, float rb, float sa, float ca, float theta, const TanBand& tb) {
  const float d1 = (ra < rb) ? rb : ra;  // std::max
  const float d2 = (rb < ra) ? rb : ra;  // std::min
  const float y = d2 * sa, x = d1 - d2 * ca;
  if (tb.quad1 && y >= 0.f && x > 0.f) {
    const double q = (double)(y / x);
    if (q > tb.hi) return true;
    if (q < tb.lo) return false;
  } else if (tb.quad1 && y > 0.f && x <= 0.f) {
    return true;
  }
  return lego_atan2f(y, x) > theta;
}

// the reference's expression, for the checks
LEGO_HD bool seg_edge_ref(float ra, float rb, float sa, float ca, float theta) {
  const float d1 = (ra < rb) ? rb : ra;
  const float d2 = (rb < ra) ? rb : ra;
  return lego_atan2f(d2 * sa, (d1 - d2 * ca)) > theta;
}

}  // namespace lego
