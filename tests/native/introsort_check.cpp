// Pins lego_introsort.h against libstdc++ std::sort (the sort the reference
// calls at featureAssociation.cpp:699): identical permutations on tie-heavy
// inputs.  Built and run by tests/test_introsort_port.py.
#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <vector>
#include "../../lego-loam_amd/csrc/lego_introsort.h"

struct smoothness_t { float value; size_t ind; };
struct by_value { bool operator()(smoothness_t const& l, smoothness_t const& r) { return l.value < r.value; } };

static uint64_t s = 12345;
static uint64_t rnd() { s += 0x9e3779b97f4a7c15ULL; uint64_t z = s; z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL; z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL; return z ^ (z >> 31); }

int main(int argc, char** argv) {
  int trials = argc > 1 ? atoi(argv[1]) : 20000;
  long bad = 0;
  for (int t = 0; t < trials; ++t) {
    int n = 1 + (int)(rnd() % 700);
    int distinct = 1 + (int)(rnd() % (t % 3 == 0 ? 4 : t % 3 == 1 ? 40 : 100000));
    std::vector<smoothness_t> a(n);
    std::vector<lego::SmoothEntry> b(n);
    int mode = t % 5;
    for (int i = 0; i < n; ++i) {
      float v;
      if (mode == 0) v = (float)(rnd() % distinct);
      else if (mode == 1) v = (float)(i % distinct);            // sawtooth
      else if (mode == 2) v = (float)((n - i) / (1 + distinct % 7)); // descending runs
      else if (mode == 3) v = (float)(rnd() % distinct) * 0.1f;
      else v = (i % 17 == 0) ? 0.0f : (float)(rnd() % distinct);
      a[i] = {v, (size_t)i};
      b[i] = {v, i};
    }
    std::sort(a.begin(), a.end(), by_value());
    uint32_t stk[lego::kIntroStack];
    lego::std_sort_by_value(b.data(), n, stk);
    for (int i = 0; i < n; ++i)
      if ((int)a[i].ind != b[i].ind) { ++bad; break; }
  }
  printf("trials %d mismatching %ld\n", trials, bad);
  return bad != 0;
}
