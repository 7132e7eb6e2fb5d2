// Pins the partition rules of lego_vgsort.h against libstdc++'s std::sort of
// (voxel idx, point index) pairs by idx (pcl::VoxelGrid's sort,
// featureAssociation.cpp:778-780, mapOptmization.cpp:1058-1091): the same
// final order of equal keys on tie-heavy, presorted, reversed, organ-pipe and
// adversarial (McIlroy "antiqsort", which drives introsort into its heap-sort
// fallback) inputs.
//
// The restatement below is the kernels' algorithm with the wave's lanes
// unrolled into a scalar loop: a count of the left stops, then one pass from
// the right ranking left and right stops by the counts after each position,
// the swapped right stops scattered by rank, the swapped left stops fetching
// their partner, the cut = the lowest unswapped left stop or swapped right
// stop; levels processed one after another, blocks of <= 16 stable-sorted,
// heap sort when a level's depth budget is spent.  Built and run by
// tests/test_numerics_shim.py.
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

struct Idx {
  unsigned idx;
  unsigned cpi;
  bool operator<(const Idx& o) const { return idx < o.idx; }
};

static uint64_t s = 987654321;
static uint64_t rnd() {
  s += 0x9e3779b97f4a7c15ULL;
  uint64_t z = s;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

// ---- the restatement
static void swp(std::vector<Idx>& a, int i, int j) { std::swap(a[i], a[j]); }
static void median_to_first(std::vector<Idx>& a, int r, int x, int y, int z) {
  int m;
  if (a[x].idx < a[y].idx) {
    if (a[y].idx < a[z].idx) m = y;
    else if (a[x].idx < a[z].idx) m = z;
    else m = x;
  } else if (a[x].idx < a[z].idx) m = x;
  else if (a[y].idx < a[z].idx) m = z;
  else m = y;
  swp(a, r, m);
}
static int partition(std::vector<Idx>& a, int s, int e, std::vector<int>& pr) {
  median_to_first(a, s, s + 1, s + (e - s) / 2, e - 1);
  const unsigned p = a[s].idx;
  int totL = 0;
  for (int i = s + 1; i < e; ++i) totL += !(a[i].idx < p);
  int Lab = 0, Rab = 0, cut = e;
  std::vector<std::pair<int, int>> swaps;
  for (int i = e - 1; i > s; --i) {
    const bool lf = !(a[i].idx < p), rf = !(p < a[i].idx);
    const bool rsw = rf && totL - Lab - (lf ? 1 : 0) >= Rab + 1;
    const bool lsw = lf && Rab >= totL - Lab;
    if (rsw) pr[s + Rab] = i;
    if ((lf && !lsw) || rsw) cut = i;
    if (lsw) swaps.push_back({i, pr[s + (totL - Lab) - 1]});
    Lab += lf;
    Rab += rf;
  }
  for (auto& w : swaps) swp(a, w.first, w.second);
  return cut;
}
static void heap_sort(std::vector<Idx>& a, int s, int e) {
  std::make_heap(a.begin() + s, a.begin() + e);
  std::sort_heap(a.begin() + s, a.begin() + e);
}
static void leaf_sort(std::vector<Idx>& a, int s, int e) { std::stable_sort(a.begin() + s, a.begin() + e); }

static int heap_segments = 0;
static void emulate(std::vector<Idx>& a) {
  const int n = (int)a.size();
  if (n <= 1) return;
  if (n <= 16) { leaf_sort(a, 0, n); return; }
  int D = 0;
  while ((2 << D) <= n) ++D;
  D *= 2;
  std::vector<int> pr(n);
  std::vector<std::pair<int, int>> cur{{0, n}}, nxt;
  for (int r = 0; !cur.empty(); ++r) {
    nxt.clear();
    for (auto [s0, e0] : cur) {
      if (D - r == 0) { heap_sort(a, s0, e0); ++heap_segments; continue; }
      const int cut = partition(a, s0, e0, pr);
      if (cut - s0 > 16) nxt.push_back({s0, cut}); else leaf_sort(a, s0, cut);
      if (e0 - cut > 16) nxt.push_back({cut, e0}); else leaf_sort(a, cut, e0);
    }
    std::swap(cur, nxt);
  }
}

// ---- McIlroy's adversary against std::sort (A Killer Adversary for Quicksort, 1999)
static std::vector<unsigned> killer(int n) {
  std::vector<int> val(n), ptr(n);
  const int gas = n;
  int nsolid = 0, candidate = 0;
  for (int i = 0; i < n; ++i) { val[i] = gas; ptr[i] = i; }
  auto cmp = [&](int x, int y) {
    if (val[x] == gas && val[y] == gas) {
      if (x == candidate) val[x] = nsolid++;
      else val[y] = nsolid++;
    }
    if (val[x] == gas) candidate = x;
    else if (val[y] == gas) candidate = y;
    return val[x] < val[y];
  };
  std::sort(ptr.begin(), ptr.end(), cmp);
  std::vector<unsigned> out(n);
  for (int i = 0; i < n; ++i) out[i] = (unsigned)(val[i] == gas ? nsolid++ : val[i]);
  return out;
}

int main(int argc, char** argv) {
  if (argc == 4 && std::string(argv[1]) == "killer") {  // keys for tests/golden/make_vg_killer.py
    std::vector<unsigned> k = killer(atoi(argv[2]));
    const unsigned div = (unsigned)atoi(argv[3]);
    for (auto& x : k) x /= div;
    fwrite(k.data(), sizeof(unsigned), k.size(), stdout);
    return 0;
  }
  if (argc == 3 && std::string(argv[1]) == "heaps") {  // heap-sorted pieces std::sort takes on these keys
    std::vector<unsigned> k;
    unsigned x;
    FILE* f = fopen(argv[2], "rb");
    if (!f) return 2;
    while (fread(&x, sizeof x, 1, f) == 1) k.push_back(x);
    fclose(f);
    std::vector<Idx> a(k.size()), b;
    for (size_t i = 0; i < k.size(); ++i) a[i] = {k[i], (unsigned)i};
    b = a;
    std::sort(a.begin(), a.end(), std::less<Idx>());
    emulate(b);
    for (size_t i = 0; i < a.size(); ++i)
      if (a[i].cpi != b[i].cpi) return 3;
    printf("%d\n", heap_segments);
    return 0;
  }
  const int trials = argc > 1 ? atoi(argv[1]) : 6000;
  long bad = 0, total = 0;
  auto check = [&](const std::vector<unsigned>& keys) {
    std::vector<Idx> a(keys.size()), b;
    for (size_t i = 0; i < keys.size(); ++i) a[i] = {keys[i], (unsigned)i};
    b = a;
    std::sort(a.begin(), a.end(), std::less<Idx>());
    emulate(b);
    ++total;
    for (size_t i = 0; i < a.size(); ++i)
      if (a[i].cpi != b[i].cpi) { ++bad; return; }
  };
  for (int t = 0; t < trials; ++t) {
    const int n = t < 40 ? t : 1 + (int)(rnd() % (t % 7 == 0 ? 70000 : 5000));
    const unsigned distinct = 1 + (unsigned)(rnd() % (t % 4 == 0 ? 3 : t % 4 == 1 ? 50 : t % 4 == 2 ? 1000 : 4000000));
    std::vector<unsigned> k(n);
    const int mode = t % 6;
    for (int i = 0; i < n; ++i) {
      if (mode == 0) k[i] = (unsigned)(rnd() % distinct);
      else if (mode == 1) k[i] = (unsigned)(i / (1 + distinct % 9));               // ascending runs
      else if (mode == 2) k[i] = (unsigned)((n - i) / (1 + distinct % 5));         // descending runs
      else if (mode == 3) k[i] = (unsigned)std::min(i, n - i) % (distinct + 1);    // organ pipe
      else if (mode == 4) k[i] = (unsigned)((i * 37) % 101 + (rnd() % 3) * 1000);  // scan-like runs
      else k[i] = (unsigned)(i + (rnd() % 8 == 0 ? rnd() % 64 : 0)) / 4;           // nearly sorted, ties
    }
    check(k);
  }
  const int hs0 = heap_segments;
  for (int n : {17, 33, 64, 100, 257, 1000, 1832, 4096, 20000}) check(killer(n));
  const int heaps = heap_segments - hs0;
  printf("inputs %ld mismatching %ld heap-sorted segments (adversarial) %d\n", total, bad, heaps);
  return (bad != 0 || heaps == 0) ? 1 : 0;
}
