// lego_introsort.h — exact restatement of libstdc++'s std::sort (GCC 11,
// /usr/include/c++/11/bits/stl_algo.h:1925-1957 introsort loop, :1861-1871
// final insertion sort with _S_threshold = 16, :79-97 median-of-three,
// stl_heap.h adjust/push/pop heap), for a (float value, int ind) array compared
// by value only (utility.h:144-148 `by_value`).
//
// featureAssociation.cpp:699 sorts each sector with std::sort; the sort is
// unstable, so the order of EQUAL curvatures — which decides which point is
// picked first — is libstdc++'s.  The kernels sort sectors with a bitonic
// network and fall back to this routine only when a sector holds ties
// (tests/test_introsort_port.py pins it against the real std::sort).
#pragma once
#include "lego_numerics.h"

namespace lego {

struct SmoothEntry {
  float value;
  int ind;
};

// Access through a pointer so the same code runs on LDS (device) and host memory.
template <typename Ptr>
struct IntroSort {
  Ptr a;
  LEGO_HD bool lt(int i, int j) const { return a[i].value < a[j].value; }
  LEGO_HD void swp(int i, int j) const {
    SmoothEntry t = a[i];
    a[i] = a[j];
    a[j] = t;
  }
  static LEGO_HD int lg(int n) { return 31 - __builtin_clz((unsigned)n); }

  LEGO_HD void move_median_to_first(int result, int x, int y, int z) const {
    if (lt(x, y)) {
      if (lt(y, z)) swp(result, y);
      else if (lt(x, z)) swp(result, z);
      else swp(result, x);
    } else if (lt(x, z)) swp(result, x);
    else if (lt(y, z)) swp(result, z);
    else swp(result, y);
  }
  LEGO_HD int unguarded_partition(int first, int last, int pivot) const {
    while (true) {
      while (lt(first, pivot)) ++first;
      --last;
      while (lt(pivot, last)) --last;
      if (!(first < last)) return first;
      swp(first, last);
      ++first;
    }
  }
  LEGO_HD int unguarded_partition_pivot(int first, int last) const {
    int mid = first + (last - first) / 2;
    move_median_to_first(first, first + 1, mid, last - 1);
    return unguarded_partition(first + 1, last, first);
  }
  LEGO_HD void push_heap(int first, int hole, int top, SmoothEntry v) const {
    int parent = (hole - 1) / 2;
    while (hole > top && a[first + parent].value < v.value) {
      a[first + hole] = a[first + parent];
      hole = parent;
      parent = (hole - 1) / 2;
    }
    a[first + hole] = v;
  }
  LEGO_HD void adjust_heap(int first, int hole, int len, SmoothEntry v) const {
    const int top = hole;
    int second = hole;
    while (second < (len - 1) / 2) {
      second = 2 * (second + 1);
      if (lt(first + second, first + (second - 1))) second--;
      a[first + hole] = a[first + second];
      hole = second;
    }
    if ((len & 1) == 0 && second == (len - 2) / 2) {
      second = 2 * (second + 1);
      a[first + hole] = a[first + (second - 1)];
      hole = second - 1;
    }
    push_heap(first, hole, top, v);
  }
  LEGO_HD void make_heap(int first, int last) const {
    if (last - first < 2) return;
    const int len = last - first;
    int parent = (len - 2) / 2;
    while (true) {
      SmoothEntry v = a[first + parent];
      adjust_heap(first, parent, len, v);
      if (parent == 0) return;
      parent--;
    }
  }
  LEGO_HD void pop_heap(int first, int last, int result) const {
    SmoothEntry v = a[result];
    a[result] = a[first];
    adjust_heap(first, 0, last - first, v);
  }
  LEGO_HD void heap_sort(int first, int last) const {  // __partial_sort(first, last, last)
    make_heap(first, last);
    while (last - first > 1) {
      --last;
      pop_heap(first, last, last);
    }
  }
  // The recursion on the right part becomes an explicit stack of packed frames
  // (first | last << 13 | depth << 26; n < 8192).  A frame's depth is below
  // every frame under it, so the stack never holds more than 2 lg n + 1 <=
  // kIntroStack frames.  The caller provides the stack: on the device a slice
  // of LDS, so the kernel needs no private (scratch) memory.
  LEGO_HD void introsort_loop(int first, int last, int depth, uint32_t* st) const {
    int sp = 0;
    st[sp++] = (uint32_t)first | ((uint32_t)last << 13) | ((uint32_t)depth << 26);
    while (sp > 0) {
      const uint32_t f = st[--sp];
      first = (int)(f & 8191u); last = (int)((f >> 13) & 8191u); depth = (int)(f >> 26);
      while (last - first > 16) {
        if (depth == 0) {
          heap_sort(first, last);
          break;
        }
        --depth;
        int cut = unguarded_partition_pivot(first, last);
        // std: __introsort_loop(cut, last, depth) first, then continue on [first, cut)
        // Order matters only for when sub-ranges are processed; they are
        // disjoint, so results are identical whichever runs first.
        st[sp++] = (uint32_t)cut | ((uint32_t)last << 13) | ((uint32_t)depth << 26);
        last = cut;
      }
    }
  }
  LEGO_HD void unguarded_linear_insert(int last) const {
    SmoothEntry v = a[last];
    int next = last - 1;
    while (v.value < a[next].value) {
      a[last] = a[next];
      last = next;
      --next;
    }
    a[last] = v;
  }
  LEGO_HD void insertion_sort(int first, int last) const {
    if (first == last) return;
    for (int i = first + 1; i != last; ++i) {
      if (lt(i, first)) {
        SmoothEntry v = a[i];
        for (int k = i; k > first; --k) a[k] = a[k - 1];
        a[first] = v;
      } else {
        unguarded_linear_insert(i);
      }
    }
  }
  LEGO_HD void final_insertion_sort(int first, int last) const {
    if (last - first > 16) {
      insertion_sort(first, first + 16);
      for (int i = first + 16; i != last; ++i) unguarded_linear_insert(i);
    } else {
      insertion_sort(first, last);
    }
  }
  LEGO_HD void sort(int first, int last, uint32_t* st) const {
    if (last - first > 1) {
      introsort_loop(first, last, lg(last - first) * 2, st);
      final_insertion_sort(first, last);
    }
  }
};

constexpr int kIntroStack = 28;  // frames: 2 lg n + 1 for n < 8192

// n < 8192; `stack` holds kIntroStack words
template <typename Ptr>
LEGO_HD void std_sort_by_value(Ptr a, int n, uint32_t* stack) {
  IntroSort<Ptr> s{a};
  s.sort(0, n, stack);
}

}  // namespace lego
