// tfp_bsearch.hpp's lb32 / ub32 (the sweep's bucket searches, tfp_scan.hip find_ab) against
// std::lower_bound / std::upper_bound: every query value around every element of random ascending
// arrays of 0..70 elements with runs of equal values (crowds), and a 5,000-element crowd.
#include <algorithm>
#include <cstdio>
#include <random>
#include <vector>
#include "../../asterisk-tiresias_amd/csrc/tfp_bsearch.hpp"

int main() {
  std::mt19937 rng(7);
  long bad = 0, n_checks = 0;
  auto check = [&](const std::vector<int32_t>& a, int32_t v) {
    const int32_t n = (int32_t)a.size();
    const int32_t* p = a.data();
    const int32_t ub = (int32_t)(std::upper_bound(a.begin(), a.end(), v) - a.begin());
    const int32_t lb = (int32_t)(std::lower_bound(a.begin(), a.end(), v) - a.begin());
    bad += tfp::ub32(p, n, v) != ub;
    bad += tfp::lb32(p, n, v) != lb;
    n_checks += 2;
  };
  for (int trial = 0; trial < 20000; trial++) {
    const int n = trial % 71;
    std::vector<int32_t> a(n);
    int32_t x = (int32_t)(rng() % 50) - 25;
    for (int i = 0; i < n; i++) {
      if (rng() % 3) x += (int32_t)(rng() % 4);  // steps of 0..3: runs of equal values
      a[i] = x;
    }
    for (int i = 0; i < n; i++)
      for (int d = -1; d <= 1; d++) check(a, a[i] + d);
    check(a, -1000);
    check(a, 1000);
  }
  std::vector<int32_t> crowd(5000, -60206000);
  for (int32_t v : {-60206001, -60206000, -60205999}) check(crowd, v);
  crowd.push_back(-1000);
  for (int32_t v : {-60206001, -60206000, -60205999, -1001, -1000, 0}) check(crowd, v);
  printf("lb32 / ub32 vs std: %ld / %ld mismatches\n%s\n", bad, n_checks, bad ? "FAIL" : "OK");
  return bad ? 1 : 0;
}
