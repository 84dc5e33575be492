// tfp_math.hpp db_of_coef WITH the LogFix table (tfp_tables.cpp log_fix_table) against this host's
// glibc `10 * log10(fabs((double)c))` (fp_handler.c:651), bit for bit, over every positive float c
// (stride 1; tests/test_math_exact.py runs a sampled stride). The frame values (q1, q2) the engine
// hands back and searches with come from this function on the device.
// usage: check_logfix <stride>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../../asterisk-tiresias_amd/csrc/tfp_math.hpp"
#include "../../asterisk-tiresias_amd/csrc/tfp_tables.hpp"

using namespace tfp;

int main(int argc, char** argv) {
  const uint64_t stride = argc > 1 ? strtoull(argv[1], 0, 10) : 1;
  const uint32_t* k;
  const double* v;
  int32_t n;
  log_fix_table(&k, &v, &n);
  const LogFix fx{k, v, n};
  // the hashed form the engine uploads (tfp_tables.cpp log_fix_hash): the same value as the sorted
  // table's binary search for every key of the 2^24 reduced-argument domain, present or not
  const uint32_t* hk;
  const double* hv;
  int32_t hn;
  log_fix_hash(&hk, &hv, &hn);
  std::vector<uint32_t> bits(1u << 19, 0u);  // (the engine's bitmap of the keys present)
  for (int32_t j = 0; j < (1 << kLogFixHashBits); j++)
    if (hk[j] != kLogFixEmpty) bits[hk[j] >> 5] |= 1u << (hk[j] & 31);
  const LogFix hx{hk, hv, hn, 1, bits.data()};
  uint64_t bad_hash = hn != n;
#pragma omp parallel for reduction(+ : bad_hash) schedule(static)
  for (int64_t key = 0; key < (1 << 24); key++) {
    const int32_t i = (int32_t)(key >> 23);
    const double x = u2d(((uint64_t)(0x3ff - i) << 52) | ((uint64_t)(key & 0x7fffff) << 29));
    bad_hash += d2u(log_fixed(x, i, hx)) != d2u(log_fixed(x, i, fx));
  }
  uint64_t tot = 0, bad = 0, bad_nofix = 0;
#pragma omp parallel for reduction(+ : tot, bad, bad_nofix) schedule(static)
  for (int64_t u = 1; u < 0x7f800000LL; u += (int64_t)stride) {
    const float c = u2f((uint32_t)u);
    const double want = 10.0 * log10(fabs((double)c));
    tot++;
    bad += d2u(db_of_coef(c, fx)) != d2u(want);
    bad += d2u(db_of_coef(c, hx)) != d2u(want);
    bad_nofix += d2u(db_of_coef(c)) != d2u(want);
  }
  printf("LogFix entries: %d\n", n);
  printf("hashed LogFix vs sorted over the 2^24 key domain: %lu mismatches\n", (unsigned long)bad_hash);
  printf("10*log10|c| with LogFix vs glibc : %lu / %lu mismatches (without the table: %lu)\n", (unsigned long)bad,
         (unsigned long)tot, (unsigned long)bad_nofix);
  bad += bad_hash;
  printf("%s\n", bad ? "FAIL" : "OK");
  return bad ? 1 : 0;
}
