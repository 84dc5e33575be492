// tfp_math.hpp db_of_coef WITH the LogFix table (tfp_tables.cpp log_fix_table) against this host's
// glibc `10 * log10(fabs((double)c))` (fp_handler.c:651), bit for bit, over every positive float c
// (stride 1; tests/test_math_exact.py runs a sampled stride). The frame values (q1, q2) the engine
// hands back and searches with come from this function on the device.
// usage: check_logfix <stride>
#include <cmath>
#include <cstdio>
#include <cstdlib>
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
  uint64_t tot = 0, bad = 0, bad_nofix = 0;
#pragma omp parallel for reduction(+ : tot, bad, bad_nofix) schedule(static)
  for (int64_t u = 1; u < 0x7f800000LL; u += (int64_t)stride) {
    const float c = u2f((uint32_t)u);
    const double want = 10.0 * log10(fabs((double)c));
    tot++;
    bad += d2u(db_of_coef(c, fx)) != d2u(want);
    bad_nofix += d2u(db_of_coef(c)) != d2u(want);
  }
  printf("LogFix entries: %d\n", n);
  printf("10*log10|c| with LogFix vs glibc : %lu / %lu mismatches (without the table: %lu)\n", (unsigned long)bad,
         (unsigned long)tot, (unsigned long)bad_nofix);
  printf("%s\n", bad ? "FAIL" : "OK");
  return bad ? 1 : 0;
}
