// Exhaustive / sampled equivalence checks of csrc/tfp_math.hpp against this host's glibc.
// Built and run by tests/test_math_exact.py (sampled stride) and by hand with stride 1
// (exhaustive; the log of that run is committed under tests/native/).
// usage: check_math <stride>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cstdint>
#include "../../asterisk-tiresias_amd/csrc/tfp_math.hpp"

using namespace tfp;

static int64_t fmt6_printf(double x) {
  char buf[512];
  snprintf(buf, sizeof buf, "%f", x);
  // parse "[-]int.frac6" into micro-units exactly
  const char* s = buf; bool neg = false;
  if (*s == '-') { neg = true; ++s; }
  int64_t v = 0;
  for (; *s && *s != '.'; ++s) v = v * 10 + (*s - '0');
  if (*s == '.') ++s;
  for (int i = 0; i < 6; ++i) v = v * 10 + (s[i] - '0');
  return neg ? -v : v;
}

int main(int argc, char** argv) {
  const uint64_t stride = argc > 1 ? strtoull(argv[1], 0, 10) : 1;
  int rc = 0;
  // 1. log10f_glibc == glibc log10f over positive finite floats (incl. subnormals)
  {
    uint64_t tot = 0, bad = 0;
#pragma omp parallel for reduction(+ : tot, bad) schedule(static)
    for (int64_t u = 1; u < 0x7f800000LL; u += (int64_t)stride) {
      const float x = u2f((uint32_t)u);
      tot++;
      if (f2u(log10f_glibc(x)) != f2u(log10f(x))) bad++;
    }
    printf("log10f_glibc vs glibc log10f : %lu / %lu mismatches\n", bad, tot);
    rc |= bad != 0;
  }
  // 2. logf_glibc == glibc logf on every float of [0.5, 2)
  {
    uint64_t tot = 0, bad = 0;
    for (uint32_t u = f2u(0.5f); u < f2u(2.0f); ++u) {
      tot++;
      if (f2u(logf_glibc(u2f(u))) != f2u(logf(u2f(u)))) bad++;
    }
    printf("logf_glibc vs glibc logf [0.5,2): %lu / %lu mismatches\n", bad, tot);
    rc |= bad != 0;
  }
  // 3. dB value: fmt6 and trunc of 10*log10|c| agree with glibc for every positive float c
  {
    uint64_t tot = 0, bad_fmt = 0, bad_trunc = 0, bits_diff = 0;
#pragma omp parallel for reduction(+ : tot, bad_fmt, bad_trunc, bits_diff) schedule(static)
    for (int64_t u = 1; u < 0x7f800000LL; u += (int64_t)stride) {
      const float c = u2f((uint32_t)u);
      const double mine = db_of_coef(c);
      const double ref = 10 * log10(fabs((double)c));
      tot++;
      if (d2u(mine) != d2u(ref)) bits_diff++;
      if (fmt6(mine) != fmt6(ref)) bad_fmt++;
      if ((int)mine != (int)ref) bad_trunc++;
    }
    printf("dB 10*log10|c| : %lu floats, %lu differ in last bits, %lu fmt6 mismatches, %lu trunc mismatches\n",
           tot, bits_diff, bad_fmt, bad_trunc);
    rc |= (bad_fmt | bad_trunc) != 0;
  }
  // 4. fmt6 == printf("%f") on random doubles, exact ties and near-ties
  {
    uint64_t tot = 0, bad = 0;
    uint64_t st = 0x9E3779B97F4A7C15ull;
    auto rnd = [&]() { st += 0x9E3779B97F4A7C15ull; uint64_t z = st; z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull; z = (z ^ (z >> 27)) * 0x94D049BB133111EBull; return z ^ (z >> 31); };
    const uint64_t n = 4000000 / (stride > 64 ? 64 : stride);
    for (uint64_t i = 0; i < n; ++i) {
      double x;
      switch (i % 4) {
        case 0: x = ((double)(rnd() >> 11) / 9007199254740992.0 - 0.5) * 1000.0; break;        // uniform
        case 1: x = (double)((int64_t)(rnd() % 2000000000) - 1000000000) / 128.0 / 1e3; break;  // k/128000: many exact ties
        case 2: { double m = (double)((int64_t)(rnd() % 1000000000) - 500000000) + 0.5; x = m / 1e6; x = u2d(d2u(x) + (int64_t)(rnd() % 5) - 2); break; }  // near half-micro
        default: x = u2d(rnd() & 0x7fefffffffffffffull); if (!(fabs(x) < 4e6)) x = fmod(x, 4e6); if (rnd() & 1) x = -x; break;
      }
      tot++;
      if (fmt6(x) != fmt6_printf(x)) { if (bad < 5) printf("  fmt6 mismatch x=%a mine=%ld printf=%ld\n", x, (long)fmt6(x), (long)fmt6_printf(x)); bad++; }
    }
    printf("fmt6 vs printf(\"%%f\") : %lu / %lu mismatches\n", bad, tot);
    rc |= bad != 0;
  }
  // 5. aubio_log10_fast (branch-free, kernel) == aubio_log10_clamped on every non-negative float
  {
    uint64_t tot = 0, bad = 0;
#pragma omp parallel for reduction(+ : tot, bad) schedule(static)
    for (int64_t u = 0; u <= 0x7f7fffffLL; u += (int64_t)stride) {
      const float x = u2f((uint32_t)u);
      tot++;
      if (f2u(aubio_log10_fast(x)) != f2u(aubio_log10_clamped(x))) bad++;
    }
    tot++;
    if (f2u(aubio_log10_fast(-0.0f)) != f2u(aubio_log10_clamped(-0.0f))) bad++;
    printf("aubio_log10_fast vs aubio_log10_clamped : %lu / %lu mismatches\n", bad, tot);
    rc |= bad != 0;
  }
  printf(rc ? "FAIL\n" : "OK\n");
  return rc;
}
