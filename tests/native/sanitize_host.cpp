// TEST HARNESS (tests/test_sanitizers.py; not product code): the host-side C/C++ of the product and
// of the checker under AddressSanitizer + UndefinedBehaviorSanitizer, on the CPU (GPU sanitizers are
// not available on this pool; the device code is not in this build):
//   - csrc/tfp_wav.cpp: WAV ingest (aubio_source's job) on valid files of every layout, every
//     truncation of their headers, size-query / capacity calls, and random bytes behind a RIFF header;
//   - csrc/tfp_tables.cpp: the DSP tables at several sample rates, the glibc log correction table;
//   - oracle/oracle.c + oracle/oracle_boxes.c: fingerprints of edge lengths, the searches (row scan,
//     sorted, per-box) on a random table with NULL rows.
// Built with -fsanitize=address,undefined -fno-sanitize-recover=all: any finding aborts.
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>
#include <string>
#include <vector>

#include "../../asterisk-tiresias_amd/csrc/tfp_tables.hpp"
#include "../../include/tiresias_fp.h"
extern "C" {
#include "../../oracle/tfp_oracle.h"
}

static int fails = 0;
#define CHECK(c)                                                      \
  do {                                                                \
    if (!(c)) {                                                       \
      fprintf(stderr, "check failed: %s (line %d)\n", #c, __LINE__); \
      fails++;                                                        \
    }                                                                 \
  } while (0)

static void put16(std::vector<uint8_t>& b, uint32_t v) { b.push_back(v & 255); b.push_back((v >> 8) & 255); }
static void put32(std::vector<uint8_t>& b, uint32_t v) { put16(b, v & 0xffff); put16(b, v >> 16); }

// RIFF/WAVE with a fmt chunk (extensible when ext), an odd-sized padding chunk, then data
static std::vector<uint8_t> wav(int fmt, int ch, int bits, int sr, const std::vector<uint8_t>& data, bool ext) {
  std::vector<uint8_t> b = {'R', 'I', 'F', 'F', 0, 0, 0, 0, 'W', 'A', 'V', 'E', 'f', 'm', 't', ' '};
  put32(b, ext ? 40 : 16);
  put16(b, ext ? 0xFFFE : fmt);
  put16(b, ch);
  put32(b, sr);
  put32(b, sr * ch * bits / 8);
  put16(b, ch * bits / 8);
  put16(b, bits);
  if (ext) {
    put16(b, 22);
    put16(b, bits);
    put32(b, 0);
    put32(b, fmt);  // subformat GUID: the format code, then the standard tail
    const uint8_t tail[12] = {0x00, 0x00, 0x00, 0x00, 0x10, 0x00, 0x80, 0x00, 0x00, 0xAA, 0x00, 0x38};
    b.insert(b.end(), tail, tail + 12);
  }
  const uint8_t pad[] = {'j', 'u', 'n', 'k', 3, 0, 0, 0, 1, 2, 3, 0};
  b.insert(b.end(), pad, pad + sizeof pad);
  b.insert(b.end(), {'d', 'a', 't', 'a'});
  put32(b, (uint32_t)data.size());
  b.insert(b.end(), data.begin(), data.end());
  const uint32_t riff = (uint32_t)b.size() - 8;
  memcpy(&b[4], &riff, 4);
  return b;
}

static void decode_all(const std::vector<uint8_t>& b) {
  int64_t n = -1;
  int32_t sr = 0;
  for (int f32 = 0; f32 < 2; f32++) {
    const int rc = f32 ? tfp_wav_decode_f32(b.data(), (int64_t)b.size(), nullptr, 0, &n, &sr)
                       : tfp_wav_decode(b.data(), (int64_t)b.size(), nullptr, 0, &n, &sr);
    if (rc != TFP_OK) continue;
    CHECK(n >= 0);
    for (int64_t cap : {n, n > 0 ? n - 1 : 0}) {  // exact and one short (TFP_E_CAPACITY)
      std::vector<int16_t> p(cap + 1);
      std::vector<float> x(cap + 1);
      int64_t got = -1;
      const int r2 = f32 ? tfp_wav_decode_f32(b.data(), (int64_t)b.size(), x.data(), cap, &got, &sr)
                         : tfp_wav_decode(b.data(), (int64_t)b.size(), p.data(), cap, &got, &sr);
      CHECK(cap >= n ? r2 == TFP_OK : r2 == TFP_E_CAPACITY);
      CHECK(got == n);
    }
  }
}

static void wav_tests() {
  std::mt19937 rng(7);
  std::vector<uint8_t> data(6 * 1001);
  for (auto& v : data) v = (uint8_t)rng();
  struct L { int fmt, ch, bits; bool ext; };
  const L layouts[] = {{1, 1, 16, false}, {1, 1, 8, false}, {1, 2, 16, false}, {1, 3, 24, false}, {1, 1, 32, false},
                       {3, 1, 32, false}, {3, 2, 64, false}, {1, 1, 16, true}, {3, 2, 32, true}, {1, 2, 24, true},
                       {2, 1, 16, false}, {1, 0, 16, false}, {1, 1, 12, false}};
  for (const L& l : layouts) {
    for (int sr : {8000, 16000, 44100}) {
      const std::vector<uint8_t> b = wav(l.fmt, l.ch, l.bits, sr, data, l.ext);
      decode_all(b);
      for (size_t cut = 0; cut < b.size(); cut += (cut < 120 ? 1 : 97))  // every header truncation
        decode_all(std::vector<uint8_t>(b.begin(), b.begin() + cut));
      std::vector<uint8_t> big = b;  // a data size past the end of the bytes
      const uint32_t huge = 0x7ffffff0u;
      memcpy(&big[big.size() - data.size() - 4], &huge, 4);
      decode_all(big);
    }
  }
  for (int i = 0; i < 300; i++) {  // random bytes behind a RIFF/WAVE header
    std::vector<uint8_t> b = {'R', 'I', 'F', 'F', 0, 0, 0, 0, 'W', 'A', 'V', 'E'};
    const size_t extra = rng() % 200;
    for (size_t k = 0; k < extra; k++) b.push_back((uint8_t)(k < 4 ? "fmt "[k] : rng()));
    decode_all(b);
  }
  int64_t n;
  int32_t sr;
  CHECK(tfp_wav_read("/nonexistent/x.wav", nullptr, 0, &n, &sr) != TFP_OK);
  CHECK(tfp_wav_read_f32("/nonexistent/x.wav", nullptr, 0, &n, &sr) != TFP_OK);
}

static void table_tests() {
  for (int sr : {8000, 11025, 16000, 22050, 44100, 48000, 96000}) {
    tfp::DspTables t;
    CHECK(tfp::build_tables(sr, &t));
  }
  tfp::DspTables t;
  CHECK(!tfp::build_tables(0, &t));
  const uint32_t* k;
  const double* v;
  int32_t n = 0;
  tfp::log_fix_table(&k, &v, &n);
  CHECK(n > 0);
}

static void oracle_tests() {
  std::mt19937 rng(11);
  tfo_tables T;
  for (int sr : {8000, 16000, 44100}) CHECK(tfo_build_tables(sr, &T) == 0);
  CHECK(tfo_build_tables(8000, &T) == 0);
  for (size_t n : {0, 1, 255, 256, 257, 511, 512, 513, 4000}) {
    std::vector<int16_t> p(n + 1);
    for (auto& v : p) v = (int16_t)(rng() % 65536 - 32768);
    const size_t nf = tfo_frame_count(n);
    std::vector<float> coef(2 * nf + 2);
    std::vector<double> db(2 * nf + 2);
    std::vector<int32_t> micro(2 * nf + 2);
    CHECK(tfo_fingerprint(&T, p.data(), n, coef.data(), db.data(), micro.data()) == nf);
    std::vector<float> x(n + 1);
    for (size_t i = 0; i < n; i++) x[i] = p[i] / 32768.f;
    if (n) x[n / 2] = INFINITY;  // non-finite input
    CHECK(tfo_fingerprint_f32(&T, x.data(), n, coef.data(), db.data(), micro.data()) == nf);
  }
  // a batch on 4 threads
  std::vector<int64_t> off = {0, 3000, 3000, 8001, 12000};
  std::vector<int16_t> pcm(12000);
  for (auto& v : pcm) v = (int16_t)(rng() % 2000 - 1000);
  size_t nf = 0;
  for (size_t c = 0; c + 1 < off.size(); c++) nf += tfo_frame_count((size_t)(off[c + 1] - off[c]));
  std::vector<int32_t> micro(2 * nf);
  std::vector<double> db(2 * nf);
  CHECK(tfo_fingerprint_batch(&T, pcm.data(), off.data(), 4, micro.data(), db.data(), 4) == nf);
  // searches on a random table with NULL rows
  const int32_t nclips = 50, nrows = 5000;
  std::vector<int32_t> m1(nrows), m2(nrows), clip(nrows), tie(nclips);
  for (int32_t r = 0; r < nrows; r++) {
    m1[r] = (rng() % 20 == 0) ? TFO_NULL : (int32_t)(rng() % 8000000) - 4000000;
    m2[r] = (rng() % 20 == 0) ? TFO_NULL : (int32_t)(rng() % 6000000) - 3000000;
    clip[r] = (int32_t)(rng() % nclips);
  }
  std::vector<std::string> us(nclips);
  std::vector<const char*> up(nclips);
  for (int32_t c = 0; c < nclips; c++) {
    char b[64];
    snprintf(b, sizeof b, "%08x-0000-4000-8000-%012x", (unsigned)c, (unsigned)rng());  /* sorts like c */
    us[c] = b;
    up[c] = us[c].c_str();
    tie[c] = c;
  }
  std::vector<int32_t> s1(nrows), s2(nrows), sc(nrows);
  CHECK(tfo_sort_rows(m1.data(), m2.data(), clip.data(), nrows, s1.data(), s2.data(), sc.data()) == nrows);
  const int32_t nq = 12;
  std::vector<int64_t> qoff(nq + 1, 0);
  for (int32_t q = 0; q < nq; q++) qoff[q + 1] = qoff[q] + (q % 5) * 7;
  std::vector<double> q1(qoff[nq] + 1), q2(qoff[nq] + 1);
  for (int64_t f = 0; f < qoff[nq]; f++) {
    q1[f] = (f % 9 == 0) ? INFINITY : (double)(rng() % 9000) / 1000.0 - 4.5;
    q2[f] = (f % 11 == 0) ? NAN : (double)(rng() % 7000) / 1000.0 - 3.5;
  }
  for (int coefs : {1, 2, 3})
    for (double tol : {0.001, 0.3, -1.0}) {
      std::vector<int32_t> w(nq), mc(nq), w2(nq), mc2(nq);
      CHECK(tfo_search_sorted_batch(s1.data(), s2.data(), sc.data(), nrows, tie.data(), nclips, q1.data(), q2.data(),
                                    qoff.data(), nq, coefs, tol, 1, 4, w.data(), mc.data(), 3) == 0);
      for (int mode = 0; mode < 3; mode++) {
        CHECK(tfo_search_boxes_batch(s1.data(), s2.data(), sc.data(), nrows, tie.data(), nclips, q1.data(), q2.data(),
                                     qoff.data(), nq, coefs, tol, 1, 4, w2.data(), mc2.data(), 3, mode) == 0);
        CHECK(w == w2 && mc == mc2);
      }
      for (int32_t q = 0; q < nq; q++) {
        int32_t ww, mm, fc;
        tfo_search(m1.data(), m2.data(), clip.data(), nrows, up.data(), nclips, q1.data() + qoff[q], q2.data() + qoff[q],
                   (int32_t)(qoff[q + 1] - qoff[q]), coefs, tol, 1, 4, &ww, &mm, &fc);
        CHECK(ww == w[q] && (ww < 0 || mm == mc[q]));
      }
    }
}

int main() {
  wav_tests();
  table_tests();
  oracle_tests();
  if (fails) {
    fprintf(stderr, "%d checks failed\n", fails);
    return 1;
  }
  printf("ok\n");
  return 0;
}
