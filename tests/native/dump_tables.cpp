// Dumps the product's host-built DspTables + dense mel (asterisk-tiresias_amd/csrc/tfp_tables.cpp)
// as raw bytes for tests/test_tables.py.  usage: dump_tables <sample_rate> <out.bin>
#include <cstdio>
#include <cstdlib>
#include "../../asterisk-tiresias_amd/csrc/tfp_tables.hpp"
int main(int argc, char** argv) {
  static tfp::DspTables t;
  static float mel[tfp::kFilters][tfp::kBins];
  const int sr = atoi(argv[1]);
  if (!tfp::build_tables(sr, &t)) return 1;
  tfp::build_mel_dense(sr, mel);
  FILE* f = fopen(argv[2], "wb");
  fwrite(&t, sizeof t, 1, f);
  fwrite(mel, sizeof mel, 1, f);
  fclose(f);
  printf("%zu %zu\n", sizeof t, sizeof mel);
  return 0;
}
