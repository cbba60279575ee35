#define SV_LB_BITS 8
#define SV_HOST_FE51 1
#include "verify_core.h"
#include <cstdio>
#include <random>
int main() {
  std::mt19937_64 rng(1);
  int hist[300] = {0};
  const int N = 2000000;
  for (int i = 0; i < N; ++i) {
    uint32_t x[16];
    for (int k = 0; k < 16; ++k) x[k] = (uint32_t)rng();
    uint32_t h[8];
    sc_reduce512(h, x);
    sv_lat lat;
    sc_lattice_reduce(lat, h, false);
    hist[lat.bits]++;
  }
  int wh[70] = {0};
  for (int b = 0; b < 300; ++b) if (hist[b]) { int w = (b + 4) / 4; wh[w] += hist[b]; }
  for (int b = 120; b < 140; ++b) if (hist[b]) printf("bits %d: %.4f\n", b, hist[b] / (double)N);
  for (int w = 0; w < 70; ++w) if (wh[w]) printf("W %d: %.5f\n", w, wh[w] / (double)N);
  for (int b = 140; b < 300; ++b) if (hist[b]) printf("bits %d: %d\n", b, hist[b]);
}
