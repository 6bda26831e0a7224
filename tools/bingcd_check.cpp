// Host build of csrc/bingcd.hpp for tests/test_bingcd.py: reads "N len_m m_hex y_hex" lines
// (N = 8 or 12 32-bit limbs), prints y^-1 mod m as hex, one line each.
#include <cstdio>
#include <cstring>
#include <string>
#include <iostream>
#include "../kzg-batch-verification-scheme_amd/csrc/bingcd.hpp"

template <int N>
static void from_hex(const std::string& h, uint32_t (&x)[N]) {
  for (int i = 0; i < N; ++i) x[i] = 0;
  int bit = 0;
  for (int k = (int)h.size() - 1; k >= 0; --k, bit += 4) {
    const char c = h[k];
    const uint32_t d = c <= '9' ? c - '0' : (c | 32) - 'a' + 10;
    x[bit >> 5] |= d << (bit & 31);
  }
}
template <int N>
static void run(int len_m, const std::string& mh, const std::string& yh) {
  uint32_t m[N], y[N], out[N];
  from_hex<N>(mh, m);
  from_hex<N>(yh, y);
  kzgmi::BinGcd<N>::inv(y, m, len_m, out);
  for (int i = N - 1; i >= 0; --i) printf("%08x", out[i]);
  printf("\n");
}
int main() {
  int n, len;
  std::string mh, yh;
  while (std::cin >> n >> len >> mh >> yh) {
    if (n == 8) run<8>(len, mh, yh);
    else if (n == 12) run<12>(len, mh, yh);
    else return 2;
  }
  return 0;
}
