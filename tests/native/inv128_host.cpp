// Host driver for tests/test_inv128.py: reads hex field elements (one per line) from stdin and
// prints inv128::inverse of each (the device inversion's source, compiled for the host).
#include <cstdio>
#include <cstring>

#include "../../janus_amd/csrc/inv128.h"

int main() {
  char line[128];
  while (fgets(line, sizeof line, stdin)) {
    uint32_t x[4] = {0, 0, 0, 0}, y[4];
    const size_t n = strcspn(line, "\r\n");
    // parse up to 32 hex digits, most significant first
    for (size_t i = 0; i < n; ++i) {
      const char ch = line[i];
      const uint32_t v = (ch >= '0' && ch <= '9') ? (uint32_t)(ch - '0') : (uint32_t)((ch | 32) - 'a' + 10);
      for (int k = 3; k > 0; --k) x[k] = (x[k] << 4) | (x[k - 1] >> 28);
      x[0] = (x[0] << 4) | v;
    }
    inv128::inverse(x, y);
    printf("%08x%08x%08x%08x\n", y[3], y[2], y[1], y[0]);
  }
  return 0;
}
