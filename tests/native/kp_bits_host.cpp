// Host driver for tests/test_keccak_pair.py: per input line (a 64-bit word in hex) prints
// kp_unzip's halves, kp_half(w, 0/1), kp_zip(e, o) and kp_spread(e, 0) | kp_spread(o, 1).
#include <stdio.h>
#include <inttypes.h>
#include "../../janus_amd/csrc/kp_bits.h"

int main() {
  unsigned long long w;
  while (scanf("%llx", &w) == 1) {
    uint32_t e, o;
    kp_unzip(w, e, o);
    printf("%08x %08x %08x %08x %016llx %016llx\n", e, o, kp_half(w, 0), kp_half(w, 1),
           (unsigned long long)kp_zip(e, o),
           (unsigned long long)(kp_spread(e, 0) | kp_spread(o, 1)));
  }
  return 0;
}
