// Test infrastructure: the nested walker's per-word UTF-8 check (kx_nested.h kxn_utf8 over the input bytes)
// against its byte-wise restatement (the generic kxn_utf8, the utf8.Valid rules protobuf-go applies to
// proto3 strings): every 3-byte sequence at several alignments around the 8-byte word boundary, as the
// whole string and with one byte more or less, then seeded random strings. Prints "tot=N bad=M".
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <initializer_list>
#include <random>
#include "kx_nested.h"

struct W {   // a byte source that is not a plain pointer: the generic, byte-wise kxn_utf8
  const uint8_t* p;
  uint8_t operator[](uint64_t i) const { return p[i]; }
  W operator+(uint64_t k) const { return W{p + k}; }
};

int main() {
  uint8_t buf[64];
  long bad = 0, tot = 0;
  for (int pre : {0, 6, 7}) {
    for (uint32_t v = 0; v < (1u << 24); v++) {
      memset(buf, 'a', sizeof buf);
      buf[pre] = v & 0xff;
      buf[pre + 1] = (v >> 8) & 0xff;
      buf[pre + 2] = v >> 16;
      for (int n : {pre + 2, pre + 3, pre + 4}) {
        const bool a = kxn_utf8((const uint8_t*)buf, (uint64_t)n, (const uint8_t*)buf);
        const bool b = kxn_utf8(W{buf}, (uint64_t)n, W{buf});
        tot++;
        if (a != b && bad++ < 5) printf("mismatch pre=%d n=%d v=%06x\n", pre, n, v);
      }
    }
  }
  std::mt19937_64 g(1);
  const uint8_t pool[] = {'a', 0xc2, 0xc3, 0xa9, 0xe4, 0xb8, 0xad, 0xf0, 0x9f, 0x98, 0x80, 0xed, 0xa0, 0x80, 0xc0,
                          0xc1, 0xf4, 0x8f, 0x90, 0xf5, 0xff, 0xbf, 0xe0, 0x9f, 0xef};
  for (long it = 0; it < 2000000; it++) {
    int n = (int)(g() % 48), off = (int)(g() % 12);
    for (int i = 0; i < 64; i++) buf[i] = (g() % 3 == 0) ? 'x' : pool[g() % sizeof(pool)];
    if (off + n > 64) n = 64 - off;
    const bool a = kxn_utf8((const uint8_t*)buf + off, (uint64_t)n, (const uint8_t*)buf);
    const bool b = kxn_utf8(W{buf + off}, (uint64_t)n, W{buf});
    tot++;
    if (a != b && bad++ < 10) printf("mismatch n=%d off=%d\n", n, off);
  }
  printf("tot=%ld bad=%ld\n", tot, bad);
  return bad != 0;
}
