// Host-only sanitizer run of the scalar drop-in (yustack_amd/csrc/yucsum_scalar.cpp,
// the code behind Checksum / ChecksumCombine / PseudoHeaderChecksum of
// checksum/checksum.go:4-35) and of the C++ mirror's header helpers
// (include/yustack/checksum.hpp), built by tests/test_cpp.py with
// -fsanitize=address,undefined. Buffers are exact-size heap allocations at every
// start alignment, so a read one byte past a packet is an ASan report; results
// are checked against the oracle (oracle/csum_oracle.c, the test-only checker).
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>
#include <vector>

#include "yucsum.h"

extern "C" {
uint16_t or_checksum(const uint8_t *buf, size_t len, uint16_t initial);
uint16_t or_checksum_combine(uint16_t a, uint16_t b);
uint16_t or_pseudo_header_checksum(uint32_t protocol, const uint8_t *src, size_t slen,
                                   const uint8_t *dst, size_t dlen);
}

static int fails = 0;
#define CHECK(c, ...)                  \
  do {                                 \
    if (!(c)) {                        \
      fprintf(stderr, __VA_ARGS__);    \
      fputc('\n', stderr);             \
      if (++fails > 10) exit(1);       \
    }                                  \
  } while (0)

int main() {
  std::mt19937_64 rng(20261017);
  // every length 0..600 at every start alignment 0..15, in an exact-size block
  for (size_t len = 0; len <= 600; ++len) {
    for (size_t a = 0; a < 16; ++a) {
      uint8_t *blk = (uint8_t *)malloc(a + len + 1);
      uint8_t *p = blk + a;
      for (size_t i = 0; i < len; ++i) p[i] = (uint8_t)rng();
      const uint16_t init = (uint16_t)rng();
      CHECK(yu_checksum(p, len, init) == or_checksum(p, len, init), "len %zu align %zu", len, a);
      free(blk);
    }
  }
  // random long buffers, past the 131072-byte uint32 wrap of the reference
  for (int it = 0; it < 12; ++it) {
    const size_t len = 131000 + (size_t)(rng() % 400000);
    std::vector<uint8_t> *v = new std::vector<uint8_t>(len);
    for (auto &b : *v) b = (uint8_t)(rng() & (it % 3 ? 0xFF : 0x00)) | (it % 3 == 2 ? 0xFF : 0);
    const uint16_t init = (uint16_t)rng();
    CHECK(yu_checksum(v->data(), len, init) == or_checksum(v->data(), len, init), "long %zu", len);
    delete v;
  }
  // all-0xFF at the wrap boundary lengths
  for (size_t len : {131070u, 131071u, 131072u, 131073u, 131074u, 262144u, 262145u}) {
    std::vector<uint8_t> v(len, 0xFF);
    CHECK(yu_checksum(v.data(), len, 0xFFFF) == or_checksum(v.data(), len, 0xFFFF), "ff %zu", len);
  }
  // NULL with length 0 (the cgo shim passes NULL for an empty slice)
  CHECK(yu_checksum(nullptr, 0, 0x1234) == or_checksum(nullptr, 0, 0x1234), "null");
  for (uint32_t a = 0; a < 65536; a += 7)
    for (uint32_t b = a & 0xFF; b < 65536; b += 4099)
      CHECK(yu_checksum_combine(a, b) == or_checksum_combine(a, b), "combine %u %u", a, b);
  // PseudoHeaderChecksum on exact-size address strings of 0..16 bytes
  for (int it = 0; it < 2000; ++it) {
    const size_t sl = rng() % 17, dl = rng() % 17;
    uint8_t *s = (uint8_t *)malloc(sl + 1), *d = (uint8_t *)malloc(dl + 1);
    for (size_t i = 0; i < sl; ++i) s[i] = (uint8_t)rng();
    for (size_t i = 0; i < dl; ++i) d[i] = (uint8_t)rng();
    const uint32_t proto = (uint32_t)(rng() % 256);
    CHECK(yu_pseudo_header_checksum(proto, s, sl, d, dl) == or_pseudo_header_checksum(proto, s, sl, d, dl),
          "pseudo %zu %zu", sl, dl);
    free(s);
    free(d);
  }
  for (int st : {YU_OK, YU_EINVAL, YU_ENODEV, YU_ENOMEM, YU_EHIP_BASE, YU_EHIP_BASE - 5, 7})
    CHECK(yu_strerror(st) != nullptr, "strerror %d", st);
  if (fails) return 1;
  printf("ok\n");
  return 0;
}
