// yucsum_scalar.cpp — the Go-signature scalar entry points of include/yucsum.h.
//
// These back the cgo shim that replaces package `checksum`
// (/root/reference/checksum/checksum.go) so that header/ipv4.go:177-179,
// header/tcp.go:165-173, header/udp.go:67-75, types/route.go:90-92,
// transport/udp/endpoint.go:175, transport/tcp/connect.go:314,580,
// network/ipv4/icmp.go:42 and checker/checker.go:32,84-88 run unchanged.
// One call = one buffer on the calling host thread (a GPU round trip per
// call would cost far more than the 20–1500-byte sum itself); the GPU path
// is the batched API in yucsum_kernels.hip.
//
// Exactness: the reference adds big-endian words into a uint32 that wraps
// mod 2^32. With H = sum of bytes at even offsets and L = sum of bytes at odd
// offsets (the odd trailing byte is at an even offset, i.e. the reference's
// `buf[l] << 8`), the reference accumulator is initial + 256*H + L mod 2^32.
// H and L are computed exactly with 8-byte SWAR lanes (each 16-bit lane
// absorbs <= 256 additions of 255 before it is flushed), so the result is
// bit-identical for every length, including the > 131072-byte wrap.
#include <stdint.h>
#include <string.h>

#include "yucsum.h"

static_assert(__BYTE_ORDER__ == __ORDER_LITTLE_ENDIAN__,
              "SWAR lanes assume a little-endian host");

namespace {

inline uint64_t load64(const uint8_t *p) {
  uint64_t q;
  memcpy(&q, p, 8);
  return q;
}

inline uint64_t hsum16x4(uint64_t x) {
  return (x & 0xFFFF) + ((x >> 16) & 0xFFFF) + ((x >> 32) & 0xFFFF) + (x >> 48);
}

}  // namespace

extern "C" {

uint16_t yu_checksum_combine(uint16_t a, uint16_t b) {
  uint32_t v = (uint32_t)a + (uint32_t)b;
  return (uint16_t)(v + (v >> 16));
}

uint16_t yu_checksum(const uint8_t *buf, size_t len, uint16_t initial) {
  const uint64_t kLanes = 0x00FF00FF00FF00FFull;
  uint64_t H = 0, L = 0;
  size_t i = 0;
  while (len - i >= 8) {
    size_t blocks = (len - i) / 8;
    if (blocks > 256) blocks = 256;
    uint64_t he = 0, lo = 0;
    for (size_t k = 0; k < blocks; ++k, i += 8) {
      const uint64_t q = load64(buf + i);
      he += q & kLanes;         // bytes at even offsets (LE lanes 0,2,4,6)
      lo += (q >> 8) & kLanes;  // bytes at odd offsets
    }
    H += hsum16x4(he);
    L += hsum16x4(lo);
  }
  for (; i + 1 < len; i += 2) {
    H += buf[i];
    L += buf[i + 1];
  }
  if (i < len) H += buf[i];  // odd trailing byte: high byte of a final word
  const uint32_t v = (uint32_t)initial + (uint32_t)(H << 8) + (uint32_t)L;
  return yu_checksum_combine((uint16_t)v, (uint16_t)(v >> 16));
}

uint16_t yu_pseudo_header_checksum(uint32_t protocol, const uint8_t *src_addr,
                                   size_t src_len, const uint8_t *dst_addr,
                                   size_t dst_len) {
  uint16_t xsum = yu_checksum(src_addr, src_len, 0);
  xsum = yu_checksum(dst_addr, dst_len, xsum);
  const uint8_t proto[2] = {0, (uint8_t)protocol};
  return yu_checksum(proto, 2, xsum);
}

int yu_abi_version(void) { return YUCSUM_ABI_VERSION; }

const char *yu_strerror(int status) {
  switch (status) {
    case YU_OK: return "ok";
    case YU_EINVAL: return "invalid argument";
    case YU_ENODEV: return "no HIP device";
    case YU_ENOMEM: return "out of memory";
    default: return status <= YU_EHIP_BASE ? "HIP runtime error" : "unknown error";
  }
}

}  // extern "C"
