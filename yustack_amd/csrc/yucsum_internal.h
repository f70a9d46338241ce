// yucsum_internal.h — library-internal entry points shared by the translation
// units of libyucsum.so. Not part of the C ABI (include/yucsum.h).
#ifndef YUCSUM_INTERNAL_H
#define YUCSUM_INTERNAL_H

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "yucsum.h"

// Protocol tables used by both the kernels and the host-side field writer, so
// the two cannot disagree on which bytes a mode owns.
namespace yu {

// Offset of the checksum field a single-field TX mode takes as zero
// (header/udp.go udpChecksum=6, header/tcp.go tcpChecksum=16,
//  header/ipv4.go ipChecksum=10, header/icmpv4.go checksum at 2); 0 otherwise.
__host__ __device__ inline uint32_t mode_field(int m) {
  switch (m) {
    case YU_MODE_UDP: return 6;
    case YU_MODE_TCP: return 16;
    case YU_MODE_IPV4: return 10;
    case YU_MODE_ICMP: return 2;
    default: return 0;
  }
}
__host__ __device__ inline bool mode_is_tx(int m) {
  return m == YU_MODE_UDP || m == YU_MODE_TCP || m == YU_MODE_IPV4 || m == YU_MODE_ICMP;
}
// Modes that may write in place (the single-field TX modes and TX_DATAGRAM).
__host__ __device__ inline bool mode_fills(int m) {
  return mode_is_tx(m) || m == YU_MODE_TX_DATAGRAM;
}
// Offset of the transport checksum field in a segment of IPv4 protocol
// `proto`, and the segment's minimum length (UDP 6/8, TCP 16/20, ICMP 2/4);
// 0 / 0 for other protocols.
__host__ __device__ inline uint32_t l4_field(uint32_t proto) {
  return proto == 17u ? 6u : (proto == 6u ? 16u : (proto == 1u ? 2u : 0u));
}
__host__ __device__ inline uint32_t l4_min(uint32_t proto) {
  return proto == 17u ? 8u : (proto == 6u ? 20u : (proto == 1u ? 4u : 0u));
}

// Measurement knobs (YU_RAGGED, YU_VARIANT, YU_NT, YU_FILL_WB, YU_RUNS,
// YU_BLOCKS_PER_CU, YU_SEG_SMALL_BLOCKS, YU_XCD, YU_HOST_COPY_THREADS,
// YU_HOST_DIRECT_MAX, and the fault injection YU_HOST_FAIL_ALLOC) force
// kernels, grids, cut-overs and failures for tools/ and the
// forced-kernel test runs. They are read only when the process also sets
// YU_TUNING=1, so a production process that inherits one of them keeps the
// library's own choices; when the gate is open, each knob that is set is named
// once on stderr. Returns the knob's value, or NULL (gate closed or unset).
inline const char *tuning_env(const char *name) {
  static const bool on = [] {
    const char *g = getenv("YU_TUNING");
    return g && g[0] == '1' && g[1] == '\0';
  }();
  if (!on) return nullptr;
  const char *v = getenv(name);
  if (v && *v) fprintf(stderr, "yucsum: tuning knob %s=%s (YU_TUNING=1)\n", name, v);
  return v;
}

}  // namespace yu

// Enqueue on `stream` a one-thread kernel that stores `value` to `flag` (a
// device view of coherent pinned host memory) with system-scope fences, so a
// host thread polling the flag sees it only after everything enqueued before
// it on the stream has completed. Returns a YU_* status.
__attribute__((visibility("hidden"))) int yu_internal_signal(uint32_t *flag, uint32_t value,
                                                       void *stream);

#endif  // YUCSUM_INTERNAL_H
