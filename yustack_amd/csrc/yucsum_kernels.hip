// yucsum_kernels.hip — gfx950 (MI355X, CDNA4, wave64) kernels for yustack's
// per-packet Internet checksum, and the batched device entry points of
// include/yucsum.h.
//
// Semantics reproduced (reference paths relative to /root/reference):
//   Checksum                checksum/checksum.go:4-18
//   ChecksumCombine         checksum/checksum.go:32-35
//   PseudoHeaderChecksum    checksum/checksum.go:24-28
//   compositions            transport/udp/endpoint.go:164-187,
//                           transport/tcp/connect.go:556-586,
//                           network/ipv4/ipv4.go:80-97, network/ipv4/icmp.go:36-45,
//                           checker/checker.go:25-40,71-99
//
// Arithmetic. The reference accumulates big-endian 16-bit words in a uint32
// that wraps mod 2^32 and folds once. Addition mod 2^32 is order-free, so any
// split of the packet across lanes, summed in uint32, reproduces the
// reference accumulator bit for bit (including the wrap for RAW buffers
// > 131072 B). Per 32-bit dword loaded little-endian from HBM:
//   v_perm_b32  swaps the bytes of each 16-bit half when the packet starts at
//               an even address (so each half becomes the big-endian word the
//               reference adds; for odd-start packets the little-endian halves
//               already carry the right weights and the perm is the identity);
//   v_sad_u16   adds both 16-bit halves into the uint32 accumulator.
// Two VALU ops per 4 bytes: the kernel stays far below the VALU ceiling and is
// bound by HBM.
//
// Layout. Loads are 16-byte (global_load_dwordx4) at 16-byte aligned
// addresses. A packet [s, e) is covered by the aligned chunks from
// floor16(s). Dwords are included iff they overlap [s, e) (one unsigned
// compare each); the few bytes a dword-granular include gets wrong — the
// head bytes before an unaligned s, the tail bytes after an unaligned e, and
// in TX modes the checksum field that Encode() zeroes — are subtracted on a
// rare, divergent correction path that only the lanes holding them enter.
//
// Work mapping (wave64-first, not a warp tiling):
//   k_small<G, U>: uniform stride, packet span <= G*U*16 bytes. A wave holds
//     64/G packets per step; each group of G lanes loads its packet window in
//     U dwordx4 loads per lane (1 KiB per wave-instruction), reduces with
//     log2(G) cross-lane adds and its leader stores the uint16 result.
//   k_loop<U>: one wave per packet, looping over 64*U*16-byte windows. Used for
//     ragged (tun-style, any alignment) batches and uniform packets > 4 KiB.
//   Both are persistent grid-stride kernels sized to the CU count.
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>

#include "yucsum.h"

namespace {

constexpr uint32_t kSelSwap = 0x02030001u;  // bytes [1,0,3,2]: BE 16-bit halves
constexpr uint32_t kSelIdent = 0x03020100u; // bytes [0,1,2,3]

struct BatchArgs {
  const uint8_t *data;
  const uint64_t *offsets;  // ragged: n+1 offsets; nullptr: uniform
  const uint16_t *initial_arr;
  const uint8_t *addrs;
  uint16_t *out;
  uint8_t *fill;  // non-null: write the field into the packet (== data)
  uint64_t stride;
  uint64_t n;
  uint32_t len;
  uint32_t initial;
  int mode;
};

__host__ __device__ __forceinline__ bool mode_is_ipv4(int m) {
  return m == YU_MODE_IPV4 || m == YU_MODE_VERIFY_IPV4;
}
__host__ __device__ __forceinline__ bool mode_is_tx(int m) {
  return m == YU_MODE_UDP || m == YU_MODE_TCP || m == YU_MODE_IPV4 ||
         m == YU_MODE_ICMP;
}
__host__ __device__ __forceinline__ bool mode_has_pseudo(int m) {
  return m == YU_MODE_UDP || m == YU_MODE_TCP || m == YU_MODE_VERIFY_TCP ||
         m == YU_MODE_VERIFY_UDP;
}
__host__ __device__ __forceinline__ uint32_t mode_proto(int m) {
  return (m == YU_MODE_TCP || m == YU_MODE_VERIFY_TCP) ? 6u : 17u;
}
// Offset of the checksum field a TX mode takes as zero
// (header/udp.go udpChecksum=6, header/tcp.go tcpChecksum=16,
//  header/ipv4.go ipChecksum=10, header/icmpv4.go checksum at 2).
__host__ __device__ __forceinline__ uint32_t mode_field(int m) {
  switch (m) {
    case YU_MODE_UDP: return 6;
    case YU_MODE_TCP: return 16;
    case YU_MODE_IPV4: return 10;
    case YU_MODE_ICMP: return 2;
    default: return 0;
  }
}
__host__ __device__ __forceinline__ uint32_t min_len(int m) {
  switch (m) {
    case YU_MODE_UDP: return 8;    // UDPMinimumSize
    case YU_MODE_TCP: return 20;   // TCPMinimumSize
    case YU_MODE_ICMP: return 4;   // ICMPv4MinimumSize
    case YU_MODE_IPV4:
    case YU_MODE_VERIFY_IPV4: return 1;  // byte 0 holds IHL
    default: return 0;
  }
}

// ChecksumCombine(uint16(v), uint16(v>>16)) — checksum/checksum.go:17,32-35
__device__ __forceinline__ uint32_t fold32(uint32_t v) {
  uint32_t w = (v & 0xFFFFu) + (v >> 16);
  return (w + (w >> 16)) & 0xFFFFu;
}

__device__ __forceinline__ uint32_t sadperm(uint32_t x, uint32_t sel,
                                            uint32_t acc) {
  return __builtin_amdgcn_sad_u16(__builtin_amdgcn_perm(x, x, sel), 0u, acc);
}

// Bytes of the dword [d, d+4) that lie in [x0, x1) as a byte mask
// (rare path only).
__device__ __forceinline__ uint32_t range_mask(uint32_t d, uint32_t x0,
                                               uint32_t x1) {
  int64_t lo = (int64_t)x0 - (int64_t)d;
  int64_t hi = (int64_t)x1 - (int64_t)d;
  lo = lo < 0 ? 0 : (lo > 4 ? 4 : lo);
  hi = hi < 0 ? 0 : (hi > 4 ? 4 : hi);
  if (hi <= lo) return 0u;
  uint64_t m = ((1ull << (8 * hi)) - 1ull) ^ ((1ull << (8 * lo)) - 1ull);
  return (uint32_t)m;
}

__device__ __forceinline__ bool overlaps(uint32_t a0, uint32_t a1, uint32_t b0,
                                         uint32_t b1) {
  return b0 < b1 && b0 < a1 && a0 < b1;
}

// Packet geometry in window-relative byte coordinates (window base =
// floor16(packet start)).
struct Geom {
  uint32_t s;     // packet start (0..15)
  uint32_t e;     // end of the summed bytes
  uint32_t s4;    // floor4(s)
  uint32_t L4;    // e - s4: dword d (rel) included iff d - s4 < L4
  uint32_t sel;   // perm selector (parity of s)
  uint32_t h1;    // head junk [s4, h1=s)
  uint32_t t0, t1;  // tail junk [e, ceil4(e))
  uint32_t f0, f1;  // TX field [f0, f1) ∩ [s, e)
  bool junk;      // any junk range non-empty
};

__device__ __forceinline__ Geom make_geom(uint32_t s, uint32_t e, int mode) {
  Geom g;
  g.s = s;
  g.e = e;
  g.s4 = s & ~3u;
  g.L4 = e - g.s4;
  g.sel = (s & 1u) ? kSelIdent : kSelSwap;
  g.h1 = s;
  g.t0 = e;
  g.t1 = (e & 3u) ? ((e + 3u) & ~3u) : e;
  if (mode_is_tx(mode)) {
    uint32_t f0 = s + mode_field(mode);
    uint32_t f1 = f0 + 2u;
    f0 = f0 < e ? f0 : e;
    f1 = f1 < e ? f1 : e;
    g.f0 = f0;
    g.f1 = f1;
  } else {
    g.f0 = g.f1 = 0;
  }
  g.junk = (s & 3u) || (e & 3u) || (g.f0 < g.f1);
  return g;
}

// Accumulate one 16-byte chunk at window-relative offset cr.
__device__ __forceinline__ void sum_chunk(const uint4 &c, uint32_t cr,
                                          const Geom &g, uint32_t &acc) {
  const uint32_t r = cr - g.s4;
  const uint32_t x0 = (r < g.L4) ? c.x : 0u;
  const uint32_t x1 = (r + 4u < g.L4) ? c.y : 0u;
  const uint32_t x2 = (r + 8u < g.L4) ? c.z : 0u;
  const uint32_t x3 = (r + 12u < g.L4) ? c.w : 0u;
  acc = sadperm(x0, g.sel, acc);
  acc = sadperm(x1, g.sel, acc);
  acc = sadperm(x2, g.sel, acc);
  acc = sadperm(x3, g.sel, acc);
  if (g.junk) {
    const uint32_t ce = cr + 16u;
    if (overlaps(cr, ce, g.s4, g.h1) || overlaps(cr, ce, g.t0, g.t1) ||
        overlaps(cr, ce, g.f0, g.f1)) {
      uint32_t junk = 0;
      const uint32_t xs[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t d = cr + 4u * j;
        const uint32_t m = range_mask(d, g.s4, g.h1) |
                           range_mask(d, g.t0, g.t1) |
                           range_mask(d, g.f0, g.f1);
        junk = sadperm(xs[j] & m, g.sel, junk);
      }
      acc -= junk;
    }
  }
}

// Byte at window-relative offset s (0..15) of chunk 0.
__device__ __forceinline__ uint32_t byte_of(const uint4 &c, uint32_t s) {
  const uint32_t di = s >> 2;
  const uint32_t w = di == 0 ? c.x : (di == 1 ? c.y : (di == 2 ? c.z : c.w));
  return (w >> (8u * (s & 3u))) & 0xFFu;
}

template <int G>
__device__ __forceinline__ uint32_t group_sum(uint32_t v) {
#pragma unroll
  for (int o = G / 2; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Per-packet epilogue: add the non-payload terms of the reference
// composition, fold, complement, store (and optionally set the field).
__device__ __forceinline__ void finish_packet(const BatchArgs &A, uint64_t p,
                                              uint32_t v, uint64_t len,
                                              uint8_t *pkt, uint32_t hdr_end) {
  const int mode = A.mode;
  if (mode == YU_MODE_RAW) {
    v += A.initial_arr ? (uint32_t)A.initial_arr[p] : A.initial;
  } else if (mode_has_pseudo(mode)) {
    uint32_t ph;
    if (A.addrs) {
      // PseudoHeaderChecksum(proto, src, dst): src/dst big-endian words + proto
      const uint32_t *a = (const uint32_t *)(A.addrs + 8 * p);
      ph = sadperm(a[0], kSelSwap, 0u);
      ph = sadperm(a[1], kSelSwap, ph);
      ph += mode_proto(mode);
    } else {
      ph = A.initial_arr ? (uint32_t)A.initial_arr[p] : A.initial;
    }
    // + Checksum(BE16(uint16(length))) — header/udp.go:70-72, tcp.go:168-170
    v += ph + (uint32_t)(len & 0xFFFFu);
  }
  uint32_t r = fold32(v);
  if (mode_is_tx(mode)) r = (~r) & 0xFFFFu;
  if (A.out) A.out[p] = (uint16_t)r;
  if (A.fill && mode_is_tx(mode)) {
    const uint32_t f = mode_field(mode);
    if (f + 2u <= hdr_end) {
      pkt[f] = (uint8_t)(r >> 8);  // binary.BigEndian.PutUint16
      pkt[f + 1] = (uint8_t)r;
    }
  }
}

// ---------------------------------------------------------------------
// k_small<G, U>: uniform stride, whole packet window in one step.
// ---------------------------------------------------------------------
template <int G, int U>
__global__ __launch_bounds__(256) void k_small(BatchArgs A) {
  constexpr int GPW = 64 / G;
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t gl = lane & (G - 1);
  const uint32_t gw = lane / G;
  const uint64_t wave = (uint64_t)blockIdx.x * (blockDim.x >> 6) +
                        (uint64_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t nwave = (uint64_t)gridDim.x * (blockDim.x >> 6);
  const int mode = A.mode;
  const bool ipv4 = mode_is_ipv4(mode);

  for (uint64_t pb = wave * GPW; pb < A.n; pb += nwave * GPW) {
    const uint64_t p = pb + gw;
    const bool active = p < A.n;
    const uint64_t soff = active ? p * A.stride : 0;
    const uintptr_t sabs = (uintptr_t)A.data + soff;
    const uint8_t *wbase = (const uint8_t *)(sabs & ~(uintptr_t)15);
    const uint32_t s = (uint32_t)(sabs & 15u);
    const uint32_t len = active ? A.len : 0u;
    const uint32_t eload = s + (ipv4 ? (len < 60u ? len : 60u) : len);

    uint4 c[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t cr = 16u * (gl + (uint32_t)u * G);
      if (cr < eload)
        c[u] = *(const uint4 *)(wbase + cr);
      else
        c[u] = make_uint4(0u, 0u, 0u, 0u);
    }

    uint32_t e = s + len;
    if (ipv4) {
      // HeaderLength() = (b[0] & 0xf) * 4 — header/ipv4.go:91-93
      uint32_t b0 = (gl == 0 && len > 0) ? byte_of(c[0], s) : 0u;
      b0 = __shfl(b0, (int)(lane & ~(uint32_t)(G - 1)), 64);
      const uint32_t hl = (b0 & 0xFu) * 4u;
      e = s + (len < hl ? len : hl);
    }
    const Geom g = make_geom(s, e, mode);

    uint32_t acc = 0;
#pragma unroll
    for (int u = 0; u < U; ++u)
      sum_chunk(c[u], 16u * (gl + (uint32_t)u * G), g, acc);

    acc = group_sum<G>(acc);
    if (active && gl == 0)
      finish_packet(A, p, acc, len, A.fill ? A.fill + soff : nullptr, e - s);
  }
}

// ---------------------------------------------------------------------
// k_loop<U>: one wave per packet, 64*U*16-byte windows (ragged / large).
// ---------------------------------------------------------------------
template <int U>
__global__ __launch_bounds__(256) void k_loop(BatchArgs A) {
  constexpr uint32_t W = 64u * 16u * U;
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t wave = (uint64_t)blockIdx.x * (blockDim.x >> 6) +
                        (uint64_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t nwave = (uint64_t)gridDim.x * (blockDim.x >> 6);
  const int mode = A.mode;
  const bool ipv4 = mode_is_ipv4(mode);

  for (uint64_t p = wave; p < A.n; p += nwave) {
    uint64_t soff, len;
    if (A.offsets) {
      soff = A.offsets[p];
      len = A.offsets[p + 1] - soff;
    } else {
      soff = p * A.stride;
      len = A.len;
    }
    const uintptr_t sabs = (uintptr_t)A.data + soff;
    const uint8_t *wbase = (const uint8_t *)(sabs & ~(uintptr_t)15);
    const uint32_t s = (uint32_t)(sabs & 15u);
    const uint32_t len32 = (uint32_t)len;
    const uint32_t eload = s + (ipv4 ? (len32 < 60u ? len32 : 60u) : len32);

    uint32_t e = s + len32;
    Geom g = make_geom(s, e, mode);
    uint32_t acc = 0;
    for (uint32_t wb = 0; wb < eload; wb += W) {
      uint4 c[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t cr = wb + 16u * (lane + 64u * (uint32_t)u);
        if (cr < eload)
          c[u] = *(const uint4 *)(wbase + cr);
        else
          c[u] = make_uint4(0u, 0u, 0u, 0u);
      }
      if (ipv4) {  // single window (eload <= 75 < W)
        uint32_t b0 = (lane == 0 && len32 > 0) ? byte_of(c[0], s) : 0u;
        b0 = __shfl(b0, 0, 64);
        const uint32_t hl = (b0 & 0xFu) * 4u;
        e = s + (len32 < hl ? len32 : hl);
        g = make_geom(s, e, mode);
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
        sum_chunk(c[u], wb + 16u * (lane + 64u * (uint32_t)u), g, acc);
    }
    acc = group_sum<64>(acc);
    if (lane == 0)
      finish_packet(A, p, acc, len, A.fill ? A.fill + soff : nullptr, e - s);
  }
}

// ---------------------------------------------------------------------
// Host side: variant selection and launch.
// ---------------------------------------------------------------------
typedef void (*KernelFn)(BatchArgs);

struct Variant {
  const char *name;
  uint32_t window;  // bytes covered per packet step (0 = loop kernel)
  KernelFn fn;
  uint32_t packets_per_wave;
};

const Variant kSmall[] = {
    {"k_small<4,1>", 64, k_small<4, 1>, 16},
    {"k_small<8,1>", 128, k_small<8, 1>, 8},
    {"k_small<16,1>", 256, k_small<16, 1>, 4},
    {"k_small<32,1>", 512, k_small<32, 1>, 2},
    {"k_small<64,1>", 1024, k_small<64, 1>, 1},
    {"k_small<32,3>", 1536, k_small<32, 3>, 2},
    {"k_small<64,2>", 2048, k_small<64, 2>, 1},
    {"k_small<64,3>", 3072, k_small<64, 3>, 1},
    {"k_small<64,4>", 4096, k_small<64, 4>, 1},
};
const Variant kLoop = {"k_loop<4>", 0, k_loop<4>, 1};

uint64_t gcd64(uint64_t a, uint64_t b) {
  while (b) {
    uint64_t t = a % b;
    a = b;
    b = t;
  }
  return a;
}

// Largest (start & 15) over the batch's packet starts.
uint32_t max_misalign(uint64_t base_mod16, uint64_t stride, uint64_t n) {
  if (n <= 1) return (uint32_t)(base_mod16 & 15u);
  uint64_t g = gcd64(stride & 15u ? (stride & 15u) : 16u, 16u);
  return (uint32_t)((base_mod16 % g) + (16u - g));
}

const Variant &pick_uniform(uint64_t base_mod16, uint64_t stride, uint32_t len,
                            uint64_t n, int mode) {
  uint64_t need = mode_is_ipv4(mode) ? (len < 60u ? len : 60u) : len;
  uint64_t span = need + max_misalign(base_mod16, stride, n);
  for (const Variant &v : kSmall)
    if (span <= v.window) return v;
  return kLoop;
}

std::atomic<int> g_cu_count[64];

int cu_count(int dev) {
  if (dev < 0 || dev >= 64) return 256;
  int c = g_cu_count[dev].load(std::memory_order_relaxed);
  if (c > 0) return c;
  if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) !=
          hipSuccess ||
      c <= 0)
    c = 256;
  g_cu_count[dev].store(c, std::memory_order_relaxed);
  return c;
}

int blocks_per_cu() {
  static int v = [] {
    const char *s = getenv("YU_BLOCKS_PER_CU");
    int x = s ? atoi(s) : 0;
    return (x >= 1 && x <= 32) ? x : 8;
  }();
  return v;
}

int hip_status(hipError_t e) {
  if (e == hipSuccess) return YU_OK;
  if (e == hipErrorNoDevice || e == hipErrorInvalidDevice) return YU_ENODEV;
  if (e == hipErrorOutOfMemory) return YU_ENOMEM;
  return YU_EHIP_BASE - (int)e;
}

int launch(const Variant &v, const BatchArgs &A, hipStream_t stream) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return hip_status(e);
  const uint64_t waves_per_block = 4;
  uint64_t waves = (A.n + v.packets_per_wave - 1) / v.packets_per_wave;
  uint64_t blocks = (waves + waves_per_block - 1) / waves_per_block;
  uint64_t cap = (uint64_t)cu_count(dev) * (uint64_t)blocks_per_cu();
  if (blocks > cap) blocks = cap;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(v.fn, dim3((unsigned)blocks), dim3(256), 0, stream, A);
  return hip_status(hipGetLastError());
}

bool aligned(const void *p, uintptr_t a) {
  return ((uintptr_t)p & (a - 1)) == 0;
}

int check_common(int mode, const uint16_t *initial_arr, const uint8_t *addrs,
                 const uint16_t *out, bool fill) {
  if (mode < 0 || mode >= YU_MODE_COUNT) return YU_EINVAL;
  if (!out && !fill) return YU_EINVAL;
  if (fill && !mode_is_tx(mode)) return YU_EINVAL;
  if (initial_arr && !aligned(initial_arr, 2)) return YU_EINVAL;
  if (addrs && !aligned(addrs, 4)) return YU_EINVAL;
  if (out && !aligned(out, 2)) return YU_EINVAL;
  return YU_OK;
}

int batch_uniform(const uint8_t *data, uint8_t *fill, uint64_t stride,
                  uint32_t len, uint64_t n, int mode,
                  const uint16_t *initial_arr, uint16_t initial,
                  const uint8_t *addrs, uint16_t *out, void *stream) {
  int rc = check_common(mode, initial_arr, addrs, out, fill != nullptr);
  if (rc) return rc;
  if (n == 0) return YU_OK;
  if (!data && len) return YU_EINVAL;
  if (mode != YU_MODE_RAW && len > YU_MAX_TRANSPORT_LEN) return YU_EINVAL;
  if (len < min_len(mode)) return YU_EINVAL;
  if (len >= 0xFFFFFFF0u) return YU_EINVAL;
  BatchArgs A;
  A.data = data;
  A.offsets = nullptr;
  A.initial_arr = initial_arr;
  A.addrs = addrs;
  A.out = out;
  A.fill = fill;
  A.stride = stride;
  A.n = n;
  A.len = len;
  A.initial = initial;
  A.mode = mode;
  const Variant &v = pick_uniform((uintptr_t)data & 15u, stride, len, n, mode);
  return launch(v, A, (hipStream_t)stream);
}

int batch_ragged(const uint8_t *data, uint8_t *fill, const uint64_t *offsets,
                 uint64_t n, int mode, const uint16_t *initial_arr,
                 uint16_t initial, const uint8_t *addrs, uint16_t *out,
                 void *stream) {
  int rc = check_common(mode, initial_arr, addrs, out, fill != nullptr);
  if (rc) return rc;
  if (n == 0) return YU_OK;
  if (!offsets || !aligned(offsets, 8) || !data) return YU_EINVAL;
  BatchArgs A;
  A.data = data;
  A.offsets = offsets;
  A.initial_arr = initial_arr;
  A.addrs = addrs;
  A.out = out;
  A.fill = fill;
  A.stride = 0;
  A.n = n;
  A.len = 0;
  A.initial = initial;
  A.mode = mode;
  return launch(kLoop, A, (hipStream_t)stream);
}

}  // namespace

extern "C" {

int yu_csum_batch_uniform(const uint8_t *data, uint64_t stride, uint32_t len,
                          uint64_t n, int mode, const uint16_t *initial_arr,
                          uint16_t initial, const uint8_t *addrs,
                          uint16_t *out, void *stream) {
  return batch_uniform(data, nullptr, stride, len, n, mode, initial_arr,
                       initial, addrs, out, stream);
}

int yu_csum_batch_ragged(const uint8_t *data, const uint64_t *offsets,
                         uint64_t n, int mode, const uint16_t *initial_arr,
                         uint16_t initial, const uint8_t *addrs,
                         uint16_t *out, void *stream) {
  return batch_ragged(data, nullptr, offsets, n, mode, initial_arr, initial,
                      addrs, out, stream);
}

int yu_csum_fill_uniform(uint8_t *data, uint64_t stride, uint32_t len,
                         uint64_t n, int mode, const uint16_t *initial_arr,
                         uint16_t initial, const uint8_t *addrs, uint16_t *out,
                         void *stream) {
  if (n > 1 && stride < len) return YU_EINVAL;  // overlapping packets
  return batch_uniform(data, data, stride, len, n, mode, initial_arr, initial,
                       addrs, out, stream);
}

int yu_csum_fill_ragged(uint8_t *data, const uint64_t *offsets, uint64_t n,
                        int mode, const uint16_t *initial_arr,
                        uint16_t initial, const uint8_t *addrs, uint16_t *out,
                        void *stream) {
  return batch_ragged(data, data, offsets, n, mode, initial_arr, initial,
                      addrs, out, stream);
}

const char *yu_uniform_variant(uint64_t stride, uint32_t len, int mode,
                               uint64_t data_align16) {
  return pick_uniform(data_align16 & 15u, stride, len, 2, mode).name;
}

int yu_device_count(void) {
  int c = 0;
  if (hipGetDeviceCount(&c) != hipSuccess) return 0;
  return c < 0 ? 0 : c;
}

}  // extern "C"
