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
// Arithmetic. The reference adds big-endian 16-bit words into a uint32 that
// wraps mod 2^32 and folds once (ChecksumCombine). Two exact formulations:
//
//  * LE (default). Sum the little-endian 16-bit halves of every 32-bit word
//    with v_sad_u16 — ONE VALU op per 4 bytes — into a uint32 S_LE. Swapping
//    the bytes of a 16-bit word multiplies it by 256 modulo 65535, so the
//    big-endian sum S_BE is congruent to swap16(fold(S_LE)) when the packet
//    starts at an even address (to fold(S_LE) when it starts at an odd one),
//    and S_BE is 0 exactly when S_LE is. The reference's result depends on
//    S_BE only through that residue and zero-ness as long as its uint32 does
//    not wrap, i.e. for buffers <= 131072 bytes: every transport/IPv4/ICMP
//    packet and every RAW packet up to that size.
//  * BE (RAW packets that may exceed 131072 bytes). v_perm_b32 turns each
//    16-bit half into the big-endian word first; the uint32 sum then equals
//    the reference's accumulator bit for bit, wrap included (addition mod
//    2^32 is order-free).
//
// Layout. A packet [s, e) is read through 16-byte loads (buffer_load_dwordx4)
// from a window that starts at floor4(s): every chunk but the last lies
// inside the packet and is summed unmasked; the last chunk's dwords are kept
// iff they start before e. The few bytes this gets wrong — up to 3 bytes
// before an unaligned s, up to 3 after an unaligned e, and in TX modes the
// two checksum-field bytes that Encode() zeroes — sit in at most four known
// dwords; the group leader gathers them from the registers of the lanes
// holding them (one cross-lane read each) and subtracts their masked bytes.
// No byte is loaded twice.
//
// Loads go through buffer descriptors based at wave-uniform addresses: a lane
// that must not load passes an out-of-range offset and gets zeros without a
// memory access, so no load sits in an exec-masked block and the compiler's
// vmcnt bookkeeping stays exact. That lets the kernels keep the next step's
// loads in flight while the current step is summed (software pipelining).
//
// Work mapping (wave64-first, not a warp tiling). Which kernel a batch gets
// depends on its layout, mode, packet size and count (pick_uniform /
// pick_ragged below, each cut-over measured):
//   k_lane<U>: dense uniform 4-aligned packets up to 112 bytes (configs 2 and
//     8): 64 whole strides per wave step parked in LDS, one lane per packet
//     summing it from there.
//   k_tiny<G>: uniform 4-aligned packets <= 16G bytes that k_lane does not take
//     (113..128 bytes, sparse small ones): a wave step covers 64 packets, each
//     load instruction one contiguous KiB, and a cross-lane transpose lets
//     every lane finish one packet.
//   k_small<G, U>: uniform stride, packet span <= G*U*16 bytes (705..3072 and
//     sparse ones). A wave holds 64/G packets per step; each group of G lanes
//     loads its packet window in U dwordx4 loads per lane, reduces with log2(G)
//     DPP adds and its last lane finishes the packet (config 3: k_small<16,6>).
//   k_seg<U, NT, K, CH>: ragged batches of more than 4096 packets, VERIFY_RX,
//     and dense uniform packets of other sizes: a segmented sum over the byte
//     stream of CH consecutive packets per wave (64, or 16 below 64K packets),
//     U KiB tiles, packet sums as prefix differences (config 4, tun RX). Its
//     TXW kind writes ragged TX batches in place, storing the fields of each
//     chunk's last tile as whole 128-byte lines.
//   k_hdr<NT>: the IPv4 header-only modes (<= 60 bytes of each packet), uniform
//     and ragged: one lane per packet, 32-byte reads.
//   k_loop<U, BE> / k_loop_rx<U>: one wave per packet, for ragged bursts of up
//     to 4096 packets and for few or sparse uniform packets > 4 KiB.
//   k_rag<G, U>: the first ragged kernel, kept as a measurement alternative.
//   All are grid-stride kernels; the grid is sized per CU and over-subscribed
//   (see blocks_per_cu), except that k_seg narrows it for small packets
//   (seg_waves).
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <type_traits>

#include "yucsum.h"
#include "yucsum_internal.h"

namespace {

constexpr uint32_t kSelSwap = 0x02030001u;  // bytes [1,0,3,2]: BE 16-bit halves
constexpr uint32_t kSelIdent = 0x03020100u; // bytes [0,1,2,3]
constexpr uint32_t kLEMax = 131072u;        // longest packet the LE sum covers

struct BatchArgs {
  const uint8_t *data;
  const uint64_t *offsets;  // ragged: n+1 offsets; nullptr: uniform
  const uint16_t *initial_arr;
  const uint8_t *addrs;
  uint16_t *out;
  uint8_t *fill;  // non-null: write the field into the packet (== data)
  uint64_t stride;
  uint64_t n;
  uint64_t end;   // one past the batch's last byte (uniform); ragged: 0
  uint32_t len;
  uint32_t initial;
  uint32_t uf;    // k_small: steps u < uf hold only full chunks
  uint32_t xcd;   // 1: XCD-aware block order (grid_wave)
  uint32_t small_waves;  // k_seg: waves that work on small-packet batches (seg_waves)
  int mode;
};

__host__ __device__ __forceinline__ bool mode_is_ipv4(int m) {
  return m == YU_MODE_IPV4 || m == YU_MODE_VERIFY_IPV4;
}
using yu::l4_field;  // protocol tables shared with the host writer (yucsum_internal.h)
using yu::l4_min;
using yu::mode_field;
using yu::mode_fills;
using yu::mode_is_tx;
__host__ __device__ __forceinline__ bool mode_has_pseudo(int m) {
  return m == YU_MODE_UDP || m == YU_MODE_TCP || m == YU_MODE_VERIFY_TCP ||
         m == YU_MODE_VERIFY_UDP;
}
__host__ __device__ __forceinline__ uint32_t mode_proto(int m) {
  return (m == YU_MODE_TCP || m == YU_MODE_VERIFY_TCP) ? 6u : 17u;
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

__device__ __forceinline__ uint32_t sad(uint32_t x, uint32_t acc) {
  return __builtin_amdgcn_sad_u16(x, 0u, acc);
}

__device__ __forceinline__ uint32_t sadperm(uint32_t x, uint32_t sel,
                                            uint32_t acc) {
  return __builtin_amdgcn_sad_u16(__builtin_amdgcn_perm(x, x, sel), 0u, acc);
}

template <bool BE>
__device__ __forceinline__ uint32_t add_word(uint32_t x, uint32_t sel,
                                             uint32_t acc) {
  return BE ? sadperm(x, sel, acc) : sad(x, acc);
}

// Residue of the packet's big-endian word sum, from the LE sum of a packet
// starting at an address of parity `odd` (see the header comment).
__device__ __forceinline__ uint32_t le_to_be(uint32_t s_le, uint32_t odd) {
  const uint32_t r = fold32(s_le);
  return odd ? r : (((r & 0xFFu) << 8) | (r >> 8));
}

// Sum over each aligned group of G lanes; the total lands in the group's
// LAST lane (lane % G == G-1). DPP row shifts inside 16-lane rows, then
// row_bcast15/31 across rows — VALU only, no LDS traffic.
template <int G>
__device__ __forceinline__ uint32_t group_total(uint32_t v) {
  static_assert(G >= 1 && G <= 64 && (G & (G - 1)) == 0, "G must be a power of two");
  if (G >= 2) v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true);  // row_shr:1
  if (G >= 4) v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true);  // row_shr:2
  if (G >= 8) v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, true);  // row_shr:4
  if (G >= 16) v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, true); // row_shr:8
  if (G >= 32) v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false); // row_bcast:15
  if (G >= 64) v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false); // row_bcast:31
  return v;
}

// OR over the whole wave, in every lane (the same DPP steps as group_total<64>,
// then lane 63's value handed round in a VGPR: the caller is short of SGPRs).
__device__ __forceinline__ uint32_t wave_or(uint32_t v) {
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true);   // row_shr:1
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true);   // row_shr:2
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, true);   // row_shr:4
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, true);   // row_shr:8
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return (uint32_t)__shfl((int)v, 63, 64);
}

// This wave's index in the grid's packet order. Blocks are dealt round-robin
// over the 8 XCDs (blocks b and b+8 share an L2), so with xcd set the order is
// swizzled to give each XCD a contiguous run of logical blocks: the one
// 128-byte line two neighbouring packets (or 64-packet chunks) share is then
// fetched by a single L2, at about the same time, instead of by two. Bijective
// for any grid size (XCDs x < n%8 hold one block more). Speed only: no
// correctness depends on where a block runs. Off by default (see use_xcd).
__device__ __forceinline__ uint64_t grid_wave(uint32_t xcd) {
  const uint32_t b = blockIdx.x, n = gridDim.x;
  uint32_t lb = b;
  if (xcd) {
    const uint32_t x = b & 7u, i = b >> 3, q = n >> 3, r = n & 7u;
    lb = (x < r ? x * (q + 1u) : r * (q + 1u) + (x - r) * q) + i;
  }
  return (uint64_t)lb * (blockDim.x >> 6) +
         (uint64_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// Wave-uniform 64-bit value (only for values uniform by construction): puts
// buffer bases in SGPRs so no waterfall loop is generated.
__device__ __forceinline__ uint64_t uniform64(uint64_t x) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)x);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(x >> 32));
  return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, uint32_t l) {
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l) << 32) |
         (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
}

// Out-of-range offset: the load returns zeros and touches no memory.
constexpr uint32_t kOOB = 0x80000000u;

// Descriptor over [base, min(ceil4(end), base + 2 GiB)). The range check is
// per dword (a dword reaching past num_records reads as 0), so the extent is
// rounded up to the dword holding the batch's last byte: loads never leave
// that dword, let alone the allocation.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_at(uint64_t base,
                                                          uint64_t end) {
  end = (end + 3u) & ~3ull;
  const uint64_t n = end > base ? end - base : 0;
  return __builtin_amdgcn_make_buffer_rsrc((void *)base, (short)0,
                                           (int)(n < kOOB ? n : kOOB), 0x00020000);
}

// Load policy. Packet bytes are read once, and non-temporal (nt, aux bit 1)
// loads stream them fastest, but an nt line does not stay in L2, so the line
// two neighbouring packets share is fetched twice. NT = 0: plain loads;
// 1: all nt; 2 (default): nt except the first and last step of a window,
// which hold the shared lines.
__device__ __forceinline__ uint4 bld16(__amdgpu_buffer_rsrc_t r, uint32_t off,
                                       bool nt) {
  const u32x4 t = nt ? __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 2)
                     : __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0);
  return make_uint4(t.x, t.y, t.z, t.w);
}

template <int NT>
__device__ __forceinline__ constexpr bool nt_step(int u, int U) {
  return NT == 1 || (NT == 2 && u != 0 && u != U - 1);
}

// ---------------------------------------------------------------------
// Junk: bytes of dwords the dword-granular sum includes but the reference
// does not, other than the unaligned tail (masked in sum_masked). Window
// coordinates (window base = floor4(packet start)); sh = start & 3; E = sh +
// summed length. Item 0: the head bytes [0, sh) of dword 0; items 1/2: the
// TX checksum field [sh+f, sh+f+2) (Encode writes 0 there), which may
// straddle two dwords. All lie in the window's first 24 bytes, i.e. in chunk
// 0 or 1 of step 0, and are read from the registers of the lanes holding
// them — never with an extra load.
// ---------------------------------------------------------------------
struct Junk {
  uint32_t off[3];   // window-relative dword offsets
  uint32_t mask[3];  // bytes to subtract (0 when the item is absent)
};

__device__ __forceinline__ Junk make_junk(uint32_t sh, uint32_t E, int mode) {
  Junk j;
  j.off[0] = 0u;
  j.mask[0] = (1u << (8u * sh)) - 1u;  // 0 for sh == 0
  const uint32_t f = mode_field(mode);
  const bool fld = mode_is_tx(mode) && sh + f + 2u <= E;
  const uint32_t fr = sh + f;
  const uint32_t fb = fr & 3u;
  j.off[1] = fr & ~3u;
  j.mask[1] = !fld ? 0u : (fb == 3u ? 0xFF000000u : (0xFFFFu << (8u * fb)));
  j.off[2] = (fr & ~3u) + 4u;
  j.mask[2] = (fld && fb == 3u) ? 0xFFu : 0u;
  return j;
}

__device__ __forceinline__ uint32_t pick_dword(const uint4 &c, uint32_t q) {
  return q == 0 ? c.x : (q == 1 ? c.y : (q == 2 ? c.z : c.w));
}

// Junk dwords of the group whose first lane is `gbase` (G = 1 << LG lanes;
// chunk k = off/16 is held by lane gbase + k in step 0; c0 = this lane's
// step-0 chunk). Every lane offers the dword its own group asks for, so all
// lanes must execute it.
template <int LG>
__device__ __forceinline__ void junk_take(const uint4 &c0, uint32_t gbase,
                                          const Junk &j, uint32_t (&x)[3]) {
  static_assert(LG >= 1, "junk chunks 0/1 must sit in different lanes of step 0");
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const uint32_t d = j.off[k];
    x[k] = __shfl(pick_dword(c0, (d >> 2) & 3u), (int)(gbase + (d >> 4)), 64);
  }
}

template <bool BE>
__device__ __forceinline__ uint32_t junk_sum(const uint32_t (&x)[3],
                                             const Junk &j, uint32_t sel) {
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < 3; ++k) s = add_word<BE>(x[k] & j.mask[k], sel, s);
  return s;
}

// ---------------------------------------------------------------------
// Per-packet side data (uint16 initial or the 8-byte {src,dst} record),
// fetched together with the packet bytes so the epilogue never waits on a
// dependent load. Absent arrays read a zero word with stride 0, so the side
// loads are unconditional too.
// ---------------------------------------------------------------------
__device__ uint32_t g_side_zero[2] = {0u, 0u};

struct Side {
  uint32_t a, b;
  uint16_t i;  // 16-bit: widened at its use, not right after its load
};

struct SidePtrs {
  const uint8_t *a;
  const uint8_t *i;
  uint32_t as, is;
};

__device__ __forceinline__ SidePtrs side_ptrs(const BatchArgs &A) {
  SidePtrs s;
  const bool use_addrs = A.addrs && mode_has_pseudo(A.mode);
  s.a = use_addrs ? A.addrs : (const uint8_t *)g_side_zero;
  s.as = use_addrs ? 8u : 0u;
  s.i = A.initial_arr ? (const uint8_t *)A.initial_arr : (const uint8_t *)g_side_zero;
  s.is = A.initial_arr ? 2u : 0u;
  return s;
}

__device__ __forceinline__ Side load_side(const SidePtrs &sp, uint64_t p) {
  const uint32_t *a = (const uint32_t *)(sp.a + p * sp.as);
  Side s;
  s.a = a[0];
  s.b = a[1];
  s.i = *(const uint16_t *)(sp.i + p * sp.is);
  return s;
}

// Per-packet epilogue. `v` is the packet's word sum (exact uint32 for BE,
// its residue for LE). Adds the non-payload terms of the reference
// composition, folds, complements, stores (and optionally sets the field).
__device__ __forceinline__ uint32_t packet_value(const BatchArgs &A, uint32_t v, uint64_t len,
                                                 const Side &sd) {
  const int mode = A.mode;
  if (mode == YU_MODE_RAW) {
    v += A.initial_arr ? sd.i : A.initial;
  } else if (mode_has_pseudo(mode)) {
    uint32_t ph;
    if (A.addrs) {
      // PseudoHeaderChecksum(proto, src, dst): src/dst big-endian words + proto
      ph = sadperm(sd.a, kSelSwap, 0u);
      ph = sadperm(sd.b, kSelSwap, ph);
      ph += mode_proto(mode);
    } else {
      ph = A.initial_arr ? sd.i : A.initial;
    }
    // + Checksum(BE16(uint16(length))) — header/udp.go:70-72, tcp.go:168-170
    v += ph + (uint32_t)(len & 0xFFFFu);
  }
  uint32_t r = fold32(v);
  if (mode_is_tx(mode)) r = (~r) & 0xFFFFu;
  return r;
}

// The field value r stored big-endian into the packet (TX fill), if the
// field lies inside the first hdr_end bytes.
__device__ __forceinline__ void store_field(const BatchArgs &A, uint32_t r, uint8_t *pkt,
                                            uint32_t hdr_end) {
  const int mode = A.mode;
  if (A.fill && pkt && mode_is_tx(mode)) {
    const uint32_t f = mode_field(mode);
    if (f + 2u <= hdr_end) {
      // binary.BigEndian.PutUint16: one 16-bit store when the field is
      // 2-aligned (always, for the 4-aligned uniform fill), else two bytes
      // Uniform batches store it non-temporally (72-B datagrams: 42.5 -> 36.4 us
      // per 1M; ragged ones measured mixed, tools/kbench KB_FILL=1).
      uint8_t *q = pkt + f;
      const uint16_t be = (uint16_t)((r >> 8) | (r << 8));
      if (((uintptr_t)q & 1u) == 0 && !A.offsets) {
        __builtin_nontemporal_store(be, (uint16_t *)q);
      } else if (((uintptr_t)q & 1u) == 0) {
        *(uint16_t *)q = be;
      } else {
        q[0] = (uint8_t)(r >> 8);
        q[1] = (uint8_t)r;
      }
    }
  }
}

// The batch's extent: the call may touch data[0, offsets[n]) (ragged; offsets
// index the caller's data array), everything for uniform batches (whose geometry
// the host checked). One scalar load per wave.
struct Extent {
  uint64_t hi;
};
__device__ __forceinline__ Extent batch_extent(const BatchArgs &A) {
  Extent e;
  e.hi = A.offsets ? A.offsets[A.n] : ~0ull;
  return e;
}

// The packet [off, off + len) whose field a fill call may write: none when not
// filling, or when the packet is out of contract: longer than
// YU_MAX_TRANSPORT_LEN (decreasing offsets wrap its length there too) or ending
// past offsets[n] (outside what the call may touch: some other packet's offsets
// decrease). Such a packet gets an unspecified value and no byte is written for
// it (include/yucsum.h, "Out of contract"). Every fill mode is a transport /
// IPv4 / ICMP / datagram mode, so the limit is the transport one.
__device__ __forceinline__ uint8_t *fill_at(const BatchArgs &A, const Extent &x, uint64_t off,
                                            uint64_t len) {
  const bool in = len <= YU_MAX_TRANSPORT_LEN && off <= x.hi && len <= x.hi - off;
  return A.fill && in ? A.fill + off : nullptr;
}

__device__ __forceinline__ void finish_packet(const BatchArgs &A, uint64_t p,
                                              uint32_t v, uint64_t len,
                                              const Side &sd, uint8_t *pkt,
                                              uint32_t hdr_end) {
  const uint32_t r = packet_value(A, v, len, sd);
  if (A.out) A.out[p] = (uint16_t)r;
  store_field(A, r, pkt, hdr_end);
}

// Chunk c at window offset cr, cut at the packet end E: dword j (window
// offset cr + 4j) is whole if it ends by E, keeps its first E&3 bytes (tm) if
// it straddles E, and is dropped otherwise. lim[j] = floor4(E) - 4j (signed:
// may be negative).
__device__ __forceinline__ uint32_t tail_cut(uint32_t x, int cr, int lim,
                                             uint32_t tm) {
  return cr < lim ? x : (cr == lim ? (x & tm) : 0u);
}

template <bool BE>
__device__ __forceinline__ uint32_t sum_masked(const uint4 &c, int cr,
                                               const int (&lim)[4], uint32_t tm,
                                               uint32_t sel, uint32_t acc) {
  acc = add_word<BE>(tail_cut(c.x, cr, lim[0], tm), sel, acc);
  acc = add_word<BE>(tail_cut(c.y, cr, lim[1], tm), sel, acc);
  acc = add_word<BE>(tail_cut(c.z, cr, lim[2], tm), sel, acc);
  acc = add_word<BE>(tail_cut(c.w, cr, lim[3], tm), sel, acc);
  return acc;
}

template <bool BE>
__device__ __forceinline__ uint32_t sum_full(const uint4 &c, uint32_t sel,
                                             uint32_t acc) {
  acc = add_word<BE>(c.x, sel, acc);
  acc = add_word<BE>(c.y, sel, acc);
  acc = add_word<BE>(c.z, sel, acc);
  acc = add_word<BE>(c.w, sel, acc);
  return acc;
}

// IPv4 modes: HeaderLength() = (b[0] & 0xf) * 4 (header/ipv4.go:91-93); b[0]
// is byte sh of dword 0 of the window, held by the group's first lane.
__device__ __forceinline__ uint32_t ipv4_hl(uint32_t w0, uint32_t sh) {
  return ((w0 >> (8u * sh)) & 0xFu) * 4u;
}

// ---------------------------------------------------------------------
// k_small<G, U, NT>: uniform stride, whole packet window in one step,
// software-pipelined: the loads of step t+1 are issued before step t is
// summed, reduced and stored.
// ---------------------------------------------------------------------
template <int G, int U>
struct SmallItem {
  uint4 c[U];
  Side sd;
  uint32_t sh, len;
};

// Fetch the windows of packets pb+gw (pb = the wave's first packet of the
// step; pb >= n fetches nothing).
template <int G, int U, int NT, bool SIDE = true>
__device__ __forceinline__ void small_fetch(const BatchArgs &A,
                                            const SidePtrs &sp, uint64_t pb,
                                            uint32_t gw, uint32_t gl, bool ipv4,
                                            SmallItem<G, U> &it) {
  const uint64_t p = pb + gw;
  const bool active = p < A.n;
  const uint64_t data = (uint64_t)(uintptr_t)A.data;
  const uint64_t base = uniform64((data + pb * A.stride) & ~3ull);
  const uint64_t sabs = data + (active ? p : pb) * A.stride;
  const uint32_t lw = (uint32_t)((sabs & ~3ull) - base);  // this group's window
  it.sh = (uint32_t)(sabs & 3u);
  it.len = active ? A.len : 0u;
  const uint32_t le = ipv4 ? (it.len < 60u ? it.len : 60u) : it.len;
  const uint32_t eload = active ? it.sh + le : 0u;
  const __amdgpu_buffer_rsrc_t r = rsrc_at(base, A.end);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint32_t cr = 16u * (gl + (uint32_t)u * G);
    it.c[u] = bld16(r, cr < eload ? lw + cr : kOOB, nt_step<NT>(u, U));
  }
  if (SIDE) it.sd = load_side(sp, active ? p : A.n - 1);
}

// PR (packets per run): 0 = wave w's step t takes packets (w + t*waves)*GPW on
// (the grid's waves interleave over the batch); PR > 0 = wave w takes PR
// consecutive packets in PR/GPW steps, then the run w + waves and so on. A
// run's side records (PR * 8 or 2 bytes) come in with one load by lanes
// 0..PR-1 when its first step is fetched, and its results leave in one store
// (PR * 2 bytes) after its last step: per-step side loads and result stores
// are small scattered requests, and a wave's loads return in order, so one
// slow side load holds up the packet bytes behind it.
template <int G, int U, int NT, int PR = 0>
__global__ __launch_bounds__(256) void k_small(BatchArgs A) {
  constexpr int GPW = 64 / G;
  constexpr int SPR = PR ? PR / GPW : 1;  // steps per run
  static_assert(PR == 0 || (PR % GPW == 0 && PR <= 64 && (SPR & (SPR - 1)) == 0),
                "a run is whole wave steps and fits the wave's lanes");
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t gl = lane & (G - 1);
  const uint32_t gw = lane / G;
  const uint64_t wave = grid_wave(A.xcd);
  const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
  const int mode = A.mode;
  const bool ipv4 = mode_is_ipv4(mode);
  const SidePtrs sp = side_ptrs(A);
  const uint32_t uf = A.uf;
  // first packet of the wave's step t
  auto first = [&](uint64_t t) -> uint64_t {
    if (PR == 0) return (wave + t * nwaves) * GPW;
    return (wave + t / SPR * nwaves) * PR + (t % SPR) * GPW;
  };

  uint64_t t = 0;
  uint64_t pb = first(0);
  if (pb >= A.n) return;
  uint32_t res = 0;  // PR: lane s < PR collects the run's result s
  Side rs, nrs;      // PR: the current / next run's side record of packet `lane`
  // Where a run's side records sit. G <= 16 (a group within one DPP row): the
  // record of step j for group g is loaded by the group's lane G-1-j, so the
  // group's last lane, which finishes the packet, holds step 0's and a row_shr:1
  // after each step brings the next one to it (no LDS permute). G > 16: lane s
  // loads the run's record s, fetched with a permute each step.
  constexpr bool kDppSide = G <= 16;
  auto run_side = [&](uint64_t q, Side &d) __attribute__((always_inline)) {
    uint64_t x = q + lane;  // lanes >= PR read the run's first record again
    bool own = lane < (uint32_t)PR;
    if (kDppSide) {
      const uint32_t jj = (uint32_t)(G - 1) - gl;  // step whose record this lane holds
      x = q + (uint64_t)jj * GPW + gw;
      own = jj < (uint32_t)SPR;
    }
    d = load_side(sp, own && x < A.n ? x : (q < A.n ? q : A.n - 1));
  };
  // One step: issue the loads of the next step into `nx`, then sum `it` and
  // finish its packets. Returns false when the wave has no next step. The
  // loop below alternates two items instead of copying nx into it: a copy
  // would wait for the prefetch to land before the back-edge.
  auto step = [&](const SmallItem<G, U> &it, SmallItem<G, U> &nx) __attribute__((always_inline)) -> bool {
    const uint64_t pn = first(t + 1);
    const bool more = pn < A.n;  // wave-uniform
    const uint32_t k = (uint32_t)(t % SPR);
    small_fetch<G, U, NT, PR == 0>(A, sp, more ? pn : A.n, gw, gl, ipv4, nx);
    if (PR && k == 0 && t) rs = nrs;  // after the prefetch: the copy waits for nrs only
    if (PR && k == SPR - 1 && more) run_side(pn, nrs);

    uint32_t E = it.sh + it.len;
    if (ipv4) {
      const uint32_t hl = __shfl(ipv4_hl(it.c[0].x, it.sh), (int)(lane & ~(uint32_t)(G - 1)), 64);
      E = it.sh + (it.len < hl ? it.len : hl);
    }
    const int F = (int)(E & ~3u);
    const int lim[4] = {F, F - 4, F - 8, F - 12};
    const uint32_t tm = (1u << (8u * (E & 3u))) - 1u;
    uint32_t acc = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int cr = 16 * (int)(gl + (uint32_t)u * G);
      if ((uint32_t)u < uf)
        acc = sum_full<false>(it.c[u], 0u, acc);
      else
        acc = sum_masked<false>(it.c[u], cr, lim, tm, 0u, acc);
    }
    const uint64_t p = pb + gw;
    const Junk j = make_junk(it.sh, E, mode);
    uint32_t jx[3] = {0u, 0u, 0u};
    if (PR && kDppSide) {
      // the junk dwords lie in step 0's chunks of the group's first lanes: each
      // lane takes its own share off its partial sum before the reduction
      uint32_t own = 0;
#pragma unroll
      for (int i = 0; i < 3; ++i)
        if ((j.off[i] >> 4) == gl) own = sad(pick_dword(it.c[0], (j.off[i] >> 2) & 3u) & j.mask[i], own);
      acc -= own;
    } else {
      junk_take<__builtin_ctz(G)>(it.c[0], lane & ~(uint32_t)(G - 1), j, jx);
    }
    acc = group_total<G>(acc);
    if (PR == 0) {
      if (gl == G - 1 && p < A.n) {
        const uint32_t v = le_to_be(acc - junk_sum<false>(jx, j, 0u), it.sh & 1u);
        finish_packet(A, p, v, it.len, it.sd,
                      A.fill ? A.fill + p * A.stride : nullptr, E - it.sh);
      }
    } else {
      // the group's side record: in its last lane (G <= 16, then shifted on for
      // the next step), else from the lane that loaded it for the run
      Side sd;
      if (kDppSide) {
        sd = rs;
        rs.a = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)rs.a, 0x111, 0xf, 0xf, true);  // row_shr:1
        rs.b = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)rs.b, 0x111, 0xf, 0xf, true);
        rs.i = (uint16_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)rs.i, 0x111, 0xf, 0xf, true);
      } else {
        const int src = (int)(k * GPW + gw);
        sd.a = (uint32_t)__shfl((int)rs.a, src, 64);
        sd.b = (uint32_t)__shfl((int)rs.b, src, 64);
        sd.i = (uint16_t)__shfl((int)rs.i, src, 64);
      }
      // every lane computes; the group's last lane holds the true value
      const uint32_t v = le_to_be(acc - (kDppSide ? 0u : junk_sum<false>(jx, j, 0u)), it.sh & 1u);
      const uint32_t r = packet_value(A, v, it.len, sd);
      if (gl == G - 1 && p < A.n && A.fill) store_field(A, r, A.fill + p * A.stride, E - it.sh);
      const uint32_t got = (uint32_t)__shfl((int)r, (int)((lane % GPW) * G + G - 1), 64);
      res = lane / GPW == k ? got : res;
      if (k == SPR - 1 || !more) {
        const uint64_t q = pb - (uint64_t)k * GPW + lane;  // the run's packet `lane`
        if (lane < (uint32_t)PR && q < A.n && A.out) A.out[q] = (uint16_t)res;
      }
    }
    pb = pn;
    ++t;
    return more;
  };
  SmallItem<G, U> a, b;
  small_fetch<G, U, NT, PR == 0>(A, sp, pb, gw, gl, ipv4, a);
  if (PR) run_side(pb, rs);
  for (;;) {
    if (!step(a, b)) break;
    if (!step(b, a)) break;
  }
}

// ---------------------------------------------------------------------
// k_tiny<G, NT>: uniform stride, packets of <= 16G bytes starting 4-byte
// aligned: RAW, the TX modes UDP / TCP / ICMP (field masked in place) and
// VERIFY_TCP / VERIFY_UDP — every mode without a per-packet header walk.
// For tiny packets k_small spends a whole per-packet epilogue on every 1 KiB
// loaded; here a wave step covers 64 packets (G KiB): group g (G lanes) loads
// chunk j of G packets (slot k holds packet pb + (64/G)k + g, so each load
// instruction reads 64/G consecutive packets = one contiguous KiB). After the
// per-slot group sums, a cross-lane transpose gives slot j's total to lane j
// of the group, and all 64 lanes finish one packet each.
// ---------------------------------------------------------------------
template <int G>
struct TinyItem {
  uint4 c[G];
  Side sd;  // side data of the packet this lane finishes
};

template <int G, int NT>
__device__ __forceinline__ void tiny_fetch(const BatchArgs &A, const SidePtrs &sp,
                                           uint64_t pb, uint32_t g, uint32_t j,
                                           TinyItem<G> &it) {
  constexpr uint32_t GPW = 64 / G;
  const uint64_t base = uniform64((uint64_t)(uintptr_t)A.data + pb * A.stride);
  const __amdgpu_buffer_rsrc_t r = rsrc_at(base, A.end);
  const bool in = 16u * j < A.len;
#pragma unroll
  for (int k = 0; k < G; ++k) {
    const uint32_t q = GPW * (uint32_t)k + g;  // packet pb + q
    const bool active = in && pb + q < A.n;
    it.c[k] = bld16(r, active ? (uint32_t)(q * A.stride) + 16u * j : kOOB, NT != 0);
  }
  const uint64_t pf = pb + GPW * j + g;
  it.sd = load_side(sp, pf < A.n ? pf : A.n - 1);
}

// Every lane of each G-lane group gets the value of the group's last lane.
template <int G>
__device__ __forceinline__ uint32_t bcast_last(uint32_t v, uint32_t lane) {
  if (G == 4)  // quad_perm [3,3,3,3]
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xFF, 0xf, 0xf, false);
  return (uint32_t)__shfl(v, (int)(lane | (G - 1)), 64);
}

// Fill with whole chunks (k_tiny): lane (g, f/16) of slot k holds the field
// chunk of packet pb + (64/G)k + g, whose value lane (g, k) computed. It patches
// the field in its register copy, and every slot goes back out with the same
// offsets it was loaded from. Only when no chunk reaches into the next packet
// (stride >= the 16-byte-rounded length), and never past the batch's last whole
// dword (the last packet's partial tail dword holds no field).
template <int G>
__device__ __forceinline__ void tiny_store(const BatchArgs &A, uint64_t pb, uint32_t g, uint32_t j,
                                           const TinyItem<G> &it, uint32_t be, uint32_t f) {
  constexpr uint32_t GPW = 64 / G;
  const uint64_t e4 = A.end & ~3ull;  // packets start 4-aligned (fill contract)
  const uint32_t fd = (f >> 2) & 3u, sh = (f & 2u) * 8u;
  const uint32_t m = 0xFFFFu << sh;
  const bool holder = j == (f >> 4);
  const bool in = 16u * j < A.len;
#pragma unroll
  for (int k = 0; k < G; ++k) {
    const uint32_t v = ((uint32_t)__shfl((int)be, (int)(g * G + (uint32_t)k), 64)) << sh;
    uint4 c = it.c[k];
    if (holder) {
      c.x = fd == 0 ? (c.x & ~m) | v : c.x;
      c.y = fd == 1 ? (c.y & ~m) | v : c.y;
      c.z = fd == 2 ? (c.z & ~m) | v : c.z;
      c.w = fd == 3 ? (c.w & ~m) | v : c.w;
    }
    const uint64_t q = pb + GPW * (uint32_t)k + g;
    uint32_t *dst = (uint32_t *)(A.fill + q * A.stride + 16u * j);
    const uint64_t da = (uint64_t)(uintptr_t)dst;
    if (in && q < A.n) {
      if (da + 16u <= e4) {
        *(uint4 *)dst = c;
      } else {  // the batch's last chunk: whole dwords only
        if (da + 4u <= e4) dst[0] = c.x;
        if (da + 8u <= e4) dst[1] = c.y;
        if (da + 12u <= e4) dst[2] = c.z;
      }
    }
  }
}

template <int G, int NT, bool WB = false>
__global__ __launch_bounds__(256) void k_tiny(BatchArgs A) {
  constexpr uint32_t GPW = 64 / G;
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t j = lane & (G - 1);
  const uint32_t g = lane / G;
  const uint64_t wave = grid_wave(A.xcd);
  const uint64_t step = (uint64_t)gridDim.x * (blockDim.x >> 6) * 64u;
  const SidePtrs sp = side_ptrs(A);
  const uint32_t E = A.len;  // window base = packet start (4-aligned)
  const int F = (int)(E & ~3u);
  const int lim[4] = {F, F - 4, F - 8, F - 12};
  const uint32_t tm = (1u << (8u * (E & 3u))) - 1u;
  const bool full = A.uf != 0;  // every chunk of every packet is whole
  // TX modes: Encode leaves the checksum field 0. Starts are 4-aligned and the
  // field offset is even, so the field is 16 bits of one dword: chunk f/16,
  // dword (f%16)/4 — masked in the lanes that load that chunk.
  const uint32_t f = mode_field(A.mode);
  const uint32_t fm = (mode_is_tx(A.mode) && j == f / 16u) ? ~(0xFFFFu << (8u * (f & 3u))) : ~0u;
  const uint32_t fd = (f >> 2) & 3u;
  const uint4 m4 = make_uint4(fd == 0 ? fm : ~0u, fd == 1 ? fm : ~0u, fd == 2 ? fm : ~0u,
                              fd == 3 ? fm : ~0u);
  // fill with whole chunks (tiny_store): its own instantiation, so the plain
  // kernel keeps its registers
  const bool wb = WB && A.fill && A.stride >= ((A.len + 15u) & ~15u);

  uint64_t pb = wave * 64u;
  if (pb >= A.n) return;
  TinyItem<G> it;
  tiny_fetch<G, NT>(A, sp, pb, g, j, it);
  for (;;) {
    const uint64_t pn = pb + step;
    const bool more = pn < A.n;  // wave-uniform
    TinyItem<G> nx;
    tiny_fetch<G, NT>(A, sp, more ? pn : A.n, g, j, nx);

    uint32_t mine = 0;
#pragma unroll
    for (int k = 0; k < G; ++k) {
      const uint4 c = make_uint4(it.c[k].x & m4.x, it.c[k].y & m4.y, it.c[k].z & m4.z,
                                 it.c[k].w & m4.w);
      uint32_t acc = full ? sum_full<false>(c, 0u, 0u)
                          : sum_masked<false>(c, 16 * (int)j, lim, tm, 0u, 0u);
      acc = bcast_last<G>(group_total<G>(acc), lane);
      mine = (j == (uint32_t)k) ? acc : mine;
    }
    const uint64_t pf = pb + GPW * j + g;
    if (wb) {
      const uint32_t r = packet_value(A, le_to_be(mine, 0u), E, it.sd);
      if (pf < A.n && A.out) A.out[pf] = (uint16_t)r;
      tiny_store<G>(A, pb, g, j, it, ((r >> 8) | (r << 8)) & 0xFFFFu, f);
    } else if (pf < A.n) {
      finish_packet(A, pf, le_to_be(mine, 0u), E, it.sd, A.fill ? A.fill + pf * A.stride : nullptr, E);
    }
    if (!more) break;
    it = nx;
    pb = pn;
  }
}

// ---------------------------------------------------------------------
// k_lane<U, NT>: uniform, 4-aligned packets of 65..16U bytes with
// len <= stride <= 16U — the sizes where k_tiny<8> leaves lanes idle (a
// 72-byte UDP datagram fills 5 of its 8 chunks) and k_small pays a group
// reduction per packet. A wave step covers 64 packets, i.e. the contiguous
// 64*stride bytes from packet pb on: U coalesced dwordx4 loads per lane,
// parked in the wave's own LDS slice (no block barrier: LDS operations of one
// wave complete in order). Each lane then sums its own packet from LDS, one
// ds_read_b32 per dword, starting at dword lane % nd so that lanes whose
// packets start on the same bank read different banks.
// ---------------------------------------------------------------------
template <int U>
__device__ __forceinline__ void lane_fetch(const BatchArgs &A, const SidePtrs &sp,
                                           uint64_t pb, uint32_t lane, uint32_t span,
                                           bool nt, uint4 (&c)[U], Side &sd) {
  const uint64_t base = uniform64((uint64_t)(uintptr_t)A.data + pb * A.stride);
  const __amdgpu_buffer_rsrc_t r = rsrc_at(base, A.end);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint32_t off = 16u * (64u * (uint32_t)u + lane);
    c[u] = bld16(r, off < span ? off : kOOB, nt);
  }
  const uint64_t p = pb + lane;
  sd = load_side(sp, p < A.n ? p : A.n - 1);
}

// LE sum of nw W-dword units of a lane's packet in LDS, starting at unit k0
// and wrapping (summation order is free; the rotation spreads the lanes over
// the LDS banks). W = 4 / 2 / 1: ds_read_b128 / b64 / b32.
template <int W>
__device__ __forceinline__ uint32_t lane_sum(const uint32_t *own, uint32_t nw, uint32_t k0) {
  uint32_t acc = 0, k = k0;
  for (uint32_t d = 0; d < nw; ++d) {
    if (W == 4) {
      const uint4 v = *(const uint4 *)(own + 4u * k);
      acc = sad(v.w, sad(v.z, sad(v.y, sad(v.x, acc))));
    } else if (W == 2) {
      const uint2 v = *(const uint2 *)(own + 2u * k);
      acc = sad(v.y, sad(v.x, acc));
    } else {
      acc = sad(own[k], acc);
    }
    k = k + 1u == nw ? 0u : k + 1u;
  }
  return acc;
}

// Stores a step's bytes from the wave's LDS slice back to the batch (fill):
// only whole dwords before the batch end — the last packet's partial tail
// dword holds no field and is left alone.
template <int U>
__device__ __forceinline__ void lane_store(const BatchArgs &A, uint64_t pb, uint32_t lane,
                                           uint32_t span, const uint4 *slice) {
  const uint64_t base = uniform64((uint64_t)(uintptr_t)A.fill + pb * A.stride);
  const uint64_t lim = (A.end & ~3ull) > base ? (A.end & ~3ull) - base : 0u;
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
      (void *)base, (short)0, (int)(lim < span ? lim : span), 0x00020000);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint32_t off = 16u * (64u * (uint32_t)u + lane);
    const uint4 c = slice[64 * u + lane];
    __builtin_amdgcn_raw_buffer_store_b128(u32x4{c.x, c.y, c.z, c.w}, r, (int)(off < span ? off : kOOB), 0, 0);
  }
}

__device__ __forceinline__ void wave_lds_fence() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int U, int NT>
__global__ __launch_bounds__(256) void k_lane(BatchArgs A) {
  __shared__ uint4 park[4][64 * U];
  const uint32_t lane = threadIdx.x & 63u;
  uint4 *slice = park[__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)];
  const uint64_t wave = grid_wave(A.xcd);
  const uint64_t step = (uint64_t)gridDim.x * (blockDim.x >> 6) * 64u;
  const SidePtrs sp = side_ptrs(A);
  const uint32_t S = (uint32_t)A.stride;
  const uint32_t E = A.len;
  const uint32_t span = 64u * S;
  const uint32_t nd = (E + 3u) >> 2;  // dwords per packet
  // bytes past E in the last dword (the dword-granular sum takes them)
  const uint32_t junk_tail = (E & 3u) ? ~((1u << (8u * (E & 3u))) - 1u) : 0u;
  // TX modes: Encode leaves the 16-bit checksum field 0; starts are 4-aligned
  // and the field offset even, so it is half of dword f/4
  const uint32_t f = mode_field(A.mode);
  const bool tx = mode_is_tx(A.mode);
  const uint32_t junk_field = 0xFFFFu << (8u * (f & 3u));
  // widest LDS read that tiles the packet and stays aligned (wave-uniform)
  const uint32_t W = ((E | S) & 15u) == 0 ? 4u : (((E | S) & 7u) == 0 ? 2u : 1u);
  const uint32_t nw = nd / W;
  const uint32_t k0 = lane % nw;
  const uint32_t *own = (const uint32_t *)slice + lane * (S >> 2);

  uint64_t pb = wave * 64u;
  if (pb >= A.n) return;
  uint4 c[U];
  Side sd;
  lane_fetch<U>(A, sp, pb, lane, span, NT != 0, c, sd);
  for (;;) {
    const uint64_t pn = pb + step;
    const bool more = pn < A.n;  // wave-uniform
    uint4 nx[U];
    Side nsd;
    lane_fetch<U>(A, sp, more ? pn : A.n, lane, span, NT != 0, nx, nsd);

#pragma unroll
    for (int u = 0; u < U; ++u) slice[64 * u + lane] = c[u];
    wave_lds_fence();
    uint32_t acc = W == 4u ? lane_sum<4>(own, nw, k0)
                           : (W == 2u ? lane_sum<2>(own, nw, k0) : lane_sum<1>(own, nw, k0));
    // the sum is exact (<= 128 bytes), so junk bytes come off by subtraction
    if (junk_tail) acc -= sad(own[nd - 1u] & junk_tail, 0u);
    if (tx) acc -= sad(own[f >> 2] & junk_field, 0u);
    wave_lds_fence();  // the next step's stores stay behind these reads

    const uint64_t p = pb + lane;
    if (A.fill) {
      // In place: the field goes into the LDS copy and the step's bytes go back
      // out as whole 16-byte chunks, so memory sees full-line writes instead of
      // one 2-byte write per packet (1M x 72-B datagrams: 42.3 -> 30.0 us,
      // 100-B: 54.9 -> 41.2; tools/kbench 14 KB_FILL=1).
      const uint32_t r = packet_value(A, le_to_be(acc, 0u), E, sd);
      if (p < A.n && A.out) A.out[p] = (uint16_t)r;
      if (p < A.n && f + 2u <= E)
        ((uint16_t *)slice)[(lane * S + f) >> 1] = (uint16_t)((r >> 8) | (r << 8));
      wave_lds_fence();
      lane_store<U>(A, pb, lane, span, slice);
    } else if (p < A.n) {
      finish_packet(A, p, le_to_be(acc, 0u), E, sd, nullptr, E);
    }
    if (!more) break;
#pragma unroll
    for (int u = 0; u < U; ++u) c[u] = nx[u];
    sd = nsd;
    pb = pn;
  }
}

// ---------------------------------------------------------------------
// k_loop<U, NT, BE>: one wave per packet, 64*U*16-byte windows (ragged /
// large packets). The wave walks a stream of (packet, window) items and
// always issues the loads of the next item — the next window of this
// packet, or the first window and side data of its next packet
// (whose offsets were read one packet ahead) — before it sums the current.
// ---------------------------------------------------------------------
struct LoopPkt {
  uint64_t soff, len;
  uint64_t base;  // floor4(packet start) as an address
  uint32_t sh, E, eload;
};

__device__ __forceinline__ void loop_pkt(const BatchArgs &A, uint64_t p,
                                         bool ipv4, LoopPkt &k) {
  if (p >= A.n) {  // no packet: every load of it is out of range
    k.soff = 0;
    k.len = 0;
    k.base = (uint64_t)(uintptr_t)A.data & ~3ull;
    k.sh = 0;
    k.E = 0;
    k.eload = 0;
    return;
  }
  if (A.offsets) {
    k.soff = A.offsets[p];
    k.len = A.offsets[p + 1] - k.soff;
  } else {
    k.soff = p * A.stride;
    k.len = A.len;
  }
  const uint64_t sabs = (uint64_t)(uintptr_t)A.data + k.soff;
  k.base = sabs & ~3ull;
  k.sh = (uint32_t)(sabs & 3u);
  // ragged packets past the limit get an unspecified value, never a hang
  const uint32_t l32 = k.len < YU_MAX_RAW_LEN ? (uint32_t)k.len : YU_MAX_RAW_LEN;
  k.E = k.sh + l32;
  k.eload = k.sh + (ipv4 ? (l32 < 60u ? l32 : 60u) : l32);
}

// Loads of window [wb, wb + 64*U*16) of packet k.
template <int U, int NT>
__device__ __forceinline__ void loop_fetch(const LoopPkt &k, uint32_t wb,
                                           uint32_t lane, uint64_t end,
                                           uint4 (&c)[U]) {
  const __amdgpu_buffer_rsrc_t r = rsrc_at(uniform64(k.base + wb), end);
  const uint32_t lim = k.eload > wb ? k.eload - wb : 0u;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint32_t cr = 16u * (lane + 64u * (uint32_t)u);
    c[u] = bld16(r, cr < lim ? cr : kOOB, NT != 0);
  }
}

template <int U, int NT, bool BE>
__global__ __launch_bounds__(256) void k_loop(BatchArgs A) {
  constexpr uint32_t W = 64u * 16u * U;
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t wave = grid_wave(A.xcd);
  const uint64_t nwave = (uint64_t)gridDim.x * (blockDim.x >> 6);
  const int mode = A.mode;
  const bool ipv4 = mode_is_ipv4(mode);
  const SidePtrs sp = side_ptrs(A);
  const bool lead = lane == 63;
  const uint64_t end = A.offsets ? (uint64_t)(uintptr_t)A.data + A.offsets[A.n] : A.end;
  const Extent ext = batch_extent(A);

  uint64_t p = wave;
  if (p >= A.n) return;
  LoopPkt cur, nxt;
  loop_pkt(A, p, ipv4, cur);
  Side sd = load_side(sp, p);
  uint32_t jx[3] = {0u, 0u, 0u};  // junk dwords, taken at window 0
  uint64_t pn = p + nwave;
  loop_pkt(A, pn, ipv4, nxt);

  uint32_t wb = 0;
  uint4 c[U];
  loop_fetch<U, NT>(cur, 0, lane, end, c);
  uint32_t acc = 0;
  for (;;) {
    const bool last = wb + W >= cur.eload;  // wave-uniform
    const bool more = !last || pn < A.n;
    // the next item: window wb+W of this packet, or window 0 of packet pn
    uint4 cn[U];
    loop_fetch<U, NT>(last ? nxt : cur, last ? 0u : wb + W, lane, end, cn);
    const Side sdn = load_side(sp, (last && pn < A.n) ? pn : p);

    uint32_t E = cur.E;
    if (ipv4) {  // single window: eload <= 63 < W
      const uint32_t hl = __shfl(ipv4_hl(c[0].x, cur.sh), 0, 64);
      const uint32_t l32 = (uint32_t)cur.len;
      E = cur.sh + (l32 < hl ? l32 : hl);
    }
    const Junk j = make_junk(cur.sh, E, mode);
    if (wb == 0) junk_take<6>(c[0], 0u, j, jx);
    const uint32_t sel = (cur.sh & 1u) ? kSelIdent : kSelSwap;
    if (wb + W <= E) {  // full window (wave-uniform)
#pragma unroll
      for (int u = 0; u < U; ++u) acc = sum_full<BE>(c[u], sel, acc);
    } else {
      const int f = (int)((E & ~3u) - wb);
      const int lim[4] = {f, f - 4, f - 8, f - 12};
      const uint32_t tm = (1u << (8u * (E & 3u))) - 1u;
#pragma unroll
      for (int u = 0; u < U; ++u)
        acc = sum_masked<BE>(c[u], 16 * (int)(lane + 64u * (uint32_t)u), lim, tm, sel, acc);
    }

    if (last) {
      acc = group_total<64>(acc);
      if (lead) {
        const uint32_t s = acc - junk_sum<BE>(jx, j, sel);
        const uint32_t v = BE ? s : le_to_be(s, cur.sh & 1u);
        finish_packet(A, p, v, cur.len, sd, fill_at(A, ext, cur.soff, cur.len),
                      E - cur.sh);
      }
      if (!more) break;
      // advance to the next packet; read the offsets of the one after it
      p = pn;
      cur = nxt;
      sd = sdn;
      pn = p + nwave;
      loop_pkt(A, pn, ipv4, nxt);
      wb = 0;
      acc = 0;
    } else {
      wb += W;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) c[u] = cn[u];
  }
}

// ---------------------------------------------------------------------
// k_hdr<NT>: the IPv4 header-only modes (IPV4 field value, VERIFY_IPV4) on
// ragged batches, one lane per packet. Only b[:HeaderLength()] (<= 60 bytes)
// of each packet is summed (header/ipv4.go:177-179, checker/checker.go:32),
// so streaming every byte (k_seg) or giving each packet a 16-lane group
// (k_rag: 4 packets per wave step) does far more work than needed. Here a
// wave step covers 64 packets: each lane loads the 64-byte window at
// floor4(start) (four dwordx4, cut at the packet's end), reads IHL from its
// first dword and sums the header bytes under byte masks.
__device__ __forceinline__ uint32_t byte_range_mask(uint32_t lo, uint32_t a, uint32_t b) {
  // bytes [a, b) of the dword holding bytes [lo, lo + 4)
  const uint32_t ka = a > lo ? (a - lo < 4u ? a - lo : 4u) : 0u;
  const uint32_t kb = b > lo ? (b - lo < 4u ? b - lo : 4u) : 0u;
  const uint64_t hi = (1ull << (8u * kb)) - 1ull, low = (1ull << (8u * ka)) - 1ull;
  return (uint32_t)(hi & ~low);
}

template <int NT>
__global__ __launch_bounds__(256) void k_hdr(BatchArgs A) {
  constexpr bool TWO = true;
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t wave = grid_wave(A.xcd);
  const uint64_t nwave = (uint64_t)gridDim.x * (blockDim.x >> 6);
  const uint64_t data = (uint64_t)(uintptr_t)A.data;
  const bool tx = mode_is_tx(A.mode);
  const Extent ext = batch_extent(A);
  for (uint64_t p0 = wave * 64u; p0 < A.n; p0 += nwave * 64u) {
    const uint64_t p = p0 + lane;
    const bool act = p < A.n;
    uint64_t s, e;
    if (A.offsets) {
      s = A.offsets[act ? p : A.n];
      e = A.offsets[act ? p + 1 : A.n];
    } else {  // lanes past the batch sit at the last packet's end
      s = act ? p * A.stride : (A.n - 1) * A.stride + A.len;
      e = act ? s + A.len : s;
    }
    // wave-uniform descriptor over the 64 packets' bytes (lane 0's start to
    // lane 63's end, which is the chunk's end: lanes past the batch sit there)
    const uint64_t base = uniform64((data + s) & ~3ull);
    // (clamped to the batch's end: out-of-contract offsets never widen what the
    // step may read past data[0, offsets[n]))
    const uint64_t le = readlane64(e, 63);
    const uint64_t cend = data + (le < ext.hi ? le : ext.hi);
    const __amdgpu_buffer_rsrc_t r = rsrc_at(base, cend);
    const uint64_t sa = data + s;
    const uint32_t sh = (uint32_t)sa & 3u;
    const uint64_t len = e - s;
    // The descriptor starts at lane 0's packet, so one out-of-contract packet of the
    // step (decreasing offsets, or longer than YU_MAX_TRANSPORT_LEN: include/yucsum.h)
    // can move every lane's window out of it: such a step stores no field (its
    // results are unspecified). In contract, lane 0's start is the step's lowest.
    const bool step_ok = !__any((int)(len > YU_MAX_TRANSPORT_LEN));
    const uint32_t lmax = sh + (uint32_t)(len < 60u ? len : 60u);  // bytes to load
    const uint64_t wo = (sa & ~3ull) - base;
    uint4 c[4];
    // the first 32 bytes, then the rest only for lanes whose header (IHL > 7
    // with the start offset) reaches past them: a 20-byte header costs one
    // 32-byte read (config 12 of tools/kbench: 55 -> 32.5 us)
#pragma unroll
    for (int k = 0; k < (TWO ? 2 : 4); ++k)
      c[k] = bld16(r, (16u * k < lmax && wo < kOOB) ? (uint32_t)wo + 16u * k : kOOB, NT != 0);
    const uint32_t hl = ipv4_hl(c[0].x, sh);
    if (TWO) {
      const uint32_t need = sh + (uint32_t)(len < hl ? len : hl);
#pragma unroll
      for (int k = 2; k < 4; ++k)
        c[k] = __any((int)(need > 32u))
                   ? bld16(r, (16u * k < need && wo < kOOB) ? (uint32_t)wo + 16u * k : kOOB, NT != 0)
                   : make_uint4(0u, 0u, 0u, 0u);
    }
    const uint32_t E = sh + (uint32_t)(len < hl ? len : hl);
    const bool fld = tx && sh + 12u <= E;  // Encode zeroes the field (network/ipv4/ipv4.go:85-94)
    const uint32_t f0 = fld ? sh + 10u : 0u, f1 = fld ? sh + 12u : 0u;
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t w[4] = {c[k].x, c[k].y, c[k].z, c[k].w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t lo = 16u * k + 4u * j;
        const uint32_t m = byte_range_mask(lo, sh, E) & ~byte_range_mask(lo, f0, f1);
        acc = sad(w[j] & m, acc);
      }
    }
    if (act) {
      const uint32_t v = le_to_be(acc, (uint32_t)sa & 1u);
      Side sd;
      sd.a = sd.b = 0u;
      sd.i = 0;
      finish_packet(A, p, v, len, sd, step_ok ? fill_at(A, ext, s, len) : nullptr, E - sh);
    }
  }
}

// k_rag<G, U, NT>: ragged batches of small packets (tun-style RX bursts,
// link/tundev/tundev.go:78-151). One packet per wave iteration (k_loop) is
// latency-bound when packets are a few hundred bytes; here a wave step holds
// 64/G packets, one per G-lane group, as in k_small, and a 3-stage pipeline
// keeps the next steps in flight: the offsets of step t+2 and the packet
// windows of step t+1 are loaded while step t is summed (phase 1). Packets
// longer than the 16*G*U-byte group window are skipped there and summed in
// phase 2, after the step loop: each wave scans 64 offsets at a time, ballots
// the long packets and sums each with all 64 lanes in 4 KiB windows. The two
// phases do not overlap, so the kernel pays the larger register budget, not
// the sum.
// ---------------------------------------------------------------------
template <int U>
struct RagItem {
  uint4 c[U];
  Side sd;         // side data of the group's packet
  uint64_t o;      // this lane's offset: offsets[min(pb + lane % (GPW+1), n)]
  uint32_t len, sh, eload;
  bool fits;       // this group's packet is summed in phase 1
};

__device__ __forceinline__ uint64_t shfl64(uint64_t v, uint32_t src) {
  const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, (int)src, 64);
  const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), (int)src, 64);
  return ((uint64_t)hi << 32) | lo;
}

// Phase 1 takes a packet iff it fits the group window and its window lies
// within 1 GiB of the step's base (the first packet of its step): lane window
// offsets are 32-bit. Phase 2 applies the same test and takes the rest.
__device__ __forceinline__ bool rag_fits(uint32_t need, uint64_t len, uint64_t from_base,
                                         uint32_t W) {
  return len <= 0xFFFFFFu && need <= W && from_base < (1ull << 30);
}

template <int G>
__device__ __forceinline__ uint64_t rag_offs(const BatchArgs &A, uint64_t pb, uint32_t lane) {
  constexpr uint32_t GPW = 64u / G;
  uint64_t i = pb + lane % (GPW + 1u);
  return A.offsets[i < A.n ? i : A.n];  // unconditional (clamped) load
}

template <int G, int U, int NT>
__device__ __forceinline__ void rag_fetch(const BatchArgs &A, const SidePtrs &sp, uint64_t pb,
                                          uint64_t o, uint32_t gw, uint32_t gl, bool ipv4,
                                          RagItem<U> &it) {
  constexpr uint32_t W = 16u * G * U;
  const uint64_t data = (uint64_t)(uintptr_t)A.data;
  const uint64_t p = pb + gw;
  const bool active = p < A.n;
  const uint64_t so = shfl64(o, gw);
  const uint64_t eo = shfl64(o, gw + 1u);
  it.o = o;
  it.len = active ? (uint32_t)(eo - so) : 0u;
  const uint64_t sabs = data + so;
  it.sh = (uint32_t)(sabs & 3u);
  const uint32_t need = it.sh + (ipv4 ? (it.len < 60u ? it.len : 60u) : it.len);
  // readfirstlane returns int: widen through uint32_t, never sign-extend
  const uint64_t o0 = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(o >> 32)) << 32) |
                      (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)o);
  const uint64_t base = uniform64((data + o0) & ~3ull);
  it.fits = active && rag_fits(need, eo - so, (sabs & ~3ull) - base, W);
  it.eload = it.fits ? need : 0u;
  const uint32_t lw = it.fits ? (uint32_t)((sabs & ~3ull) - base) : 0u;
  const __amdgpu_buffer_rsrc_t r = rsrc_at(base, data + A.offsets[A.n]);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint32_t cr = 16u * (gl + (uint32_t)u * G);
    it.c[u] = bld16(r, cr < it.eload ? lw + cr : kOOB, nt_step<NT>(u, U));
  }
  it.sd = load_side(sp, active ? p : A.n - 1);
}

// One packet summed by the whole wave in 4 KiB windows, no prefetch: the
// fallback for steps holding a packet longer than the group window.
template <bool BE>
__device__ __forceinline__ uint32_t rag_serial_sum(uint64_t sabs, uint32_t len, uint32_t E,
                                                   uint32_t lane, uint64_t end,
                                                   uint32_t (&jx)[3], const Junk &j) {
  constexpr uint32_t W = 64u * 16u * 4u;
  const uint32_t sh = (uint32_t)(sabs & 3u);
  const uint32_t sel = (sh & 1u) ? kSelIdent : kSelSwap;
  uint32_t acc = 0;
  for (uint32_t wb = 0; wb < sh + len; wb += W) {
    const __amdgpu_buffer_rsrc_t r = rsrc_at(uniform64((sabs & ~3ull) + wb), end);
    const uint32_t lim = sh + len - wb;
    uint4 c[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint32_t cr = 16u * (lane + 64u * (uint32_t)u);
      c[u] = bld16(r, cr < lim ? cr : kOOB, true);
    }
    if (wb == 0) junk_take<6>(c[0], 0u, j, jx);
    if (wb + W <= E) {  // full window (wave-uniform)
#pragma unroll
      for (int u = 0; u < 4; ++u) acc = sum_full<BE>(c[u], sel, acc);
    } else {  // last window: E - wb < W, so the int limits cannot overflow
      const int f = (int)((E & ~3u) - wb);
      const int limj[4] = {f, f - 4, f - 8, f - 12};
      const uint32_t tm = (1u << (8u * (E & 3u))) - 1u;
#pragma unroll
      for (int u = 0; u < 4; ++u)
        acc = sum_masked<BE>(c[u], 16 * (int)(lane + 64u * (uint32_t)u), limj, tm, sel, acc);
    }
  }
  acc = group_total<64>(acc);
  const uint32_t s = acc - junk_sum<BE>(jx, j, sel);
  return BE ? s : le_to_be(s, sh & 1u);
}

template <int G, int U, int NT>
__global__ __launch_bounds__(256) void k_rag(BatchArgs A) {
  constexpr uint32_t GPW = 64u / G;
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t gl = lane & (G - 1);
  const uint32_t gw = lane / G;
  const uint64_t wave = grid_wave(A.xcd);
  const uint64_t step = (uint64_t)gridDim.x * (blockDim.x >> 6) * GPW;
  const int mode = A.mode;
  const bool ipv4 = mode_is_ipv4(mode);
  const SidePtrs sp = side_ptrs(A);
  const uint64_t data = (uint64_t)(uintptr_t)A.data;
  const uint64_t end = data + A.offsets[A.n];
  const Extent ext = batch_extent(A);

  uint64_t pb = wave * GPW;
  if (pb >= A.n) return;
  uint64_t o1 = rag_offs<G>(A, pb + step, lane);
  RagItem<U> it;
  rag_fetch<G, U, NT>(A, sp, pb, rag_offs<G>(A, pb, lane), gw, gl, ipv4, it);
  for (;;) {
    const uint64_t pn = pb + step;
    const bool more = pn < A.n;  // wave-uniform
    const uint64_t o2 = rag_offs<G>(A, pb + 2 * step, lane);
    RagItem<U> nx;
    rag_fetch<G, U, NT>(A, sp, more ? pn : A.n, o1, gw, gl, ipv4, nx);

    uint32_t E = it.sh + it.len;
    if (ipv4) {
      const uint32_t hl = __shfl(ipv4_hl(it.c[0].x, it.sh), (int)(lane & ~(uint32_t)(G - 1)), 64);
      E = it.sh + (it.len < hl ? it.len : hl);
    }
    const int F = (int)(E & ~3u);
    const int lim[4] = {F, F - 4, F - 8, F - 12};
    const uint32_t tm = (1u << (8u * (E & 3u))) - 1u;
    uint32_t acc = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int cr = 16 * (int)(gl + (uint32_t)u * G);
      if (__all((int)(!it.fits || cr + 16 <= F)))  // every chunk whole: skip the cut
        acc = sum_full<false>(it.c[u], 0u, acc);
      else
        acc = sum_masked<false>(it.c[u], cr, lim, tm, 0u, acc);
    }
    acc = group_total<G>(acc);
    const Junk j = make_junk(it.sh, E, mode);
    uint32_t jx[3];
    junk_take<__builtin_ctz(G)>(it.c[0], lane & ~(uint32_t)(G - 1), j, jx);
    const uint64_t so = shfl64(it.o, gw);  // all lanes: a cross-lane read needs active sources
    if (gl == G - 1 && it.fits) {
      const uint32_t v = le_to_be(acc - junk_sum<false>(jx, j, 0u), it.sh & 1u);
      finish_packet(A, pb + gw, v, it.len, it.sd, fill_at(A, ext, so, it.len), E - it.sh);
    }
    if (!more) break;
    it = nx;
    o1 = o2;
    pb = pn;
  }

  // phase 2: the packets phase 1 skipped (longer than the group window, or
  // farther than 1 GiB from their step's base), one whole-wave sum each
  const uint64_t nwave = (uint64_t)gridDim.x * (blockDim.x >> 6);
  constexpr uint32_t W1 = 16u * G * U;
  for (uint64_t cb = wave * 64u; cb < A.n; cb += nwave * 64u) {
    const uint64_t i = cb + lane;
    const uint64_t ic = i < A.n ? i : A.n - 1;
    const uint64_t so = A.offsets[ic];
    const uint64_t eo = A.offsets[ic + 1];
    const uint64_t bo = A.offsets[ic - ic % GPW];  // its step's base packet
    const uint64_t sabs = data + so;
    const uint64_t len = eo - so;
    const uint32_t l32 = len < 0x0FFFFFFFu ? (uint32_t)len : 0x0FFFFFFFu;
    const uint32_t need = (uint32_t)(sabs & 3u) + (ipv4 ? (l32 < 60u ? l32 : 60u) : l32);
    const bool skipped =
        i < A.n && !rag_fits(need, len, (sabs & ~3ull) - ((data + bo) & ~3ull), W1);
    uint64_t mask = __ballot((int)skipped);
    while (mask) {  // wave-uniform
      const uint32_t q = (uint32_t)__builtin_ctzll(mask);
      mask &= mask - 1u;
      const uint64_t ps = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(so >> 32), q) << 32) |
                          (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)so, q);
      const uint64_t pe = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(eo >> 32), q) << 32) |
                          (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)eo, q);
      const uint64_t p = cb + q;
      const uint32_t plen = pe - ps < YU_MAX_RAW_LEN ? (uint32_t)(pe - ps) : YU_MAX_RAW_LEN;
      const uint64_t pabs = data + ps;
      const uint32_t sh = (uint32_t)(pabs & 3u);
      uint32_t E = sh + plen;
      if (ipv4) {  // only reached for packets far from their step base
        const __amdgpu_buffer_rsrc_t r = rsrc_at(uniform64(pabs & ~3ull), end);
        const uint32_t hl = ipv4_hl(__builtin_amdgcn_raw_buffer_load_b32(r, 0, 0, 0), sh);
        E = sh + (plen < hl ? plen : hl);
      }
      const Junk j = make_junk(sh, E, mode);
      uint32_t pjx[3];
      const uint32_t v = plen > kLEMax ? rag_serial_sum<true>(pabs, E - sh, E, lane, end, pjx, j)
                                       : rag_serial_sum<false>(pabs, E - sh, E, lane, end, pjx, j);
      const Side sd = load_side(sp, p);
      if (lane == 63) finish_packet(A, p, v, plen, sd, fill_at(A, ext, ps, plen), E - sh);
    }
  }
}

// ---------------------------------------------------------------------
// k_seg<U, NT>: ragged batches as a segmented sum over one byte stream.
//
// The packets of a ragged batch tile [offsets[0], offsets[n]) back to back,
// so a chunk of 64 consecutive packets is one contiguous byte range. A wave
// takes a chunk (lane l owns packet 64c + l) and streams the range in tiles
// of 64 lanes x U x 16 bytes — every load a full, coalesced dwordx4 whatever
// the packet sizes — while keeping P(x), the running LE sum (v_sad_u16) of
// the chunk's bytes before position x. A packet's sum is P(end) - P(start):
// prefix differences are exact mod 2^32 and a packet's LE sum stays below
// 2^32 up to 131072 bytes (the LE-sum limit of the header comment). In TX
// modes the checksum field is two more points, P(s+f+2) - P(s+f), taken off.
//
// Per tile: each lane sums its U chunks, a DPP scan over the wave orders the
// chunk sums by address, and only if a packet boundary falls in the tile are
// the chunk bytes and their exclusive prefixes parked in LDS, where each lane
// whose point lies in the tile reads the one chunk it needs and adds the
// bytes before the point. Packets larger than a tile cost one scan per tile
// and no LDS traffic; small packets cost a few LDS reads each instead of a
// lane group per packet, so HBM sees the same byte stream for any mix.
//
// RAW packets longer than 131072 bytes need the reference's exact uint32
// accumulator (its wrap). A chunk holding one also keeps T(x), the plain byte
// sum (v_sad_u8): with A/B the sums of the bytes at even/odd addresses,
// L = A + 256 B and T = A + B (mod 2^32), so B = (L - T) * 255^-1 and A = T - B,
// and the big-endian word sum is 256 A + B (even start) or A + 256 B (odd
// start) — bit-exact mod 2^32 at any length.
//
// Pipelining: the loads of the next tile — of this chunk, or the first tile
// of the wave's next chunk, whose offsets and side data were read one chunk
// ahead — are issued before the current tile is summed.
// ---------------------------------------------------------------------
constexpr uint32_t kInv255 = 0xFEFEFEFFu;  // 255 * kInv255 == 1 (mod 2^32)

struct SegChunk {
  uint64_t ox, oy;  // this lane's packet [ox, oy) as offsets into data (lanes
                    // past the batch: the chunk end)
  uint64_t b0;      // floor4 address of the chunk's first byte (wave-uniform)
  uint64_t xe;      // chunk end relative to b0 (wave-uniform)
  Side sd;
};

// Loads only: the packet bounds and side data of the chunk starting at
// packet p0. Ragged: offsets[]; uniform: i*stride (packets may leave gaps,
// which are streamed but belong to no packet, or overlap).
// A chunk is CH packets, lane l < CH owning packet p0 + l; lanes past the
// chunk (l >= CH) or the batch sit at the chunk's end, so lane 63 always
// holds it.
template <int CH, bool SIDE = true>
__device__ __forceinline__ void seg_load(const BatchArgs &A, const SidePtrs &sp,
                                         uint64_t p0, uint32_t lane, SegChunk &k) {
  const uint64_t n = A.n;
  const uint64_t i = p0 + lane;
  const uint64_t ce = p0 < n ? (n - p0 < (uint64_t)CH ? n : p0 + CH) : n;  // chunk end (packets)
  const bool own = lane < (uint32_t)CH && i < n;
  // ragged: two (clamped) offset loads; uniform: arithmetic, with lanes past
  // the chunk at its end (its last packet's end)
  const uint64_t last = p0 < n ? ce - 1u : 0u;
  const uint64_t uy = (own ? i : last) * A.stride + A.len;
  const uint64_t *offs = A.offsets ? A.offsets : (const uint64_t *)g_side_zero;
  const uint64_t ry = offs[A.offsets ? (own ? i + 1 : ce) : 0];
  const uint64_t rx = offs[A.offsets ? (own ? i : ce) : 0];
  k.ox = A.offsets ? rx : (own ? i * A.stride : uy);
  k.oy = A.offsets ? ry : uy;
  if (SIDE) k.sd = load_side(sp, own ? i : n - 1);  // b0/xe: seg_geom
}


// Wave-uniform geometry of a loaded chunk starting at packet p0 (waits for
// its offsets). No such chunk: an empty range, so its loads are all masked.
// line128: the tiles start at the 128-byte line holding the chunk's first byte
// (the in-place writer's whole-line write-back, k_seg), unless that line begins
// before the batch; else at its dword. The bytes in front are loaded but lie
// before every point, and the line was fetched for the previous chunk anyway.
//
// Out-of-contract chunks (device ragged batches, whose offsets the host never
// reads): a packet whose offsets decrease or whose length exceeds lim, the
// mode's limit (include/yucsum.h), or which ends past the batch's end
// (data + offsets[n], what the call may touch).
//  - The writing kinds (each = true: TX, TXW, DG) test every packet of the
//    chunk, wave-uniformly, on the offsets already loaded, and the chunk's end
//    against the batch's (in-chunk order then puts every packet before it). A
//    chunk holding such a packet gets xe = 0: it streams nothing (its results
//    are unspecified) and stores no field (k_seg's epilogue stores only for
//    xe > 0, which loses nothing: an in-contract chunk with xe == 0 holds only
//    empty packets).
//    Every other chunk lies back to back from its first offset, each packet
//    within the limit, so its positions are exact (< 64 x 65536 bytes: the
//    32-bit positions never wrap).
//  - The read-only kinds (plain, RX) only bound the chunk's span to what CH
//    in-contract packets can cover, so a chunk's time is bounded whatever the
//    offsets say (a decreasing chunk end would wrap xe); a packet out of
//    contract gets an unspecified result, its neighbours stay exact.
__device__ __forceinline__ void seg_geom(uint64_t data, uint64_t n, uint64_t p0, SegChunk &k,
                                         uint32_t, bool ragged, uint32_t lim, bool each, uint32_t ch,
                                         uint64_t end, bool line128 = false) {
  if (p0 >= n) {
    k.b0 = data & ~3ull;
    k.xe = 0;
    return;
  }
  const uint64_t s = data + readlane64(k.ox, 0);
  const uint64_t e = data + readlane64(k.oy, 63);  // lane 63's end = the chunk end
  const uint64_t l = s & ~127ull;
  k.b0 = line128 && l >= (data & ~3ull) ? l : s & ~3ull;
  k.xe = e - k.b0;
  // (lanes past the chunk sit at its end: length 0)
  if (ragged && (each ? (__any((int)(k.oy - k.ox > (uint64_t)lim)) != 0 || e > end)
                      : k.xe > (uint64_t)ch * lim + 131u))  // (+ b0's up to 131 bytes in front)
    k.xe = 0;
}

// The TX kind (UDP / TCP / ICMP fields: packets <= 65535 bytes, so a chunk spans
// < 4.2 MB) keeps a loaded chunk in fewer registers, which its in-place
// write-back needs: each lane holds only the low dword of its packet's end
// offset, and the chunk's first offset is one 8-byte value all lanes load alike
// (read to SGPRs by seg_geom). A lane's start is its left neighbour's end
// (ragged batches lie back to back) or i * stride (uniform); every position and
// length is a 32-bit difference from the first offset. Per chunk in flight: 3
// VGPRs instead of 4 (two 64-bit offsets).
struct SegChunk32 {
  uint32_t ey;  // low dword of this lane's packet end (lanes past the batch or
                // the chunk: the chunk end)
  uint32_t eh;  // its high dword (ragged; dead once seg_geom has checked the chunk)
  uint64_t s0;  // the chunk's first offset (ragged: offsets[p0]; uniform: p0 * stride)
  uint64_t b0;  // address the chunk's tiles start at (wave-uniform, see seg_geom)
  uint64_t xe;  // chunk end relative to b0 (wave-uniform)
  Side sd;
};

template <int CH, bool SIDE = true>
__device__ __forceinline__ void seg_load(const BatchArgs &A, const SidePtrs &sp,
                                         uint64_t p0, uint32_t lane, SegChunk32 &k) {
  const uint64_t n = A.n;
  const uint64_t i = p0 + lane;
  const uint64_t ce = p0 < n ? (n - p0 < (uint64_t)CH ? n : p0 + CH) : n;
  const bool own = lane < (uint32_t)CH && i < n;
  const uint64_t last = p0 < n ? ce - 1u : 0u;
  const uint64_t *offs = A.offsets ? A.offsets : (const uint64_t *)g_side_zero;
  const uint64_t ry = offs[A.offsets ? (own ? i + 1 : ce) : 0];
  const uint64_t r0 = offs[A.offsets ? (p0 < n ? p0 : n) : 0];
  k.ey = A.offsets ? (uint32_t)ry : (uint32_t)((own ? i : last) * A.stride + A.len);
  k.eh = (uint32_t)(ry >> 32);
  k.s0 = A.offsets ? r0 : (p0 < n ? p0 : 0u) * A.stride;
  if (SIDE) k.sd = load_side(sp, own ? i : n - 1);
}

// (the same checks, on the 64-bit ends: a lane's start is its left neighbour's
// end, lane 0's the chunk's first offset)
__device__ __forceinline__ void seg_geom(uint64_t data, uint64_t n, uint64_t p0, SegChunk32 &k,
                                         uint32_t lane, bool ragged, uint32_t lim, bool, uint32_t,
                                         uint64_t end, bool line128 = false) {
  if (p0 >= n) {
    k.b0 = data & ~3ull;
    k.xe = 0;
    k.s0 = 0;
    return;
  }
  const uint64_t s0 = uniform64(k.s0);
  k.s0 = s0;
  const uint64_t s = data + s0;
  const uint64_t l = s & ~127ull;
  k.b0 = line128 && l >= (data & ~3ull) ? l : s & ~3ull;
  k.xe = (uint64_t)((uint32_t)__builtin_amdgcn_readlane((int)k.ey, 63) - (uint32_t)s0) + (s - k.b0);
  if (ragged) {
    const uint64_t ye = ((uint64_t)k.eh << 32) | k.ey;
    const uint64_t yl = shfl64(ye, lane ? lane - 1u : 0u);
    const uint64_t c1 = readlane64(ye, 63);  // the chunk end
    if (__any((int)(ye - (lane ? yl : s0) > (uint64_t)lim)) || data + c1 > end) k.xe = 0;
  }
}

// This lane's packet as (position relative to b0, length).
template <int CH>
__device__ __forceinline__ void seg_xlen(const BatchArgs &A, const SegChunk &k, uint32_t,
                                         uint64_t, uint64_t &x, uint64_t &len) {
  x = (uint64_t)(uintptr_t)A.data + k.ox - k.b0;
  len = k.oy - k.ox;
}

template <int CH>
__device__ __forceinline__ void seg_xlen(const BatchArgs &A, const SegChunk32 &k, uint32_t lane,
                                         uint64_t p0, uint32_t &x, uint32_t &len) {
  const uint32_t h = (uint32_t)((uint64_t)(uintptr_t)A.data + k.s0 - k.b0);  // bytes before the chunk
  const uint32_t s0 = (uint32_t)k.s0;
  uint32_t ox;
  if (A.offsets) {  // back to back: the left neighbour's end
    const uint32_t l = (uint32_t)__shfl((int)k.ey, (int)(lane ? lane - 1u : 0u), 64);
    ox = lane ? l : s0;
  } else {  // lanes past the batch sit at the chunk end (ey)
    const bool own = lane < (uint32_t)CH && p0 + lane < A.n;
    ox = own ? (uint32_t)((p0 + lane) * A.stride) : k.ey;
  }
  x = ox - s0 + h;
  len = k.ey - ox;
}

// Loads of tile t (bytes [t*T, t*T + T) past b0) of a chunk ending xe past
// b0. One call site with selected arguments and a compile-time load policy:
// no load sits in a branch, so the next tile's loads stay in flight while the
// current one is summed. (The one 128-byte line two neighbouring chunks share
// is fetched by both: <= 2% of a chunk of 64 packets >= 40 bytes.)
template <int U, bool NTL>
__device__ __forceinline__ void seg_fetch(uint64_t b0, uint64_t xe, uint64_t t, uint32_t lane,
                                          uint64_t end, uint4 (&c)[U]) {
  constexpr uint32_t T = 64u * 16u * U;
  const uint64_t tb = t * T;
  const __amdgpu_buffer_rsrc_t r = rsrc_at(uniform64(b0 + tb), end);
  const uint64_t rem = xe > tb ? xe - tb : 0u;
  const uint32_t lim = rem < T ? (uint32_t)rem : T;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint32_t cr = 16u * (lane + 64u * (uint32_t)u);
    c[u] = bld16(r, cr < lim ? cr : kOOB, NTL);
  }
}

// Sum of the first r (0..15) bytes of a 16-byte chunk: LE halves (sad_u16)
// or plain bytes (sad_u8).
template <bool BYTES>
__device__ __forceinline__ uint32_t seg_part(const uint4 &d, uint32_t r) {
  const uint32_t w = r >> 2;
  const uint32_t mk = (1u << (8u * (r & 3u))) - 1u;
  const uint32_t v[4] = {d.x, d.y, d.z, d.w};
  uint32_t acc = 0;
#pragma unroll
  for (uint32_t j = 0; j < 4; ++j) {
    const uint32_t x = j < w ? v[j] : (j == w ? (v[j] & mk) : 0u);
    acc = BYTES ? __builtin_amdgcn_sad_u8(x, 0u, acc) : sad(x, acc);
  }
  return acc;
}

// P (or T, BYTES) at tile offset q from the parked tile: the exclusive prefix at
// q's 8-byte half chunk (pre2: two per 16-byte chunk, at its start and middle)
// plus the bytes of that half chunk before q. One 4-byte and one 8-byte LDS read
// and ~10 VALU (a 16-byte chunk prefix needed the 16 bytes and twice the VALU).
template <bool BYTES>
__device__ __forceinline__ uint32_t seg_point(const uint32_t *pre2, const uint2 *half, uint32_t q) {
  const uint32_t h = q >> 3, r = q & 7u;
  const uint2 d = half[h];
  const uint32_t mk = (1u << (8u * (r & 3u))) - 1u;
  const uint32_t lo = r >= 4u ? d.x : (d.x & mk);
  const uint32_t hi = r >= 4u ? (d.y & mk) : 0u;
  return BYTES ? __builtin_amdgcn_sad_u8(hi, 0u, __builtin_amdgcn_sad_u8(lo, 0u, pre2[h]))
               : sad(hi, sad(lo, pre2[h]));
}

// One point of a lane: position x (relative to b0), and P / T at x once the
// tile holding x has gone by.
template <typename Pos>
struct SegPt {
  Pos x;
  uint32_t p, t;
};

// RX verification (YU_MODE_VERIFY_RX): the IPv4 header of a received packet
// fixes two more points — the header end and the transport end — and the
// pseudo-header. Its first 20 bytes (up to 6 dwords from floor4(start)) are
// gathered from the tiles' LDS copies as they go by (a header may straddle
// two tiles), then parsed.
struct SegRx {
  uint32_t h[6];    // header window dwords
  uint32_t need;    // mask of the window dwords still to gather (0: parsed)
  uint32_t flags;   // YU_RX_* bits known at parse time
  uint32_t pseudo;  // LE-free big-endian word sum of src, dst, proto, length
  uint32_t proto;
  uint32_t ipf;     // TX_DATAGRAM: LE sum of the IPv4 checksum field's bytes
  uint32_t hl;      // TX_DATAGRAM: header length (0 outside the contract)
  uint32_t fo;      // TX_DATAGRAM: transport field offset in the packet (0: none)
  uint32_t h20;     // k_seg: the header is the plain 20 bytes (IHL 5) of a valid packet
  uint32_t hsum;    // k_seg: then the address-ordered LE sum of those 20 bytes
  uint32_t tnext;   // k_seg, ragged: TotalLength() == len, so the transport end is
                    // the next lane's start point (no point of its own)
};

// TX_DATAGRAM on a parsed header (rx_parse): the datagram is in contract when
// 20 <= HeaderLength() <= TotalLength() <= len; its transport field exists
// when the protocol is UDP / TCP / ICMP and the segment holds its header.
// Returns (and records in rx.fo) the transport field offset from the packet
// start (0: none), and records the IPv4 field's bytes 10 and 11 as the
// address-ordered LE sum they add to (byte 10 is a low byte when the packet
// starts at an even address) for subtraction.
__device__ __forceinline__ uint32_t dg_parse(SegRx &rx, uint32_t sh, uint32_t hl, uint32_t tl) {
  const bool ok = !(rx.flags & YU_RX_INVALID) && hl >= 20u;
  rx.hl = ok ? hl : 0u;
  const uint32_t w2 = __builtin_amdgcn_alignbyte(rx.h[3], rx.h[2], sh);  // bytes 8..11 (sh 0: h[2])
  const uint32_t f = w2 >> 16;
  rx.ipf = (sh & 1u) ? ((f >> 8) | ((f & 0xFFu) << 8)) : f;
  const uint32_t fo = l4_field(rx.proto);
  rx.fo = ok && fo && tl - hl >= l4_min(rx.proto) ? hl + fo : 0u;
  return rx.fo;
}

// A 16-bit field value stored big-endian (binary.BigEndian.PutUint16).
__device__ __forceinline__ void put_be16(uint8_t *q, uint32_t r) {
  if (((uintptr_t)q & 1u) == 0) {
    *(uint16_t *)q = (uint16_t)(((r >> 8) | (r << 8)) & 0xFFFFu);
  } else {
    q[0] = (uint8_t)(r >> 8);
    q[1] = (uint8_t)r;
  }
}

// Parse the gathered header of a packet of length len starting sh = start&3
// bytes into h[0] (header/ipv4.go:91-118,126-138). Returns the header and
// total lengths through hl/tl.
__device__ __forceinline__ void rx_parse(SegRx &rx, uint32_t sh, uint64_t len, uint32_t &hl,
                                         uint32_t &tl) {
  // bytes 4j..4j+3 of the header (v_alignbyte with sh 0 returns h[j] itself)
  uint32_t w[5];
#pragma unroll
  for (int j = 0; j < 5; ++j)
    if (j != 1) w[j] = __builtin_amdgcn_alignbyte(rx.h[j + 1], rx.h[j], sh);
  hl = (w[0] & 0xFu) * 4u;                                // HeaderLength()
  tl = ((w[0] >> 8) & 0xFF00u) | (w[0] >> 24);            // TotalLength(), BE
  const uint32_t proto = (w[2] >> 8) & 0xFFu;             // Protocol()
  const bool valid = hl <= tl && tl <= len;               // IsValid (len >= 20 checked)
  // The usual 20-byte header is wholly in registers: its sum in the order of
  // the stream's LE prefix sums (byte 0 is a low byte when the packet starts
  // at an even address), so k_seg needs no point at the header end.
  // Summed straight from the address-aligned window dwords, whose 16-bit halves
  // already weigh each byte by its address parity: dword 0 less the sh bytes
  // before the start, dword 5 only those sh bytes' counterparts past byte 20.
  const uint32_t head = (1u << (8u * sh)) - 1u;
  uint32_t hs = sad(rx.h[0] & ~head, 0u);
#pragma unroll
  for (int j = 1; j < 5; ++j) hs = sad(rx.h[j], hs);
  rx.hsum = sad(rx.h[5] & head, hs);
  rx.h20 = valid && hl == 20u;
  const bool l4 = valid && (proto == 6u || proto == 17u || proto == 1u);
  rx.flags = valid ? 0u : YU_RX_INVALID;
  if (l4) rx.flags |= YU_RX_L4;
  rx.proto = proto;
  // PseudoHeaderChecksum(proto, src, dst) + BE16(len(payload))
  // (checker/checker.go:80-88); ICMP has none (network/ipv4/icmp.go:36-45)
  uint32_t ph = sadperm(w[3], kSelSwap, 0u);
  ph = sadperm(w[4], kSelSwap, ph);
  rx.pseudo = proto == 1u ? 0u : ph + proto + ((tl - hl) & 0xFFFFu);
  if (!valid) hl = tl = 0;
}

// Waves that take part in a k_seg launch. The grid is sized for large
// packets (many tiles per 64-packet chunk). When a ragged batch's packets
// average under kSegSmallMean bytes, a chunk is one or two tiles, and a wave
// that handles a single chunk spends its life waiting on two dependent loads
// (offsets, then bytes). So only A.small_waves waves (3 blocks per CU) work,
// each streaming several chunks with the next chunk's loads in flight; the
// other waves exit at once. The mean comes from two scalar loads of the
// offsets, which the host cannot read without a device synchronisation.
// Measured (kbench, round 1): U{40..200} 33 -> 25.5 us, U{40..600} 61 -> 58 us,
// but U{40..1000} 91 -> 93 us and U{64..1500} 127 -> 131 us, so the cut is a
// 400-byte mean.
constexpr uint64_t kSegSmallMean = 400;

typedef const __attribute__((address_space(4))) uint64_t c_u64;

__device__ __forceinline__ uint64_t seg_waves(const BatchArgs &A) {
  const uint64_t all = (uint64_t)gridDim.x * (blockDim.x >> 6);
  if (!A.offsets || A.small_waves == 0 || A.small_waves >= all) return all;
  c_u64 *o = (c_u64 *)A.offsets;  // read-only here: scalar loads
  const uint64_t bytes = o[A.n] - o[0];
  return bytes < kSegSmallMean * A.n ? (uint64_t)A.small_waves : all;
}

// Kinds of k_seg by the points a lane evaluates (compile-time, so a kind
// carries no code or registers for the others): plain (RAW / VERIFY_TCP /
// VERIFY_UDP: start and end), TX (UDP / TCP / ICMP: + the checksum field's
// two ends), RX (VERIFY_RX: + header and transport ends), DG (TX_DATAGRAM:
// RX's points; the IPv4 field comes off the parsed header's registers and
// the transport field's two bytes are read from the tile that holds them).
constexpr int kSegPlain = 0, kSegTx = 1, kSegRx = 2, kSegDg = 3;
// TXW: the TX kind writing ragged batches in place with the whole-line write-back
// (32-bit chunk loads, the park fused into the scan: the registers the
// write-back needs; TX itself keeps the layout that serves its result-array
// form best, 26.1 vs 26.8 us on kbench 8)
constexpr int kSegTxW = 4;

// (the DG kind asks for at least 3 waves per SIMD, which it would otherwise
// miss by a few VGPRs; the other kinds are left alone)
template <int U, int NT, int K, int CH = 64>
__global__ __launch_bounds__(256, K == kSegDg ? 3 : 1) void k_seg(BatchArgs A) {
  constexpr bool DG = K == kSegDg;
  constexpr bool RX = K == kSegRx || DG;  // parses each packet's IPv4 header
  constexpr bool TXW = K == kSegTxW;
  constexpr bool tx = K == kSegTx || TXW;
  constexpr bool FB = tx || DG;                 // a field whose bytes are read from the tile
  constexpr bool FILLK = FB;                    // a kind that may write fields (seg_geom)
  constexpr int NP = K == kSegRx || DG ? 4 : 2;  // point slots in use
  constexpr uint32_t T = 64u * 16u * U;
  constexpr uint32_t NC = 64u * U;  // chunks per tile
  __shared__ uint4 s_data[4][NC];   // the tile's bytes
  // exclusive prefixes per 16-byte chunk (plain kind: L, then T) or per 8-byte half
  // chunk (the others, seg_point)
  __shared__ uint32_t s_pre[4][K == kSegPlain ? NC : 2 * NC];
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t wave = grid_wave(A.xcd);
  const uint64_t nwave = seg_waves(A);
  const int mode = A.mode;
  const uint32_t fld = mode_field(mode);
  const SidePtrs sp = side_ptrs(A);
  const uint64_t data = (uint64_t)(uintptr_t)A.data;
  const uint64_t end = A.offsets ? data + A.offsets[A.n] : A.end;
  const uint32_t *s_dw = (const uint32_t *)s_data[wid];
  const bool contig = A.offsets != nullptr;  // ragged: packets back to back
  // TXW kind (writing a ragged batch in place): the fields go into the parked
  // last tile of each chunk and its whole 128-byte lines are stored back with
  // non-temporal stores. See the chunk epilogue.
  const bool wbk = TXW && A.fill && contig;
  // a packet's length limit (include/yucsum.h); a chunk holding a longer one is
  // out of contract (seg_geom). Only the plain kind takes RAW packets.
  const uint32_t lim = K == kSegPlain && mode == YU_MODE_RAW ? YU_MAX_RAW_LEN : YU_MAX_TRANSPORT_LEN;
  // Positions relative to the chunk's b0: 64-bit for the plain kind (RAW packets
  // up to YU_MAX_RAW_LEN), 32-bit for the TX / RX / DG kinds, whose packets are
  // at most 65535 bytes (include/yucsum.h), so a 64-packet chunk spans < 4.2 MB
  // (uniform batches with sparser strides take k_loop_rx, pick_uniform). Half the
  // VALU work on every point test and offset.
  using Pos = typename std::conditional<K == kSegPlain, uint64_t, uint32_t>::type;
  // CH < 64: lane CH holds no packet but sits at the chunk's end, so its start
  // point is the chunk's end point and every packet's end is its successor's start
  constexpr bool kMarker = CH < 64;
  // points from half-chunk prefixes (seg_point): the 32-bit kinds; the plain
  // kind's registers (exact path) leave no room for the halves' sums
  constexpr bool HP = K != kSegPlain;
  constexpr Pos kNoPt = ~(Pos)0;             // a point slot not in use

  uint64_t ch = wave;
  if (wave >= nwave || ch * CH >= A.n) return;
  using Chunk = typename std::conditional<TXW, SegChunk32, SegChunk>::type;
  Chunk cur, nxt;
  seg_load<CH, !RX>(A, sp, ch * CH, lane, cur);
  seg_load<CH, !RX>(A, sp, (ch + nwave) * CH, lane, nxt);
  seg_geom(data, A.n, ch * CH, cur, lane, contig, lim, FILLK, CH, end, wbk);

  // per-chunk state
  SegPt<Pos> pt[4];  // start, end, then (RX, DG) header and transport end
  SegRx rx;
  // A header window that starts 4-aligned and crosses two tiles never gathers
  // h[5] (its bytes lie past the 20-byte header), yet rx_parse reads it under a
  // zero mask: give it a defined value once, not per chunk.
#pragma unroll
  for (int j = 0; j < 6; ++j) rx.h[j] = 0u;
  // TX, DG: the checksum field's next unread byte (kNoPt: none or done; DG: the
  // transport field), the bytes of it still to read (2, or 1 when the field
  // straddles two tiles) and the address-ordered LE sum of those read:
  // P(field end) - P(field start) without two more point evaluations per tile
  Pos fx = 0;
  uint32_t fk = 0, fsum = 0;
  bool exact = false;
  uint32_t carry_l = 0, carry_t = 0;
  typename std::conditional<TXW, uint32_t, uint64_t>::type plen = 0;  // this lane's packet length
  auto begin_chunk = [&](const Chunk &k, uint64_t p0) __attribute__((always_inline)) {
    typename std::conditional<TXW, uint32_t, uint64_t>::type x64, len;
    seg_xlen<CH>(A, k, lane, p0, x64, len);
    plen = len;
    const Pos x = (Pos)x64;
    const Pos y = x + (Pos)len;
    pt[0].x = x;
    // ragged packets lie back to back: P(end) is the next lane's P(start), so
    // only lane 63 evaluates an end point (the chunk end); RX needs none
    pt[1].x = RX || (contig && (kMarker || lane != 63u)) ? kNoPt : y;
    if (tx) {  // the checksum field, when the packet holds it
      const bool f = fld + 2u <= len;
      fx = f ? x + fld : kNoPt;
      fk = f ? 2u : 0u;
      fsum = 0u;
    }
    if (RX) {  // header and transport ends, once the header is parsed
      const uint32_t sh = (uint32_t)x & 3u;
      rx.need = len >= 20u ? (1u << (((19u + sh) >> 2) + 1u)) - 1u : 0u;
      // an unparsed packet (len < 20) reports only these; rx_parse sets the rest
      rx.flags = YU_RX_INVALID;
      rx.hl = rx.fo = rx.tnext = 0u;
      pt[2].x = pt[3].x = kNoPt;
      if (DG) {
        pt[2].x = pt[3].x = fx = kNoPt;
        fk = fsum = 0u;
      }
    }
#pragma unroll
    for (int i = 0; i < NP; ++i) pt[i].p = pt[i].t = 0u;
    exact = K == kSegPlain && mode == YU_MODE_RAW && __any((int)(len > kLEMax));
    carry_l = carry_t = 0u;
  };
  begin_chunk(cur, ch * CH);

  uint64_t t = 0;
  // One tile: issue the loads of the next item into cn, then sum c.
  // Returns true when the wave has no next item.
  auto step = [&](const uint4 (&c)[U], uint4 (&cn)[U]) __attribute__((always_inline)) -> bool {
    // the chunk's tiles cover [0, xe); a point at a tile's end (xe itself,
    // when tile-aligned) takes the running sums after that tile
    const bool last = t * T + T >= cur.xe;  // wave-uniform
    // The wave's next loads go out at raised priority, ahead of the other waves'
    // sums on its SIMD, so they are in flight sooner (small ragged RX 26.6 -> 26.3
    // us, U{64..1500} 129.0 -> 127.1; no gain for k_small, a loss for k_lane:
    // profiles/r04/kbench_ab_r04p_setprio.log)
    __builtin_amdgcn_s_setprio(2);
    Chunk nn;  // the chunk after next: its loads go out before this
                  // step's tile loads, so waiting on them never waits on those
    if (last) {
      seg_geom(data, A.n, (ch + nwave) * CH, nxt, lane, contig, lim, FILLK, CH, end, wbk);
      seg_load<CH, !RX>(A, sp, (ch + 2u * nwave) * CH, lane, nn);  // (RX, DG: no side data)
    }
    seg_fetch<U, NT != 0>(last ? nxt.b0 : cur.b0, last ? nxt.xe : cur.xe, last ? 0u : t + 1u, lane,
                          end, cn);
    __builtin_amdgcn_s_setprio(0);


    const Pos tb = (Pos)(t * T);
    bool here = false;  // a packet boundary (or header) lies in this tile
#pragma unroll
    for (int i = 0; i < NP; ++i)
      if (!(RX && i == 1)) here |= pt[i].x - tb < T;  // (RX and DG have no end point)
    if (FB) here |= fx - tb < T;
    if (RX) {  // a header window [floor4(start), +24) still being gathered
      const Pos hs = pt[0].x & ~(Pos)3;
      here |= rx.need != 0u && hs < tb + T && hs + 24u > tb;
    }
    const bool park = __any((int)here);
    // chunk sums, address-ordered exclusive prefixes (DPP scan per u). The TX
    // kind parks each column as its scan completes (FUSE: no prefix array
    // live across the scan, registers its in-place write-back needs); the
    // others after the scan
    constexpr bool FUSE = TXW;
    // chunk prefix; HP: also the chunk's first half's sum (half-chunk prefixes)
    uint32_t pl[U], ph[U], ptt[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      ph[u] = sad(c[u].y, sad(c[u].x, 0u));
      const uint32_t s = sad(c[u].w, sad(c[u].z, ph[u]));
      const uint32_t inc = group_total<64>(s);
      pl[u] = carry_l + inc - s;
      carry_l += (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
      if (FUSE && park) {
        s_data[wid][u * 64 + lane] = c[u];
        ((uint2 *)s_pre[wid])[u * 64 + lane] = make_uint2(pl[u], pl[u] + ph[u]);
      }
    }
    if (exact) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        uint32_t s = __builtin_amdgcn_sad_u8(c[u].x, 0u, 0u);
        s = __builtin_amdgcn_sad_u8(c[u].y, 0u, s);
        s = __builtin_amdgcn_sad_u8(c[u].z, 0u, s);
        s = __builtin_amdgcn_sad_u8(c[u].w, 0u, s);
        const uint32_t inc = group_total<64>(s);
        ptt[u] = carry_t + inc - s;
        carry_t += (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
      }
    }
    if (park) {
      if (!FUSE) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          s_data[wid][u * 64 + lane] = c[u];
          if (HP)
            ((uint2 *)s_pre[wid])[u * 64 + lane] = make_uint2(pl[u], pl[u] + ph[u]);
          else
            s_pre[wid][u * 64 + lane] = pl[u];
        }
      }
      __builtin_amdgcn_wave_barrier();
      bool parsed = false;
      if (RX && rx.need) {  // gather header dwords held by this tile, parse
        const Pos q0 = (pt[0].x & ~(Pos)3) - tb;
        if (q0 <= (Pos)(T - 24u)) {
          // the whole 24-byte window lies in this tile (q0 wraps past T when
          // the window began in an earlier one): six reads, no bookkeeping
          const uint32_t d = (uint32_t)q0 >> 2;
#pragma unroll
          for (int j = 0; j < 6; ++j) rx.h[j] = s_dw[d + (uint32_t)j];
          rx.need = 0u;
        } else {  // a window across two tiles: the dwords this one holds
#pragma unroll
          for (int j = 0; j < 6; ++j) {
            const Pos q = q0 + 4u * (uint32_t)j;
            if (((rx.need >> j) & 1u) && q < T) {
              rx.h[j] = s_dw[(uint32_t)q >> 2];
              rx.need &= ~(1u << j);
            }
          }
        }
        if (rx.need == 0u) {
          uint32_t hl, tl;
          rx_parse(rx, (uint32_t)pt[0].x & 3u, plen, hl, tl);
          // a well-formed datagram fills its packet: in a ragged chunk its
          // transport end is the next lane's start (the marker lane's, for the
          // chunk's last packet), already evaluated; when every lane's is, the
          // wave skips the transport-end slot altogether
          rx.tnext = contig && kMarker && tl == (uint32_t)plen ? 1u : 0u;
          if (DG) {
            // in contract HeaderLength() >= 20: every point lies at or past
            // byte 20, so never in a tile that has gone by
            const uint32_t fo = dg_parse(rx, (uint32_t)pt[0].x & 3u, hl, tl);
            if (rx.hl) {
              pt[2].x = rx.h20 ? kNoPt : pt[0].x + hl;
              pt[3].x = rx.tnext ? kNoPt : pt[0].x + tl;
            }
            if (fo) {
              fx = pt[0].x + fo;
              fk = 2u;
            }
          } else {
            pt[2].x = rx.h20 ? kNoPt : pt[0].x + hl;
            pt[3].x = rx.tnext ? kNoPt : pt[0].x + tl;
          }
          parsed = true;
        }
      }
#pragma unroll
      for (int i = 0; i < NP; ++i) {
        const Pos q = pt[i].x - tb;
        if (!(RX && i == 1) && q < T) {
          if (HP) {
            pt[i].p = seg_point<false>(s_pre[wid], (const uint2 *)s_data[wid], (uint32_t)q);
          } else {
            const uint32_t k = (uint32_t)q >> 4;
            pt[i].p = s_pre[wid][k] + seg_part<false>(s_data[wid][k], (uint32_t)q & 15u);
          }
        }
      }
      if (FB) {  // the field's bytes, weighted by address parity
        const Pos q = fx - tb;
        if (q < T) {
          const uint8_t *sb = (const uint8_t *)s_data[wid];
          const uint32_t b = sb[q];
          fsum += (q & 1u) ? b << 8 : b;
          if (fk == 2u && q + 1u < T) {
            const uint32_t b1 = sb[q + 1u];
            fsum += (q & 1u) ? b1 : b1 << 8;
          }
          const bool split = fk == 2u && q + 1u == T;  // the field's second byte opens the next tile
          fk = split ? 1u : 0u;
          fx = split ? fx + 1u : kNoPt;
        }
      }
      if (RX && !DG && parsed) {
        // A header straddling two tiles is parsed in the second, but a header
        // or total length under 20 bytes (IsValid accepts IHL 0..4) can put
        // its point in the first, whose bytes have gone by. Such a point lies
        // inside the gathered 24-byte window: P(point) = P(start) + the LE sum
        // of the window bytes in between, taken from the registers.
        const uint32_t sh = (uint32_t)pt[0].x & 3u;
#pragma unroll
        for (int i = 2; i < 4; ++i) {
          if (pt[i].x < tb) {
            const uint32_t b = sh + (uint32_t)(pt[i].x - pt[0].x);  // < sh + 20
            uint32_t s = pt[0].p;
#pragma unroll
            for (int j = 0; j < 6; ++j)
              s = sad(rx.h[j] & byte_range_mask(4u * (uint32_t)j, sh, b), s);
            pt[i].p = s;
          }
        }
      }
      __builtin_amdgcn_wave_barrier();
      if (exact) {  // second pass, same buffer: the byte-sum prefixes
#pragma unroll
        for (int u = 0; u < U; ++u) s_pre[wid][u * 64 + lane] = ptt[u];
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int i = 0; i < NP; ++i) {
          const Pos q = pt[i].x - tb;
          if (q < T) {
            const uint32_t k = (uint32_t)q >> 4;
            pt[i].t = s_pre[wid][k] + seg_part<true>(s_data[wid][k], (uint32_t)q & 15u);
          }
        }
        __builtin_amdgcn_wave_barrier();
      }
    }
#pragma unroll
    for (int i = 0; i < NP; ++i)
      if (!(RX && i == 1) && pt[i].x - tb == T) pt[i].p = carry_l;
    if (exact) {
#pragma unroll
      for (int i = 0; i < NP; ++i)
        if (pt[i].x - tb == T) pt[i].t = carry_t;
    }

    if (!last) {
      ++t;
      return false;
    }
    // end sums: the next lane's start (ragged), else this lane's end point
    const int nl = (int)(lane < 63u ? lane + 1u : 63u);
    const uint32_t nx_p = (uint32_t)__shfl((int)pt[0].p, nl, 64);
    const uint32_t nx_t = (uint32_t)__shfl((int)pt[0].t, nl, 64);
    const bool own_end = !contig || (!kMarker && lane == 63u);
    const uint32_t p3 = RX && rx.tnext ? nx_p : pt[3].p;  // P(transport end)
    const uint32_t pe = own_end ? pt[1].p : nx_p;
    const uint32_t te = own_end ? pt[1].t : nx_t;
    const uint64_t p = ch * CH + lane;
    // TX in place (wbk): this lane's field offset in the tile (wf: it has one),
    // its line when stored whole (64: not), its value
    Pos wq = 0;
    bool wf = false;
    uint32_t wl = 64u, wr = 0u;
    // an out-of-contract chunk (xe == 0, seg_geom) stores nothing: no field, no line
    const bool wr_ok = A.fill && cur.xe != 0u;
    const bool wbc = wbk && cur.xe != 0u;
    Pos x0 = 0;  // the chunk's start (wbk: the TX kind, 32-bit)
    if (wbc) x0 = (Pos)(uint32_t)__shfl((int)(uint32_t)pt[0].x, 0, 64);
    if (lane < (uint32_t)CH && p < A.n) {
      const uint32_t odd = (uint32_t)pt[0].x & 1u;
      if (DG) {
        // IPv4 header field: ^Checksum(b[:HeaderLength()]) with the field as 0
        // (network/ipv4/ipv4.go:85-94); transport field: the sender's value
        // over b[HeaderLength():TotalLength()] with its field as 0 and the
        // pseudo header + length from the datagram (sendUDP / sendTCP /
        // sendICMPv4, see include/yucsum.h)
        uint32_t ip = 0u, l4 = 0u;
        const uint32_t p2 = rx.h20 ? pt[0].p + rx.hsum : pt[2].p;  // P(header end)
        if (rx.hl) ip = ~fold32(le_to_be(p2 - pt[0].p - rx.ipf, odd)) & 0xFFFFu;
        if (rx.fo) l4 = ~fold32(le_to_be(p3 - p2 - fsum, odd) + rx.pseudo) & 0xFFFFu;
        if (A.out) {  // out[2p], out[2p + 1]: one 32-bit store when aligned
          if (((uintptr_t)A.out & 3u) == 0u) {
            ((uint32_t *)A.out)[p] = ip | (l4 << 16);
          } else {
            A.out[2u * p] = (uint16_t)ip;
            A.out[2u * p + 1u] = (uint16_t)l4;
          }
        }
        if (wr_ok) {
          uint8_t *pk = A.fill + (cur.b0 + pt[0].x - data);
          if (rx.hl) put_be16(pk + 10u, ip);
          if (rx.fo) put_be16(pk + rx.fo, l4);
        }
      } else if (RX) {
        // header: Checksum(b[:HeaderLength()]) in {0, 0xffff}; transport:
        // pseudo + BE16(len) + segment in {0, 0xffff} (checker/checker.go:32-35,80-92)
        uint32_t r = rx.flags;
        if (!(r & YU_RX_INVALID)) {
          const uint32_t p2 = rx.h20 ? pt[0].p + rx.hsum : pt[2].p;  // P(header end)
          const uint32_t ip = fold32(le_to_be(p2 - pt[0].p, odd));
          if (ip == 0u || ip == 0xFFFFu) r |= YU_RX_IP_OK;
          if (r & YU_RX_L4) {
            const uint32_t l4 = fold32(le_to_be(p3 - p2, odd) + rx.pseudo);
            if (l4 == 0u || l4 == 0xFFFFu) r |= YU_RX_L4_OK;
          }
        }
        if (A.out) A.out[p] = (uint16_t)r;
      } else {
        uint32_t v;
        if (exact) {
          const uint32_t L = pe - pt[0].p;
          const uint32_t S = te - pt[0].t;
          const uint32_t b = (L - S) * kInv255;  // odd-address bytes
          const uint32_t a = S - b;              // even-address bytes
          v = odd ? a + (b << 8) : (a << 8) + b;
        } else {
          v = le_to_be(pe - pt[0].p - (tx ? fsum : 0u), odd);
        }
        const uint64_t len = plen;
        uint8_t *pk = wr_ok ? A.fill + (cur.b0 + pt[0].x - data) : nullptr;
        if (tx && wbc && park && fld + 2u <= len) {
          // the field's offset in the parked (last) tile, wrapping below it;
          // its line is stored whole below when the field lies in one line of
          // this tile that holds no byte outside this chunk
          wq = pt[0].x + fld - tb;
          wf = true;
          const Pos ls = wq & ~(Pos)127;
          // (wq wraps for a field in an earlier tile: wq <= T - 2 keeps those out,
          // a field ending right at this tile's start included)
          if (wq <= T - 2u && (wq & 127u) != 127u && tb + ls >= x0 && tb + ls + 128u <= cur.xe) {
            wl = (uint32_t)wq >> 7;
            pk = nullptr;  // no 2-byte store
          }
        }
        const uint32_t r = packet_value(A, v, len, cur.sd);
        if (A.out) A.out[p] = (uint16_t)r;
        wr = r;
        if (pk) store_field(A, r, pk, (uint32_t)(len < 0xFFFFFFFFu ? len : 0xFFFFFFFFu));
      }
    }
    if (tx && wbc && park) {  // wave-uniform: the in-place write-back
      // 1. Every field byte that lies in the tile goes into its parked copy, the
      //    ones left to their 2-byte stores too (same bytes: a line stored whole
      //    that holds one stays right).
      uint8_t *sb = (uint8_t *)s_data[wid];
      if (wf && wq < T) sb[wq] = (uint8_t)(wr >> 8);
      if (wf && wq + 1u < T) sb[wq + 1u] = (uint8_t)wr;  // (wq + 1 == 0: a field from the tile before)
      // 2. The lines holding a field of their own, as a 64-bit mask (T / 128 <= 64 lines).
      const uint64_t m = (uint64_t)wave_or(wl < 32u ? 1u << wl : 0u) |
                         ((uint64_t)wave_or(wl >= 32u && wl < 64u ? 1u << (wl - 32u) : 0u) << 32);
      wave_lds_fence();
      // 3. Those lines from the tile copy, as full-line 16-byte stores (8 lanes
      //    per line, one contiguous KiB per instruction), non-temporal. Memory
      //    then sees whole lines, not one partial write per field.
      const __amdgpu_buffer_rsrc_t wr_r = __builtin_amdgcn_make_buffer_rsrc(
          (void *)(A.fill + (cur.b0 + tb - data)), (short)0, (int)T, 0x00020000);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t k = (uint32_t)u * 64u + lane;
        const uint4 d = s_data[wid][k];
        const uint32_t off = ((m >> (k >> 3)) & 1u) ? 16u * k : kOOB;
        __builtin_amdgcn_raw_buffer_store_b128(u32x4{d.x, d.y, d.z, d.w}, wr_r, (int)off, 0, 2);  // nt
      }
    }
    if ((ch + nwave) * CH >= A.n) return true;
    cur = nxt;
    nxt = nn;
    ch += nwave;
    begin_chunk(cur, ch * CH);
    t = 0;
    return false;
  };

  // ping-pong: the loads of tile i+1 land in the buffer tile i-1 used, so
  // no register copy waits on them
  uint4 ca[U], cb[U];
  seg_fetch<U, NT != 0>(cur.b0, cur.xe, 0, lane, end, ca);
  for (;;) {
    if (step(ca, cb)) break;
    if (step(cb, ca)) break;
  }
}

// ---------------------------------------------------------------------
// k_loop_rx<U, NT>: VERIFY_RX for small bursts, a wave per datagram as in
// k_loop (k_seg's one wave per 64-packet chunk leaves a burst's GPU idle).
// Window 0 holds the header: the wave parses it from lanes 0-1's registers,
// then every dword counts toward the header sum [sh, sh+hl) or the transport
// sum [sh+hl, sh+tl) through byte masks (window coordinates, base floor4 of
// the start). Same checks and result bits as k_seg's RX kind.
// ---------------------------------------------------------------------
template <int U, int NT, bool DG = false>
__global__ __launch_bounds__(256) void k_loop_rx(BatchArgs A) {
  constexpr uint32_t W = 64u * 16u * U;
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t wave = grid_wave(A.xcd);
  const uint64_t nwave = (uint64_t)gridDim.x * (blockDim.x >> 6);
  const uint64_t end = A.offsets ? (uint64_t)(uintptr_t)A.data + A.offsets[A.n] : A.end;
  const Extent ext = batch_extent(A);

  uint64_t p = wave;
  if (p >= A.n) return;
  LoopPkt cur, nxt;
  loop_pkt(A, p, false, cur);
  uint64_t pn = p + nwave;
  loop_pkt(A, pn, false, nxt);
  uint32_t wb = 0;
  uint4 c[U];
  loop_fetch<U, NT>(cur, 0, lane, end, c);
  uint32_t ah = 0, at = 0, hl = 0, tl = 0, fo = 0;
  SegRx rx;
  for (;;) {
    const bool last = wb + W >= cur.eload;  // wave-uniform
    const bool more = !last || pn < A.n;
    uint4 cn[U];
    loop_fetch<U, NT>(last ? nxt : cur, last ? 0u : wb + W, lane, end, cn);
    if (wb == 0) {  // header window dwords 0..5: lane 0's chunk, half of lane 1's
      rx.h[0] = (uint32_t)__builtin_amdgcn_readlane((int)c[0].x, 0);
      rx.h[1] = (uint32_t)__builtin_amdgcn_readlane((int)c[0].y, 0);
      rx.h[2] = (uint32_t)__builtin_amdgcn_readlane((int)c[0].z, 0);
      rx.h[3] = (uint32_t)__builtin_amdgcn_readlane((int)c[0].w, 0);
      rx.h[4] = (uint32_t)__builtin_amdgcn_readlane((int)c[0].x, 1);
      rx.h[5] = (uint32_t)__builtin_amdgcn_readlane((int)c[0].y, 1);
      rx.flags = YU_RX_INVALID;
      rx.pseudo = 0u;
      hl = tl = 0u;
      if (cur.len >= 20u) rx_parse(rx, cur.sh, cur.len, hl, tl);  // IsValid: minimum size
      if (DG) {  // TX_DATAGRAM: the two fields come off by byte masks
        rx.hl = 0u;
        fo = cur.len >= 20u ? dg_parse(rx, cur.sh, hl, tl) : 0u;
        if (!rx.hl) hl = tl = 0u;
      }
    }
    const uint32_t a = cur.sh, b = cur.sh + hl, e = cur.sh + tl;
    // DG: the IPv4 field [10, 12) and the transport field [fo, fo + 2) are
    // left out of the header and transport sums (empty ranges when absent)
    const uint32_t ia = DG && rx.hl ? cur.sh + 10u : 0u, ta = DG && fo ? cur.sh + fo : 0u;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t w[4] = {c[u].x, c[u].y, c[u].z, c[u].w};
      const uint32_t base = wb + 16u * (lane + 64u * (uint32_t)u);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t lo = base + 4u * (uint32_t)j;
        if (DG) {
          ah = sad(w[j] & byte_range_mask(lo, a, b) & ~byte_range_mask(lo, ia, ia + (ia ? 2u : 0u)), ah);
          at = sad(w[j] & byte_range_mask(lo, b, e) & ~byte_range_mask(lo, ta, ta + (ta ? 2u : 0u)), at);
        } else {
          ah = sad(w[j] & byte_range_mask(lo, a, b), ah);
          at = sad(w[j] & byte_range_mask(lo, b, e), at);
        }
      }
    }
    if (last) {
      ah = group_total<64>(ah);
      at = group_total<64>(at);
      if (DG && lane == 63u) {  // TX_DATAGRAM: as k_seg's DG kind
        const uint32_t odd = cur.sh & 1u;
        const uint32_t ip = rx.hl ? ~fold32(le_to_be(ah, odd)) & 0xFFFFu : 0u;
        const uint32_t l4 = fo ? ~fold32(le_to_be(at, odd) + rx.pseudo) & 0xFFFFu : 0u;
        if (A.out) {
          A.out[2u * p] = (uint16_t)ip;
          A.out[2u * p + 1u] = (uint16_t)l4;
        }
        if (uint8_t *pk = fill_at(A, ext, cur.soff, cur.len)) {
          if (rx.hl) put_be16(pk + 10u, ip);
          if (fo) put_be16(pk + fo, l4);
        }
      } else if (lane == 63u) {
        // header: Checksum(b[:HeaderLength()]) in {0, 0xffff}; transport:
        // pseudo + BE16(len) + segment in {0, 0xffff} (checker/checker.go:32-35,80-92)
        uint32_t r = rx.flags;
        if (!(r & YU_RX_INVALID)) {
          const uint32_t odd = cur.sh & 1u;
          const uint32_t ip = fold32(le_to_be(ah, odd));
          if (ip == 0u || ip == 0xFFFFu) r |= YU_RX_IP_OK;
          if (r & YU_RX_L4) {
            const uint32_t l4 = fold32(le_to_be(at, odd) + rx.pseudo);
            if (l4 == 0u || l4 == 0xFFFFu) r |= YU_RX_L4_OK;
          }
        }
        if (A.out) A.out[p] = (uint16_t)r;
      }
      if (!more) break;
      p = pn;
      cur = nxt;
      pn = p + nwave;
      loop_pkt(A, pn, false, nxt);
      wb = 0;
      ah = at = 0u;
    } else {
      wb += W;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) c[u] = cn[u];
  }
}

// ---------------------------------------------------------------------
// Host side: variant selection and launch.
// ---------------------------------------------------------------------
typedef void (*KernelFn)(BatchArgs);

struct Variant {
  const char *name;
  uint32_t window;  // bytes covered per packet step (0 = loop kernel)
  KernelFn fn[3];   // by load policy (bld16): plain, nt, hybrid
  uint32_t G;       // lanes per packet
  uint32_t ppw;     // packets per wave step
  KernelFn fill = nullptr;  // in-place fill instantiation, if it has its own
  uint32_t run = 0;  // packets per wave run (k_small), 0 = ppw
  // k_small without runs (PR = 0), by load policy like fn: the in-place fill,
  // and batches too small to give every wave of the grid a whole run
  KernelFn inter[3] = {nullptr, nullptr, nullptr};
};

// k_small runs of 16 packets per wave (one side-record load and one result
// store per run): config 3 235-246 -> 235-240 us against the interleaved
// mapping (PR = 0; equal on some boxes), 64-packet runs 248; 1M x 768 B 131.5
// -> 122.6, x 3000 B 467.8 -> 450.7; 256K x 768 B 43.8 -> 35.0. The in-place
// fill keeps the interleaved mapping (config 9: 313 vs 328 us with runs), and
// so do batches of fewer than 8 runs per CU (see launch).
// profiles/r02/kbench_ab_k_small_runs.log
constexpr int kSmallRun = 16;
#define YU_SMALL(G, U)                                                                     \
  {"k_small<" #G "," #U ">", 16u * G * U,                                                  \
   {k_small<G, U, 0, kSmallRun>, k_small<G, U, 1, kSmallRun>, k_small<G, U, 2, kSmallRun>}, \
   G, 64u / G, nullptr, kSmallRun,                                                         \
   {k_small<G, U, 0, 0>, k_small<G, U, 1, 0>, k_small<G, U, 2, 0>}}
#define YU_TINY(G, FILL) \
  {"k_tiny<" #G ">", 16u * G, {k_tiny<G, 0>, k_tiny<G, 1>, k_tiny<G, 1>}, G, 64u, FILL}

// k_tiny<8> (113..128 bytes) fills with single field stores: its whole-chunk
// instantiation would spill scalar registers
const Variant kTiny[] = {YU_TINY(4, (k_tiny<4, 1, true>)), YU_TINY(8, nullptr)};

// window = the largest stride a wave step's U KiB hold (64 packets)
#define YU_LANE(U) \
  {"k_lane<" #U ">", 16u * U, {k_lane<U, 0>, k_lane<U, 1>, k_lane<U, 1>}, 1, 64u}
const Variant kLane[] = {YU_LANE(2), YU_LANE(3), YU_LANE(4),
                         YU_LANE(5), YU_LANE(6), YU_LANE(7), YU_LANE(8)};

// Ordered by window; for each window the variant with the most packets per
// wave comes first (amortises the per-packet epilogue over more bytes).
const Variant kSmall[] = {
    YU_SMALL(4, 1),  YU_SMALL(8, 1),  YU_SMALL(8, 2),  YU_SMALL(16, 2),
    YU_SMALL(16, 3), YU_SMALL(16, 4), YU_SMALL(16, 6), YU_SMALL(32, 4),
    YU_SMALL(32, 6), YU_SMALL(64, 4),
};
const Variant kLoopLE = {"k_loop<4,LE>", 0, {k_loop<4, 0, false>, k_loop<4, 1, false>, k_loop<4, 1, false>}, 64, 1};
const Variant kLoopBE = {"k_loop<4,BE>", 0, {k_loop<4, 0, true>, k_loop<4, 1, true>, k_loop<4, 1, true>}, 64, 1};
const Variant kLoopRx = {"k_loop<4,rx>", 0, {k_loop_rx<4, 0>, k_loop_rx<4, 1>, k_loop_rx<4, 1>}, 64, 1};
const Variant kLoopDg = {"k_loop<4,dg>", 0,
                         {k_loop_rx<4, 0, true>, k_loop_rx<4, 1, true>, k_loop_rx<4, 1, true>}, 64, 1};
const Variant kRag = {"k_rag<16,6>", 1536, {k_rag<16, 6, 0>, k_rag<16, 6, 1>, k_rag<16, 6, 2>}, 16, 4};
// plain loads by default: for scattered 32-byte header reads they beat nt
// ones (30.7 vs 32.5 us, kbench 12)
const Variant kHdr = {"k_hdr", 0, {k_hdr<0>, k_hdr<1>, k_hdr<0>}, 64, 64};
// 64 packets per chunk. (63 packets and a marker lane, kMarker, which drops the
// end-point slot: small RX datagrams 27.0 -> 26.6 us, but config 4 703 -> 714 and
// U{64..1500} 127 -> 129 from the 1.6 % more chunks; the 16-packet chunks use it.
// profiles/r03/kbench_ab_kseg_lean.log)
#define YU_SEG(U, K, name) \
  {name, 0, {k_seg<U, 0, K, 64>, k_seg<U, 1, K, 64>, k_seg<U, 1, K, 64>}, 64, 64}
#define YU_SEG16(U, K, name) \
  {name, 0, {k_seg<U, 0, K, 16>, k_seg<U, 1, K, 16>, k_seg<U, 1, K, 16>}, 64, 16}
const Variant kSeg4 = YU_SEG(4, kSegPlain, "k_seg<4>");
const Variant kSeg8 = YU_SEG(8, kSegPlain, "k_seg<8>");
const Variant kSegTx4 = YU_SEG(4, kSegTx, "k_seg<4,tx>");
const Variant kSegTx8 = YU_SEG(8, kSegTx, "k_seg<8,tx>");
const Variant kSegRx4 = YU_SEG(4, kSegRx, "k_seg<4,rx>");
const Variant kSegRx8 = YU_SEG(8, kSegRx, "k_seg<8,rx>");
// 16-packet chunks: 4x the waves for mid-size ragged batches (see pick_ragged)
const Variant kSeg8c16 = YU_SEG16(8, kSegPlain, "k_seg<8,c16>");
const Variant kSegTx8c16 = YU_SEG16(8, kSegTx, "k_seg<8,tx,c16>");
// the TX kinds' in-place form for ragged batches (the whole-line write-back)
const Variant kSegTxW4 = YU_SEG(4, kSegTxW, "k_seg<4,txw>");
const Variant kSegTxW8c16 = YU_SEG16(8, kSegTxW, "k_seg<8,txw,c16>");
const Variant kSegRx8c16 = YU_SEG16(8, kSegRx, "k_seg<8,rx,c16>");
// (no 4 KiB-tile DG kind: datagram batches take the ragged picks, 8 KiB)
const Variant kSegDg8 = YU_SEG(8, kSegDg, "k_seg<8,dg>");
const Variant kSegDg8c16 = YU_SEG16(8, kSegDg, "k_seg<8,dg,c16>");
// In place, from 64K packets on: smaller chunks. The TXW kind at 48 packets (1M UDP
// datagrams U{40..200}: 48.7 -> 46.3 us; U{64..1500} TCP 192.9 -> 190.4: a small
// datagram chunk then fits one 8 KiB tile, so all its fields go out as whole
// lines), TX_DATAGRAM at 40 (U{40..1500}: 204.3 -> 198.7 us). The read-only kinds
// keep 64 (RX U{40..200} 26.5 vs 27.5 at 48 and 30.3 at 40; plain unchanged).
// profiles/r04/kbench_ab_r04v_seg_chunk.log (and r04s/r04t/r04u for 32..60)
#define YU_SEGC(U, K, CH, name) \
  {name, 0, {k_seg<U, 0, K, CH>, k_seg<U, 1, K, CH>, k_seg<U, 1, K, CH>}, 64, CH}
const Variant kSegTxW8c48 = YU_SEGC(8, kSegTxW, 48, "k_seg<8,txw,c48>");
const Variant kSegDg8c40 = YU_SEGC(8, kSegDg, 40, "k_seg<8,dg,c40>");

// The k_seg kind for a mode (not the IPv4 header-only modes).
const Variant &seg_for(bool u8, int mode) {
  if (mode == YU_MODE_VERIFY_RX) return u8 ? kSegRx8 : kSegRx4;
  if (mode == YU_MODE_TX_DATAGRAM) return kSegDg8;
  if (mode_is_tx(mode)) return u8 ? kSegTx8 : kSegTx4;
  return u8 ? kSeg8 : kSeg4;
}

// Ragged kernel choice: the segmented stream sum with 8 KiB tiles, except for
// the IPv4 modes, which read only each packet's header (k_rag's per-packet
// windows). 8 KiB tiles beat 4 KiB ones from ~800-byte packets up (config 4:
// 84.9 vs 83.4 % of peak, U{64..1500}: 80.5 vs 77.7 %) and lose below
// (U{40..200}: 54 vs 61-66 %). Measurement override YU_RAGGED=loop|rag|seg4|seg8.
// Small bursts (n <= kSmallBurst, e.g. a tun read burst on the host path) go to
// k_loop instead: k_seg gives each 64-packet chunk to one wave, which streams
// the chunk's tiles one after another, so a burst of few chunks leaves the GPU
// idle and pays one memory latency per tile. One wave per packet instead
// (tools/kbench KB_N, profiles/r01/kbench_ragged_burst_size.log): 64 packets of
// U{64..1500} 8.6 -> 3.4 us, 1024 of them 10.7 -> 3.8, 2048 jumbo packets
// U{64..9000} 43.2 -> 5.7; at 4096 small packets U{40..200} the two tie (4.7);
// from 16384 packets on k_seg wins on small packets (5.4 vs 11.5). VERIFY_RX
// bursts take k_loop_rx, the same shape.
constexpr uint64_t kSmallBurst = 4096;
// the largest uniform stride k_seg's 32-bit kinds take: 63 strides plus a 65535-byte
// packet and its 3 head bytes stay under 2^31 bytes
constexpr uint64_t kSeg32Stride = ((1ull << 31) - 65535u - 3u) / 63u;
constexpr uint64_t kMidBatch = 65536;

const Variant &pick_ragged(int mode, uint64_t n) {
  static const char *f = yu::tuning_env("YU_RAGGED");
  const bool seg4 = f && strcmp(f, "seg4") == 0;
  const bool rx = mode == YU_MODE_VERIFY_RX;  // only k_seg verifies whole datagrams
  const bool dg = mode == YU_MODE_TX_DATAGRAM;  // and fills both fields of one
  const Variant &loop = rx ? kLoopRx : (dg ? kLoopDg : (mode == YU_MODE_RAW ? kLoopBE : kLoopLE));  // BE: exact past 131072 B
  const Variant &c16 = rx ? kSegRx8c16 : (dg ? kSegDg8c16 : (mode_is_tx(mode) ? kSegTx8c16 : kSeg8c16));
  if (f && strcmp(f, "loop") == 0) return loop;
  if (f && strcmp(f, "rag") == 0 && !rx && !dg) return kRag;
  if (mode_is_ipv4(mode)) return kHdr;  // header-only: one lane per packet
  if (f && strcmp(f, "seg16") == 0) return c16;
  if (n <= kSmallBurst && !f) return loop;
  // up to 64K packets: 16-packet chunks, 4x the waves (U{64..1500}: 8192
  // packets 11.2 -> 6.3 us, 32768 11.7 -> 8.7; U{40..200} 5.1 -> 4.4; jumbo
  // 44.2 -> 17.0; VERIFY_RX 13.3 -> 7.1); from 65536 on 64-packet chunks win
  // again (13.1 vs 14.7 us; profiles/r01/kbench_kseg_chunk16_sweep.log)
  if (n < kMidBatch && !f) return c16;
  return seg_for(!seg4, mode);
}

// Tuning override (measurement only, read under YU_TUNING=1: yu::tuning_env):
// YU_VARIANT=<name> forces a k_small variant whenever it covers the shape.
const char *forced_variant() {
  static const char *v = yu::tuning_env("YU_VARIANT");
  return v;
}

const Variant &pick_uniform(uint64_t base, uint64_t stride, uint32_t len,
                            uint64_t n, int mode) {
  const uint64_t need = mode_is_ipv4(mode) ? (len < 60u ? len : 60u) : len;
  // the window starts at floor4(start): up to 3 extra bytes in front
  const bool aligned4 = ((base | (n > 1 ? stride : 0)) & 3u) == 0;
  const uint64_t span = need + (aligned4 ? 0 : 3);
  // lane window offsets are 32-bit: (64/G - 1) strides + the window
  auto fits = [&](const Variant &v) {
    return span <= v.window && v.ppw * stride + v.window < kOOB;
  };
  // k_tiny: no junk bytes (4-aligned starts, no TX field, no IPv4 header walk)
  const bool tiny_ok = aligned4 && !mode_is_ipv4(mode) && mode != YU_MODE_VERIFY_RX &&
                       mode != YU_MODE_TX_DATAGRAM;
  // k_lane: the same modes, one wave step = 64 whole strides in LDS, so only
  // where gaps between packets waste at most half the bytes it loads
  auto lane_fits = [&](const Variant &v) {
    return tiny_ok && (stride & 3u) == 0 && len >= 1u && len <= stride && stride <= v.window &&
           2u * stride <= 3u * (uint64_t)len;
  };
  if (mode == YU_MODE_VERIFY_RX || mode == YU_MODE_TX_DATAGRAM) {
    // k_seg's RX / DG kinds keep positions in 32 bits: a 64-packet chunk must
    // span less than 2 GiB, so sparser uniform batches take a wave per datagram
    if (n > 1 && stride > kSeg32Stride) return mode == YU_MODE_VERIFY_RX ? kLoopRx : kLoopDg;
    return pick_ragged(mode, n);
  }
  // IPv4 header-only modes: one lane per packet (1M x 1500-B datagrams:
  // 29.9 us vs 36.9 with k_small<4,1>, kbench 13)
  if (mode_is_ipv4(mode) && !forced_variant()) return kHdr;
  if (const char *f = forced_variant()) {
    if (!mode_is_ipv4(mode) && strncmp(f, "k_seg<", 6) == 0 && (n < 2 || stride <= kSeg32Stride))
      return seg_for(f[6] == '8', mode);
    if (mode_is_ipv4(mode) && strcmp(f, kHdr.name) == 0) return kHdr;
    for (const Variant &v : kSmall)
      if (strcmp(v.name, f) == 0 && fits(v)) return v;
    for (const Variant &v : kTiny)
      if (strcmp(v.name, f) == 0 && tiny_ok && fits(v)) return v;
    for (const Variant &v : kLane)
      if (strcmp(v.name, f) == 0 && lane_fits(v)) return v;
  }
  // k_lane up to 112 bytes (72-byte UDP datagrams: 16.4 vs 20.0 us with
  // k_tiny<8>; 64-byte packets, config 2: 14.2 vs 14.8 with k_tiny<4>),
  // k_tiny<8> above, where all its lanes load (128 bytes: 23.6 vs 24.6 us;
  // tools/kbench 2 and 14); k_tiny<4> for sparse small packets
  if (len <= 112u)
    for (const Variant &v : kLane)
      if (lane_fits(v)) return v;
  if (tiny_ok)
    for (const Variant &v : kTiny)
      if (fits(v)) return v;
  // Dense packets up to 704 bytes that k_lane / k_tiny do not take (129..704
  // bytes, or not 4-aligned): the segmented stream sum beats per-packet lane
  // groups, whose loads scatter over partly used windows (160 B: 34.6 vs 50.0 us;
  // 320: 58-66 vs 88-89; 512: 87 vs 103; 704: 116 vs 120; unaligned 66 B: 26.8
  // vs 38.6; from 768 on k_small is as fast or faster; tools/kbench 14,
  // profiles/r01/kbench_uniform_size_sweep.log)
  // (k_seg gives one wave to 64 packets: only batches of 64K packets or more
  // have enough of them to fill the GPU; smaller ones keep the per-packet shapes)
  const bool dense = 2u * stride <= 3u * (uint64_t)len && n >= kMidBatch;
  if (len <= 704u && dense) return seg_for(len >= 448u, mode);
  // and above 3 KiB, where it streams 8 KiB tiles past k_small<64,4> and the
  // one-wave-per-packet k_loop (4096 B: 636 vs 664 us; 9000 B: 1373 vs 1464;
  // 16 KiB: 0.88 vs 0.81 of peak) — given enough 64-packet chunks to fill the
  // GPU (one wave each); a few huge packets keep k_loop's wave per packet
  if (len > 3072u && dense) return seg_for(true, mode);
  for (const Variant &v : kSmall)
    if (fits(v)) return v;
  return len > kLEMax ? kLoopBE : kLoopLE;
}

bool is_tiny(const Variant &v) { return v.ppw == 64u && v.G < 64u; }

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

// Tuning knobs (read once, measurement only, and only under YU_TUNING=1:
// yu::tuning_env). YU_BLOCKS_PER_CU: grid size in 256-thread blocks per CU;
// YU_NT: load policy 0/1/2 (see bld16).
int env_int(const char *name, int lo, int hi, int dflt) {
  const char *s = yu::tuning_env(name);
  if (!s || !*s) return dflt;
  int x = atoi(s);
  return (x >= lo && x <= hi) ? x : dflt;
}

// Grid size in 256-thread blocks per CU. The grid is deliberately larger than
// what is resident at once (5-8 blocks/CU): finished blocks are replaced by
// fresh ones, which evens out the per-CU tail. Measured optimum on MI355X
// (tools/kbench, round 1): 64 for MTU-size and larger packets, 16 for the
// small-packet lane-group variants (G < 16). The 64-packet-step kernels
// (k_lane, k_tiny: `step64`) run best on 6 (round 2, each wave then streams
// about 4 steps with the next in flight): 1M x 64 B 14.2 -> 13.4 us, 72 B 16.0
// -> 14.8, 32 B 10.4 -> 8.4, 100 B 21.7 -> 20.8, 124 B 25.0 -> 23.8
// (profiles/r02/kbench_ab_lane_grid.log).
// Uniform batches on 4 KiB k_seg tiles (dense 129..447-byte packets, `seg4u`)
// run on 10: each wave then streams 2-3 chunks with the next tile in flight
// instead of one chunk per wave (1M UDP datagrams, medians of 6 launches of
// 30: 136 B 33.0 -> 30.5 us, 160 B 34.5 -> 32.9, 256 B 50.2 -> 47.8, 320 B
// 58.8 -> 56.9, 384 B 70.3 -> 66.7, 200 and 420 B within 1 %;
// profiles/r02/kbench_grid_mid_uniform_{a,b}.log).
int blocks_per_cu(uint32_t G, bool step64, bool seg4u) {
  static int v = env_int("YU_BLOCKS_PER_CU", 1, 1024, 0);
  if (v) return v;
  if (seg4u) return 10;
  return step64 ? 6 : (G < 16 ? 16 : 64);
}

int use_nt() {
  static int v = env_int("YU_NT", 0, 2, 2);
  return v;
}

// k_small writing the field in place loads plainly unless YU_NT says otherwise: the
// field's line is then more often still cached when the 2-byte store reaches it
// (config 9: 320.9 -> 312.2 us on one box, 326.2 -> 321.2 on another; all-nt 330.2;
// k_lane's 72-byte writer gains nothing, 29.9 vs 30.8; profiles/r03/kbench_ab_fill_nt.log)
int fill_nt() {
  static int v = env_int("YU_NT", 0, 2, 0);
  return v;
}

// The ragged in-place writer of k_seg's TX kind (wbk): 0 = one 2-byte store per
// field; 1 = the fields patched into the parked tile and their 128-byte lines
// stored whole. YU_FILL_WB overrides.
int fill_wb() {
  static int v = env_int("YU_FILL_WB", 0, 1, 1);
  return v;
}

// YU_XCD: 1 = XCD-aware block order (grid_wave), 0 (default) = plain blockIdx.
// Measured (round 1, tools/ab.sh): no gain on any config — these kernels
// share at most one line between neighbouring blocks, and the Infinity Cache
// already absorbs its second fetch — and -1..3 % on configs 2/3, so it is off.
// YU_SEG_SMALL_BLOCKS: blocks per CU that work on a small-packet ragged
// batch (seg_waves); 0 = the whole grid.
int seg_small_blocks() {
  static int v = env_int("YU_SEG_SMALL_BLOCKS", 0, 64, 3);
  return v;
}

int use_xcd() {
  static int v = env_int("YU_XCD", 0, 1, 0);
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
  const bool seg4u = !A.offsets && (&v == &kSeg4 || &v == &kSegTx4);
  const uint64_t cap = (uint64_t)cu_count(dev) * (uint64_t)blocks_per_cu(v.G, is_tiny(v), seg4u);
  // k_small: runs from 8 runs per CU up (1500-B packets, runs vs interleaved:
  // 16384 packets 8.0 vs 7.2 us, 32768 11.3 vs 12.5, 131072 35.3 vs 38.8; 768-B
  // packets 6.6 vs 5.0, 7.5 vs 8.2, 19.7 vs 22.0; kbench_ab_k_small_runs.log)
  // (YU_RUNS: 0 never, 2 whenever not filling — measurement only)
  static const int runs_knob = env_int("YU_RUNS", 0, 2, 1);
  const bool runs = v.run && !A.fill &&
                    (runs_knob == 2 || (runs_knob == 1 && A.n / v.run >= 8u * (uint64_t)cu_count(dev)));
  const uint64_t ppw = runs ? v.run : v.ppw;
  uint64_t waves = (A.n + ppw - 1) / ppw;
  uint64_t blocks = (waves + waves_per_block - 1) / waves_per_block;
  if (blocks > cap) blocks = cap;
  if (blocks < 1) blocks = 1;
  BatchArgs a = A;
  a.xcd = (uint32_t)use_xcd();
  a.small_waves = (uint32_t)cu_count(dev) * 4u * (uint32_t)seg_small_blocks();
  KernelFn k = A.fill && v.fill ? v.fill : v.fn[use_nt()];
  if (v.run && !runs) k = v.inter[A.fill ? fill_nt() : use_nt()];
  // TX_DATAGRAM in place loads plainly too (fill_nt): a datagram's header line is
  // then more often still cached when its two field stores arrive (1M datagrams
  // U{40..1500}: 211.5 -> 203.1 us; the TXW kind is better off non-temporal, 48.7
  // vs 52.1 us; profiles/r04/kbench_ab_r04k_fill_nt.log)
  if (A.fill && (&v == &kSegDg8 || &v == &kSegDg8c16 || &v == &kSegDg8c40))
    k = v.fn[fill_nt()];
  hipLaunchKernelGGL(k, dim3((unsigned)blocks), dim3(256), 0, stream, a);
  return hip_status(hipGetLastError());
}

bool aligned(const void *p, uintptr_t a) {
  return ((uintptr_t)p & (a - 1)) == 0;
}

int check_common(int mode, const uint16_t *initial_arr, const uint8_t *addrs,
                 const uint16_t *out, bool fill, uint64_t n) {
  if (mode < 0 || mode >= YU_MODE_COUNT) return YU_EINVAL;  // EINVAL:mode
  if (!out && !fill && n) return YU_EINVAL;                // EINVAL:out (an empty batch may pass NULL)
  if (fill && !mode_fills(mode)) return YU_EINVAL;         // EINVAL:fill-mode
  if (initial_arr && !aligned(initial_arr, 2)) return YU_EINVAL;  // EINVAL:side-align
  if (addrs && !aligned(addrs, 4)) return YU_EINVAL;              // EINVAL:side-align
  if (out && !aligned(out, 2)) return YU_EINVAL;                  // EINVAL:side-align
  return YU_OK;
}

// Ragged in place: the TX kinds of k_seg take their TXW form (the whole-line
// write-back, 1M UDP datagrams U{40..200}: 67.5 -> 48.9 us, kbench 8, DESIGN.md
// §5.4) unless YU_FILL_WB=0.
const Variant &pick_ragged_fill(int mode, uint64_t n, bool fill) {
  const Variant &v = pick_ragged(mode, n);
  if (fill && &v == &kSegDg8)
    return kSegDg8c40;
  if (!fill || !fill_wb()) return v;
  if (&v == &kSegTx8) return kSegTxW8c48;
  if (&v == &kSegTx8c16) return kSegTxW8c16;
  if (&v == &kSegTx4) return kSegTxW4;
  return v;
}

int batch_uniform(const uint8_t *data, uint8_t *fill, uint64_t stride,
                  uint32_t len, uint64_t n, int mode,
                  const uint16_t *initial_arr, uint16_t initial,
                  const uint8_t *addrs, uint16_t *out, void *stream) {
  int rc = check_common(mode, initial_arr, addrs, out, fill != nullptr, n);
  if (rc) return rc;
  if (n == 0) return YU_OK;
  if (!data) return YU_EINVAL;                                              // EINVAL:data
  if (mode != YU_MODE_RAW && len > YU_MAX_TRANSPORT_LEN) return YU_EINVAL;  // EINVAL:len-transport
  if (len < min_len(mode)) return YU_EINVAL;                                // EINVAL:len-min
  if (len > YU_MAX_RAW_LEN) return YU_EINVAL;  // EINVAL:len-raw (window offsets stay in uint32)
  // the batch [data, data + (n-1)*stride + len) must not wrap the address space
  if (n > 1 && stride > (UINT64_MAX - (uint64_t)(uintptr_t)data - len) / (n - 1))
    return YU_EINVAL;  // EINVAL:span
  // fill: packets must start 4-byte aligned. The uniform writers (k_tiny's and
  // k_lane's write-back, k_small) store whole dwords of each packet's window,
  // so no dword may hold bytes of two packets.
  if (fill && (((uintptr_t)data | stride) & 3u)) return YU_EINVAL;  // EINVAL:fill-align
  BatchArgs A;
  A.data = data;
  A.offsets = nullptr;
  A.initial_arr = initial_arr;
  A.addrs = addrs;
  A.out = out;
  A.fill = fill;
  A.stride = stride;
  A.n = n;
  A.end = (uint64_t)(uintptr_t)data + (n - 1) * stride + len;
  A.len = len;
  A.initial = initial;
  A.mode = mode;
  const Variant &v = pick_uniform((uintptr_t)data, stride, len, n, mode);
  if (is_tiny(v))
    A.uf = len >= 16u * v.G ? 1u : 0u;  // k_tiny: all chunks whole?
  else
    A.uf = v.window ? (mode_is_ipv4(mode) ? 0u : len / (16u * v.G)) : 0u;
  return launch(v, A, (hipStream_t)stream);
}

int batch_ragged(const uint8_t *data, uint8_t *fill, const uint64_t *offsets,
                 uint64_t n, int mode, const uint16_t *initial_arr,
                 uint16_t initial, const uint8_t *addrs, uint16_t *out,
                 void *stream) {
  int rc = check_common(mode, initial_arr, addrs, out, fill != nullptr, n);
  if (rc) return rc;
  if (n == 0) return YU_OK;
  if (!offsets || !aligned(offsets, 8)) return YU_EINVAL;  // EINVAL:offsets
  if (!data) return YU_EINVAL;                             // EINVAL:data
  BatchArgs A;
  A.data = data;
  A.offsets = offsets;
  A.initial_arr = initial_arr;
  A.addrs = addrs;
  A.out = out;
  A.fill = fill;
  A.stride = 0;
  A.n = n;
  A.end = 0;
  A.len = 0;
  A.initial = initial;
  A.uf = 0;
  A.mode = mode;
  // k_seg streams the batch's bytes (exact BE recovery for chunks holding a
  // RAW packet > 131072 bytes); k_rag takes the IPv4 header-only modes.
  return launch(pick_ragged_fill(mode, n, fill != nullptr), A, (hipStream_t)stream);
}

// Completion signal for the host path's direct mode (yucsum_internal.h):
// stored after the work before it on the stream, with system-scope release,
// into coherent pinned host memory.
__global__ void k_signal(volatile uint32_t *flag, uint32_t value) {
  __threadfence_system();
  *flag = value;
  __threadfence_system();
}

}  // namespace

int yu_internal_signal(uint32_t *flag, uint32_t value, void *stream) {
  hipLaunchKernelGGL(k_signal, dim3(1), dim3(1), 0, (hipStream_t)stream, flag, value);
  return hip_status(hipGetLastError());
}

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
  if (n > 1 && stride < len) return YU_EINVAL;  // EINVAL:fill-overlap (overlapping packets)
  return batch_uniform(data, data, stride, len, n, mode, initial_arr, initial,
                       addrs, out, stream);
}

int yu_csum_fill_ragged(uint8_t *data, const uint64_t *offsets, uint64_t n,
                        int mode, const uint16_t *initial_arr,
                        uint16_t initial, const uint8_t *addrs, uint16_t *out,
                        void *stream) {
  // Any alignment (include/yucsum.h): the ragged writers store each field as one
  // 16-bit store (even address) or two byte stores, and the TXW kind's whole-line
  // write-back stores only 128-byte lines that lie inside its own chunk's packets.
  return batch_ragged(data, data, offsets, n, mode, initial_arr, initial,
                      addrs, out, stream);
}

const char *yu_uniform_variant(uint64_t stride, uint32_t len, int mode,
                               uint64_t data_align16) {
  return pick_uniform(data_align16 & 15u, stride, len, 2, mode).name;
}

const char *yu_uniform_variant_n(uint64_t stride, uint32_t len, uint64_t n, int mode,
                                 uint64_t data_align16) {
  if (mode < 0 || mode >= YU_MODE_COUNT) return "";
  return pick_uniform(data_align16 & 15u, stride, len, n, mode).name;
}

const char *yu_ragged_variant(int mode) {
  if (mode < 0 || mode >= YU_MODE_COUNT) return "";
  return pick_ragged(mode, 1u << 20).name;
}

const char *yu_ragged_variant_n(int mode, uint64_t n) {
  if (mode < 0 || mode >= YU_MODE_COUNT) return "";
  return pick_ragged(mode, n).name;
}

const char *yu_ragged_fill_variant_n(int mode, uint64_t n) {
  if (mode < 0 || mode >= YU_MODE_COUNT) return "";
  return pick_ragged_fill(mode, n, true).name;
}

int yu_device_count(void) {
  int c = 0;
  if (hipGetDeviceCount(&c) != hipSuccess) return 0;
  return c < 0 ? 0 : c;
}

}  // extern "C"
