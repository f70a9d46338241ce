// yustack/checksum.hpp — C++ host-side mirror of yustack's checksum-facing Go
// API, over the C ABI of yucsum.h. Header-only; no HIP or torch types.
//
// The reference is Go (/root/reference); its checksum path is reached through
// package-level functions and header methods. This header keeps their names,
// argument meaning and error behaviour so C++ callers (and the parity tests
// in tests/cpp) read like the reference's own code:
//
//   Go (reference)                                   here
//   checksum.Checksum         checksum/checksum.go:4    yustack::checksum::Checksum
//   checksum.PseudoHeaderChecksum          :24          yustack::checksum::PseudoHeaderChecksum
//   checksum.ChecksumCombine               :32          yustack::checksum::ChecksumCombine
//   header.IPv4.CalculateChecksum header/ipv4.go:177    yustack::header::IPv4::CalculateChecksum
//   header.TCP.CalculateChecksum  header/tcp.go:165     yustack::header::TCP::CalculateChecksum
//   header.UDP.CalculateChecksum  header/udp.go:67      yustack::header::UDP::CalculateChecksum
//   checker.IPv4 / checker.TCP    checker/checker.go:25,71  yustack::checker::IPv4 / TCP
//
// The scalar functions are total (never fail), like the Go ones. The batched
// GPU entry points (yustack::batch) throw yustack::Error on a non-zero status:
// there is no CPU fallback.
#ifndef YUSTACK_CHECKSUM_HPP
#define YUSTACK_CHECKSUM_HPP

#include <stdint.h>

#include <stdexcept>
#include <string>
#include <string_view>
#include <vector>

#include "yucsum.h"

namespace yustack {

class Error : public std::runtime_error {
 public:
  Error(int status, const std::string &what)
      : std::runtime_error(what + ": " + yu_strerror(status) + " (" +
                           std::to_string(status) + ")"),
        status_(status) {}
  int status() const { return status_; }

 private:
  int status_;
};

namespace checksum {

// checksum/checksum.go:4-18
inline uint16_t Checksum(const uint8_t *buf, size_t len, uint16_t initial) {
  return yu_checksum(buf, len, initial);
}
inline uint16_t Checksum(std::string_view buf, uint16_t initial) {
  return yu_checksum(reinterpret_cast<const uint8_t *>(buf.data()), buf.size(), initial);
}
inline uint16_t Checksum(const std::vector<uint8_t> &buf, uint16_t initial) {
  return yu_checksum(buf.data(), buf.size(), initial);
}

// checksum/checksum.go:32-35
inline uint16_t ChecksumCombine(uint16_t a, uint16_t b) {
  return yu_checksum_combine(a, b);
}

// checksum/checksum.go:24-28 (Go strings -> byte strings, as []byte(s))
inline uint16_t PseudoHeaderChecksum(uint32_t protocol, std::string_view srcAddr,
                                     std::string_view dstAddr) {
  return yu_pseudo_header_checksum(
      protocol, reinterpret_cast<const uint8_t *>(srcAddr.data()), srcAddr.size(),
      reinterpret_cast<const uint8_t *>(dstAddr.data()), dstAddr.size());
}

}  // namespace checksum

namespace header {

constexpr int IPv4MinimumSize = 20;   // header/ipv4.go:68
constexpr int TCPMinimumSize = 20;    // header/tcp.go:109
constexpr int UDPMinimumSize = 8;     // header/udp.go:35
constexpr int ICMPv4MinimumSize = 4;  // header/icmpv4.go:13

inline uint16_t be16(const uint8_t *p) { return (uint16_t)((p[0] << 8) | p[1]); }
inline void put16(uint8_t *p, uint16_t v) {
  p[0] = (uint8_t)(v >> 8);
  p[1] = (uint8_t)v;
}
inline void put32(uint8_t *p, uint32_t v) {
  put16(p, (uint16_t)(v >> 16));
  put16(p + 2, (uint16_t)v);
}

// header/ipv4.go: a view over the bytes starting at the IPv4 header.
struct IPv4 {
  uint8_t *b;
  int HeaderLength() const { return (b[0] & 0xf) * 4; }  // :91-93
  uint16_t TotalLength() const { return be16(b + 2); }
  uint8_t Protocol() const { return b[9]; }
  uint16_t Checksum() const { return be16(b + 10); }
  void SetChecksum(uint16_t v) { put16(b + 10, v); }  // :165-167
  std::string_view SourceAddress() const { return {reinterpret_cast<const char *>(b + 12), 4}; }
  std::string_view DestinationAddress() const { return {reinterpret_cast<const char *>(b + 16), 4}; }
  uint16_t CalculateChecksum() const {  // :177-179
    return checksum::Checksum(b, (size_t)HeaderLength(), 0);
  }
  // :146-157 (Encode) — the fields the send paths and tests set
  void Encode(int IHL, uint16_t TotalLength_, uint8_t Protocol_, std::string_view Src,
              std::string_view Dst, uint8_t TTL = 64, uint16_t ID = 0) {
    b[0] = (uint8_t)((4 << 4) | ((IHL / 4) & 0xf));
    b[1] = 0;
    put16(b + 2, TotalLength_);
    put16(b + 4, ID);
    put16(b + 6, 0);
    b[8] = TTL;
    b[9] = Protocol_;
    put16(b + 10, 0);
    for (int i = 0; i < 4; ++i) {
      b[12 + i] = (uint8_t)Src[i];
      b[16 + i] = (uint8_t)Dst[i];
    }
  }
};

// header/tcp.go
struct TCP {
  uint8_t *b;
  int DataOffset() const { return (b[12] >> 4) * 4; }
  uint16_t Checksum() const { return be16(b + 16); }
  void SetChecksum(uint16_t v) { put16(b + 16, v); }  // :156-158
  uint16_t CalculateChecksum(uint16_t partialChecksum, uint16_t totalLen) const {  // :165-173
    uint8_t tmp[2];
    put16(tmp, totalLen);
    uint16_t cksm = checksum::Checksum(tmp, 2, partialChecksum);
    return checksum::Checksum(b, (size_t)DataOffset(), cksm);
  }
  void Encode(uint16_t SrcPort, uint16_t DstPort, uint32_t SeqNum, uint32_t AckNum,
              uint8_t DataOffset_, uint8_t Flags, uint16_t WindowSize) {  // :176-186
    put16(b, SrcPort);
    put16(b + 2, DstPort);
    put32(b + 4, SeqNum);
    put32(b + 8, AckNum);
    b[12] = (uint8_t)((DataOffset_ / 4) << 4);
    b[13] = Flags;
    put16(b + 14, WindowSize);
    put16(b + 16, 0);
    put16(b + 18, 0);
  }
};

// header/udp.go
struct UDP {
  uint8_t *b;
  uint16_t Length() const { return be16(b + 4); }
  uint16_t Checksum() const { return be16(b + 6); }
  void SetChecksum(uint16_t v) { put16(b + 6, v); }  // :60-62
  uint16_t CalculateChecksum(uint16_t partialChecksum, uint16_t totalLength) const {  // :67-75
    uint8_t tmp[2];
    put16(tmp, totalLength);
    uint16_t c = checksum::Checksum(tmp, 2, partialChecksum);
    return checksum::Checksum(b, UDPMinimumSize, c);
  }
  void Encode(uint16_t SrcPort, uint16_t DstPort, uint16_t Length_) {  // :78-83
    put16(b, SrcPort);
    put16(b + 2, DstPort);
    put16(b + 4, Length_);
    put16(b + 6, 0);
  }
};

}  // namespace header

namespace checker {

// checker/checker.go:25-40 (the checksum part): valid iff 0 or 0xFFFF.
inline bool IPv4(const uint8_t *pkt, size_t len, uint16_t *sum = nullptr) {
  if (len < (size_t)header::IPv4MinimumSize) return false;
  header::IPv4 ip{const_cast<uint8_t *>(pkt)};
  if ((size_t)ip.HeaderLength() > len) return false;
  const uint16_t x = ip.CalculateChecksum();
  if (sum) *sum = x;
  return x == 0 || x == 0xffff;
}

// checker/checker.go:71-99 (protocol and checksum part).
inline bool TCP(const uint8_t *pkt, size_t len, uint16_t *sum = nullptr) {
  if (!IPv4(pkt, len)) return false;
  header::IPv4 ip{const_cast<uint8_t *>(pkt)};
  if (ip.Protocol() != 6) return false;
  const uint8_t *tcp = pkt + ip.HeaderLength();
  const uint16_t l = (uint16_t)(ip.TotalLength() - ip.HeaderLength());
  uint16_t xsum = checksum::Checksum(ip.SourceAddress(), 0);
  xsum = checksum::Checksum(ip.DestinationAddress(), xsum);
  const uint8_t proto[2] = {0, 6};
  xsum = checksum::Checksum(proto, 2, xsum);
  const uint8_t lb[2] = {(uint8_t)(l >> 8), (uint8_t)l};
  xsum = checksum::Checksum(lb, 2, xsum);
  xsum = checksum::Checksum(tcp, l, xsum);
  if (sum) *sum = xsum;
  return xsum == 0 || xsum == 0xffff;
}

}  // namespace checker

// Batched device API (the GPU hot path). All pointers are device pointers.
namespace batch {

enum Mode : int {
  RAW = YU_MODE_RAW,
  UDP = YU_MODE_UDP,
  TCP = YU_MODE_TCP,
  IPV4 = YU_MODE_IPV4,
  ICMP = YU_MODE_ICMP,
  VERIFY_IPV4 = YU_MODE_VERIFY_IPV4,
  VERIFY_TCP = YU_MODE_VERIFY_TCP,
  VERIFY_UDP = YU_MODE_VERIFY_UDP,
  VERIFY_RX = YU_MODE_VERIFY_RX,  // out[i] = YU_RX_* bits
  TX_DATAGRAM = YU_MODE_TX_DATAGRAM,  // out[2i] = IPv4 field, out[2i+1] = transport field
};

// Results per packet in `out` (YU_MODE_OUTPUTS): 2 for TX_DATAGRAM, else 1.
inline constexpr uint64_t Outputs(Mode m) { return YU_MODE_OUTPUTS(m); }

struct Side {
  const uint16_t *initial_arr = nullptr;  // per-packet initial / pseudo partial
  uint16_t initial = 0;
  const uint8_t *addrs = nullptr;         // per-packet {src[4], dst[4]}
};

inline void Uniform(const uint8_t *data, uint64_t stride, uint32_t len, uint64_t n, Mode m,
                    uint16_t *out, const Side &s = {}, void *stream = nullptr) {
  int rc = yu_csum_batch_uniform(data, stride, len, n, m, s.initial_arr, s.initial, s.addrs,
                                 out, stream);
  if (rc) throw Error(rc, "yu_csum_batch_uniform");
}

inline void Ragged(const uint8_t *data, const uint64_t *offsets, uint64_t n, Mode m,
                   uint16_t *out, const Side &s = {}, void *stream = nullptr) {
  int rc = yu_csum_batch_ragged(data, offsets, n, m, s.initial_arr, s.initial, s.addrs, out,
                                stream);
  if (rc) throw Error(rc, "yu_csum_batch_ragged");
}

// In-place writers (SetChecksum on the device; include/yucsum.h, Preconditions).
// FillUniform needs data and stride multiples of 4 and stride >= len (else Error with
// YU_EINVAL: [fill-align], [fill-overlap]); FillRagged takes any alignment — a packed,
// unaligned tun burst as it lies — so an unaligned uniform batch goes through
// FillRagged with offsets[i] = i * stride. Only the fields change. Both throw
// YU_EINVAL for a mode with no field ([fill-mode]: RAW, VERIFY_*).
inline void FillUniform(uint8_t *data, uint64_t stride, uint32_t len, uint64_t n, Mode m,
                        uint16_t *out = nullptr, const Side &s = {}, void *stream = nullptr) {
  int rc = yu_csum_fill_uniform(data, stride, len, n, m, s.initial_arr, s.initial, s.addrs,
                                out, stream);
  if (rc) throw Error(rc, "yu_csum_fill_uniform");
}

inline void FillRagged(uint8_t *data, const uint64_t *offsets, uint64_t n, Mode m,
                       uint16_t *out = nullptr, const Side &s = {}, void *stream = nullptr) {
  int rc = yu_csum_fill_ragged(data, offsets, n, m, s.initial_arr, s.initial, s.addrs, out,
                               stream);
  if (rc) throw Error(rc, "yu_csum_fill_ragged");
}

// Host buffers in, host results out (pinned staging + pipelined copies, or
// the direct path for bursts up to 4 MiB). Here `Side` holds HOST pointers.
// A device list shards the batch over several GPUs (the *_multi calls).
inline void HostUniform(const uint8_t *data, uint64_t stride, uint32_t len, uint64_t n, Mode m,
                        uint16_t *out, const Side &s = {}, int device = 0) {
  int rc = yu_csum_batch_host_uniform(data, stride, len, n, m, s.initial_arr, s.initial,
                                      s.addrs, out, device);
  if (rc) throw Error(rc, "yu_csum_batch_host_uniform");
}

inline void HostUniform(const uint8_t *data, uint64_t stride, uint32_t len, uint64_t n, Mode m,
                        uint16_t *out, const Side &s, const std::vector<int> &devices) {
  int rc = yu_csum_batch_host_uniform_multi(data, stride, len, n, m, s.initial_arr, s.initial,
                                            s.addrs, out, devices.data(), (int)devices.size());
  if (rc) throw Error(rc, "yu_csum_batch_host_uniform_multi");
}

// A tun read burst packed back to back: packet i = data[offsets[i], offsets[i+1]).
inline void HostRagged(const uint8_t *data, const uint64_t *offsets, uint64_t n, Mode m,
                       uint16_t *out, const Side &s = {}, int device = 0) {
  int rc = yu_csum_batch_host_ragged(data, offsets, n, m, s.initial_arr, s.initial, s.addrs,
                                     out, device);
  if (rc) throw Error(rc, "yu_csum_batch_host_ragged");
}

inline void HostRagged(const uint8_t *data, const uint64_t *offsets, uint64_t n, Mode m,
                       uint16_t *out, const Side &s, const std::vector<int> &devices) {
  int rc = yu_csum_batch_host_ragged_multi(data, offsets, n, m, s.initial_arr, s.initial,
                                           s.addrs, out, devices.data(), (int)devices.size());
  if (rc) throw Error(rc, "yu_csum_batch_host_ragged_multi");
}

// Scatter-gather packets (the tun endpoint's readv views,
// link/tundev/tundev.go:116-125): packet i = iov[first_iov[i] .. first_iov[i+1]).
inline void HostPackets(const yu_iovec *iov, const uint64_t *first_iov, uint64_t n, Mode m,
                        uint16_t *out, const Side &s = {}, int device = 0) {
  int rc = yu_csum_batch_host_iov(iov, first_iov, n, m, s.initial_arr, s.initial, s.addrs, out,
                                  device);
  if (rc) throw Error(rc, "yu_csum_batch_host_iov");
}

inline void HostPackets(const yu_iovec *iov, const uint64_t *first_iov, uint64_t n, Mode m,
                        uint16_t *out, const Side &s, const std::vector<int> &devices) {
  int rc = yu_csum_batch_host_iov_multi(iov, first_iov, n, m, s.initial_arr, s.initial,
                                        s.addrs, out, devices.data(), (int)devices.size());
  if (rc) throw Error(rc, "yu_csum_batch_host_iov_multi");
}

// Host-memory field writer (SetChecksum in place, TX modes): the batch above,
// then each result stored big-endian into the packet's field by the CPU, at any
// alignment (as Go's SetChecksum). `out` may be null.
inline void FillHostUniform(uint8_t *data, uint64_t stride, uint32_t len, uint64_t n, Mode m,
                            uint16_t *out = nullptr, const Side &s = {}, int device = 0) {
  int rc = yu_csum_fill_host_uniform(data, stride, len, n, m, s.initial_arr, s.initial, s.addrs,
                                     out, device);
  if (rc) throw Error(rc, "yu_csum_fill_host_uniform");
}

inline void FillHostRagged(uint8_t *data, const uint64_t *offsets, uint64_t n, Mode m,
                           uint16_t *out = nullptr, const Side &s = {}, int device = 0) {
  int rc = yu_csum_fill_host_ragged(data, offsets, n, m, s.initial_arr, s.initial, s.addrs, out,
                                    device);
  if (rc) throw Error(rc, "yu_csum_fill_host_ragged");
}

inline void FillHostPackets(const yu_iovec *iov, const uint64_t *first_iov, uint64_t n, Mode m,
                            uint16_t *out = nullptr, const Side &s = {}, int device = 0) {
  int rc = yu_csum_fill_host_iov(iov, first_iov, n, m, s.initial_arr, s.initial, s.addrs, out,
                                 device);
  if (rc) throw Error(rc, "yu_csum_fill_host_iov");
}

// Host-path staging of `device` (include/yucsum.h, "Host-path staging"): the pinned
// and device bytes its bounded context pools hold now; at most HostContexts() x
// (YU_HOST_CONTEXT_PINNED_MAX + YU_HOST_BURST_CONTEXT_PINNED_MAX) pinned and the
// _DEVICE_MAX sums on the device between calls (bulk and burst contexts).
struct Staging {
  uint64_t pinned, device;
};
inline Staging HostStaging(int device = 0) {
  uint64_t d = 0;
  const uint64_t p = yu_host_staging_bytes(device, &d);
  return {p, d};
}
inline int HostContexts() { return yu_host_contexts(); }
// Frees the staging of the device's idle contexts.
inline void HostStagingTrim(int device = 0) {
  int rc = yu_host_staging_trim(device);
  if (rc) throw Error(rc, "yu_host_staging_trim");
}

}  // namespace batch
}  // namespace yustack

#endif  // YUSTACK_CHECKSUM_HPP
