/*
 * csum_oracle.c — TEST INFRASTRUCTURE ONLY. CPU restatement of yustack's
 * Internet-checksum path, used as the parity checker for the HIP engine.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library, and only as the checker / the reported CPU baseline.
 * The product (yustack_amd/, libyucsum.so) never links or calls it.
 *
 * Every function is a literal restatement of the reference Go code it cites
 * (paths relative to /root/reference). The loop shapes are kept on purpose:
 * compiled with -O2 -fno-tree-vectorize this is the "reference-faithful"
 * scalar baseline.
 *
 * PARITY UNPINNED (by the task's rule): the reference is Go, no Go toolchain
 * exists in this image, and it ships no known-answer vectors,
 * so neither the reference's fixtures nor the reference itself run here can
 * pin this oracle. The evidence it rests on instead: (1) known answers
 * produced by EXECUTING the reference's own source
 * (checksum/checksum.go, header/{ipv4,tcp,udp}.go) with a minimal Go-subset
 * interpreter, tests/golden/goexec.py -> tests/golden/refexec.json (every
 * batch mode, the Checksum/Combine/PseudoHeaderChecksum functions, the uint32
 * wrap); (2) RFC 1071 §3's published example; (3) the reference's own
 * test-side verification property (checker/checker.go:32-35,80-92) on packets
 * built as its test harnesses build them (transport/tcp/testing/context/
 * context.go:164-209, transport/udp/udp_test.go:105-144); and (4) an
 * independent Python twin (oracle/oracle.py) plus a closed form, all checked
 * in tests/test_oracle.py; (5) datagrams the Linux kernel verified or built
 * (tests/golden/kernel_verified.npz). The interpreter in (1) is written for
 * this repo, a stand-in for the absent Go toolchain, not the reference run.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define OR_MODE_RAW 0
#define OR_MODE_UDP 1
#define OR_MODE_TCP 2
#define OR_MODE_IPV4 3
#define OR_MODE_ICMP 4
#define OR_MODE_VERIFY_IPV4 5
#define OR_MODE_VERIFY_TCP 6
#define OR_MODE_VERIFY_UDP 7
#define OR_MODE_VERIFY_RX 8
#define OR_MODE_TX_DATAGRAM 9
#define OR_RX_IP_OK 1
#define OR_RX_L4 2
#define OR_RX_L4_OK 4
#define OR_RX_INVALID 8

/* checksum/checksum.go:32-35 — ChecksumCombine */
uint16_t or_checksum_combine(uint16_t a, uint16_t b) {
  uint32_t v = (uint32_t)a + (uint32_t)b;
  return (uint16_t)(v + (v >> 16));
}

/* checksum/checksum.go:4-18 — Checksum. uint32 accumulator, wraps mod 2^32;
 * odd trailing byte added first as a high byte; big-endian byte pairs. */
uint16_t or_checksum(const uint8_t *buf, size_t len, uint16_t initial) {
  uint32_t v = (uint32_t)initial;
  size_t l = len;
  if (l & 1) {
    l--;
    v += (uint32_t)buf[l] << 8;
  }
  for (size_t i = 0; i < l; i += 2) {
    v += ((uint32_t)buf[i] << 8) + (uint32_t)buf[i + 1];
  }
  return or_checksum_combine((uint16_t)v, (uint16_t)(v >> 16));
}

/* checksum/checksum.go:24-28 — PseudoHeaderChecksum */
uint16_t or_pseudo_header_checksum(uint32_t protocol, const uint8_t *src,
                                   size_t src_len, const uint8_t *dst,
                                   size_t dst_len) {
  uint16_t xsum = or_checksum(src, src_len, 0);
  xsum = or_checksum(dst, dst_len, xsum);
  uint8_t p[2] = {0, (uint8_t)protocol};
  return or_checksum(p, 2, xsum);
}

/* header/udp.go:67-75 — UDP.CalculateChecksum(partialChecksum, totalLength) */
uint16_t or_udp_calculate_checksum(const uint8_t *udp_hdr, uint16_t partial,
                                   uint16_t total_length) {
  uint8_t tmp[2] = {(uint8_t)(total_length >> 8), (uint8_t)total_length};
  uint16_t c = or_checksum(tmp, 2, partial);
  return or_checksum(udp_hdr, 8, c); /* b[:UDPMinimumSize] */
}

/* header/tcp.go:165-173 — TCP.CalculateChecksum(partialChecksum, totalLen) */
uint16_t or_tcp_calculate_checksum(const uint8_t *tcp_hdr, uint16_t partial,
                                   uint16_t total_len) {
  uint8_t tmp[2] = {(uint8_t)(total_len >> 8), (uint8_t)total_len};
  uint16_t cksm = or_checksum(tmp, 2, partial);
  size_t data_offset = (size_t)(tcp_hdr[12] >> 4) * 4; /* DataOffset() */
  return or_checksum(tcp_hdr, data_offset, cksm);       /* b[:DataOffset()] */
}

/* header/ipv4.go:177-179 — IPv4.CalculateChecksum, HeaderLength() at :91-93 */
uint16_t or_ipv4_calculate_checksum(const uint8_t *ip_hdr) {
  uint8_t hl = (uint8_t)((ip_hdr[0] & 0xf) * 4);
  return or_checksum(ip_hdr, hl, 0);
}

/* Pseudo-header partial for packet p of a batch: the 8-byte {src,dst}
 * record when given (types/route.go:90-92 -> checksum.go:24-28), else the
 * caller-supplied PseudoHeaderChecksum value. */
static uint16_t batch_pseudo(uint32_t proto, const uint8_t *addrs,
                             const uint16_t *initial_arr, uint16_t initial,
                             uint64_t p) {
  if (addrs) return or_pseudo_header_checksum(proto, addrs + 8 * p, 4,
                                              addrs + 8 * p + 4, 4);
  return initial_arr ? initial_arr[p] : initial;
}

/* One packet of a batch, composed exactly as the reference call sites.
 * `pkt`/`len` is the packet as it sits in the batch buffer. TX modes take
 * the checksum field as 0, because the reference's Encode writes 0 before
 * CalculateChecksum (header/udp.go:78-83, header/tcp.go:176-186,
 * header/ipv4.go:146-157; the ICMP header comes from a fresh zeroed
 * Prependable, network/ipv4/icmp.go:37-42). */
uint16_t or_packet(int mode, const uint8_t *pkt, uint64_t len,
                   const uint16_t *initial_arr, uint16_t initial,
                   const uint8_t *addrs, uint64_t p) {
  uint8_t hdr[64];
  switch (mode) {
    case OR_MODE_RAW: {
      uint16_t init = initial_arr ? initial_arr[p] : initial;
      return or_checksum(pkt, (size_t)len, init);
    }
    case OR_MODE_UDP: {
      /* transport/udp/endpoint.go:164-187 (sendUDP) */
      memcpy(hdr, pkt, 8);
      hdr[6] = hdr[7] = 0; /* Encode: Checkum field zero value */
      uint16_t length = 8; /* hdr.UsedLength() */
      uint16_t xsum = batch_pseudo(17, addrs, initial_arr, initial, p);
      const uint8_t *data = pkt + 8;
      uint64_t dlen = len - 8;
      length = (uint16_t)(length + (uint16_t)dlen);
      xsum = or_checksum(data, (size_t)dlen, xsum);
      return (uint16_t)~or_udp_calculate_checksum(hdr, xsum, length);
    }
    case OR_MODE_TCP: {
      /* transport/tcp/connect.go:556-586 (sendTCP) and :288-322 */
      size_t doff = (size_t)(pkt[12] >> 4) * 4;
      /* in contract 20 <= DataOffset <= len (every segment sendTCP encodes);
       * outside it the value is unspecified, but never a read past the packet */
      if (doff > len) doff = (size_t)len;
      memset(hdr, 0, sizeof(hdr));
      memcpy(hdr, pkt, doff < 20 && len >= 20 ? 20 : doff);
      hdr[16] = hdr[17] = 0; /* Encode: Checksum field zero value */
      uint16_t length = (uint16_t)doff;
      uint16_t xsum = batch_pseudo(6, addrs, initial_arr, initial, p);
      const uint8_t *data = pkt + doff;
      uint64_t dlen = len - doff;
      length = (uint16_t)(length + (uint16_t)dlen);
      xsum = or_checksum(data, (size_t)dlen, xsum);
      return (uint16_t)~or_tcp_calculate_checksum(hdr, xsum, length);
    }
    case OR_MODE_IPV4: {
      /* network/ipv4/ipv4.go:80-97 */
      /* the packet as Encode left it: same bytes, checksum field 0; the
       * header length is read from byte 0 of that packet */
      size_t cp = len < sizeof(hdr) ? (size_t)len : sizeof(hdr);
      memcpy(hdr, pkt, cp);
      if (cp >= 12) hdr[10] = hdr[11] = 0; /* Encode: Checksum zero value */
      /* b[:IHL*4], clamped to the packet as a Go slice of it would be */
      size_t hl = cp ? (size_t)(hdr[0] & 0xf) * 4 : 0;
      return (uint16_t)~or_checksum(hdr, hl < cp ? hl : cp, 0);
    }
    case OR_MODE_ICMP: {
      /* network/ipv4/icmp.go:36-45 */
      memcpy(hdr, pkt, 4);
      hdr[2] = hdr[3] = 0; /* fresh Prependable: zero */
      uint16_t inner = or_checksum(pkt + 4, (size_t)(len - 4), 0);
      return (uint16_t)~or_checksum(hdr, 4, inner);
    }
    case OR_MODE_VERIFY_IPV4: {
      /* checker/checker.go:32; b[:IHL*4] clamped to the packet */
      size_t hl = len ? (size_t)(pkt[0] & 0xf) * 4 : 0;
      return or_checksum(pkt, hl < len ? hl : (size_t)len, 0);
    }
    case OR_MODE_VERIFY_TCP:
    case OR_MODE_VERIFY_UDP: {
      /* checker/checker.go:80-88 */
      uint32_t proto = mode == OR_MODE_VERIFY_TCP ? 6 : 17;
      uint16_t l = (uint16_t)len;
      uint16_t xsum = batch_pseudo(proto, addrs, initial_arr, initial, p);
      uint8_t lb[2] = {(uint8_t)(l >> 8), (uint8_t)l};
      xsum = or_checksum(lb, 2, xsum);
      return or_checksum(pkt, (size_t)len, xsum);
    }
    case OR_MODE_VERIFY_RX: {
      /* A received IPv4 packet checked as checker.IPv4 + checker.TCP do
       * (checker/checker.go:25-40,71-92), addresses, protocol and lengths
       * read from the packet itself (header/ipv4.go:91-138,182-189). */
      if (len < 20) return OR_RX_INVALID;               /* IsValid: minimum */
      size_t hl = (size_t)(pkt[0] & 0xf) * 4;           /* HeaderLength() */
      size_t tl = ((size_t)pkt[2] << 8) | pkt[3];       /* TotalLength() */
      if (hl > tl || tl > len) return OR_RX_INVALID;    /* IsValid */
      uint16_t r = 0;
      uint16_t x = or_checksum(pkt, hl, 0);             /* CalculateChecksum */
      if (x == 0 || x == 0xffff) r |= OR_RX_IP_OK;
      uint8_t proto = pkt[9];                           /* Protocol() */
      if (proto == 6 || proto == 17 || proto == 1) {
        r |= OR_RX_L4;
        const uint8_t *pl = pkt + hl;                   /* Payload() */
        size_t plen = tl - hl;
        uint16_t xs;
        if (proto == 1) {
          xs = or_checksum(pl, plen, 0);                /* ICMP: no pseudo */
        } else {
          uint16_t l = (uint16_t)plen;
          xs = or_pseudo_header_checksum(proto, pkt + 12, 4, pkt + 16, 4);
          uint8_t lb[2] = {(uint8_t)(l >> 8), (uint8_t)l};
          xs = or_checksum(lb, 2, xs);
          xs = or_checksum(pl, plen, xs);
        }
        if (xs == 0 || xs == 0xffff) r |= OR_RX_L4_OK;
      }
      return r;
    }
    default:
      return 0;
  }
}

/* A whole outgoing IPv4 datagram (YU_MODE_TX_DATAGRAM, include/yucsum.h):
 * the two fields the reference's senders store before the link endpoint
 * writes it (network/ipv4/ipv4.go:80-97 after transport/udp/endpoint.go:
 * 164-187, transport/tcp/connect.go:556-586 or network/ipv4/icmp.go:36-45),
 * each composed exactly as the single-field modes above, with the pseudo
 * header taken from the datagram's own addresses and protocol. res[0] = IPv4
 * header field, res[1] = transport field; {0, 0} outside the contract
 * 20 <= HeaderLength() <= TotalLength() <= len. */
void or_tx_datagram(const uint8_t *pkt, uint64_t len, uint16_t res[2]) {
  res[0] = res[1] = 0;
  if (len < 20) return;
  size_t hl = (size_t)(pkt[0] & 0xf) * 4;     /* HeaderLength() */
  size_t tl = ((size_t)pkt[2] << 8) | pkt[3]; /* TotalLength() */
  if (hl < 20 || hl > tl || tl > len) return;
  res[0] = or_packet(OR_MODE_IPV4, pkt, len, NULL, 0, NULL, 0);
  const uint8_t *seg = pkt + hl;                /* Payload() */
  uint64_t slen = tl - hl;
  const uint8_t *rec = pkt + 12;                /* {src[4], dst[4]}: types/route.go:90-92 */
  switch (pkt[9]) {                             /* Protocol() */
    case 17:
      if (slen >= 8) res[1] = or_packet(OR_MODE_UDP, seg, slen, NULL, 0, rec, 0);
      break;
    case 6:
      if (slen >= 20) res[1] = or_packet(OR_MODE_TCP, seg, slen, NULL, 0, rec, 0);
      break;
    case 1:
      if (slen >= 4) res[1] = or_packet(OR_MODE_ICMP, seg, slen, NULL, 0, NULL, 0);
      break;
    default:
      break;
  }
}

/* Results per packet: 2 for TX_DATAGRAM (out[2p], out[2p+1]), else 1. */
static void or_one(int mode, const uint8_t *pkt, uint64_t len,
                   const uint16_t *initial_arr, uint16_t initial,
                   const uint8_t *addrs, uint16_t *out, uint64_t p) {
  if (mode == OR_MODE_TX_DATAGRAM)
    or_tx_datagram(pkt, len, out + 2 * p);
  else
    out[p] = or_packet(mode, pkt, len, initial_arr, initial, addrs, p);
}

void or_batch_uniform(const uint8_t *data, uint64_t stride, uint32_t len,
                      uint64_t n, int mode, const uint16_t *initial_arr,
                      uint16_t initial, const uint8_t *addrs, uint16_t *out,
                      uint64_t first, uint64_t count) {
  (void)n;
  for (uint64_t p = first; p < first + count; ++p)
    or_one(mode, data + p * stride, len, initial_arr, initial, addrs, out, p);
}

void or_batch_ragged(const uint8_t *data, const uint64_t *offsets, uint64_t n,
                     int mode, const uint16_t *initial_arr, uint16_t initial,
                     const uint8_t *addrs, uint16_t *out, uint64_t first,
                     uint64_t count) {
  (void)n;
  for (uint64_t p = first; p < first + count; ++p)
    or_one(mode, data + offsets[p], offsets[p + 1] - offsets[p], initial_arr,
           initial, addrs, out, p);
}

/* ---- static even split over host threads (cpu_baseline leg) ---- */
typedef struct {
  const uint8_t *data;
  const uint64_t *offsets;
  uint64_t stride;
  uint32_t len;
  uint64_t n;
  int mode;
  const uint16_t *initial_arr;
  uint16_t initial;
  const uint8_t *addrs;
  uint16_t *out;
  uint64_t first, count;
} or_job;

static void *or_worker(void *arg) {
  or_job *j = (or_job *)arg;
  if (j->offsets)
    or_batch_ragged(j->data, j->offsets, j->n, j->mode, j->initial_arr,
                    j->initial, j->addrs, j->out, j->first, j->count);
  else
    or_batch_uniform(j->data, j->stride, j->len, j->n, j->mode,
                     j->initial_arr, j->initial, j->addrs, j->out, j->first,
                     j->count);
  return NULL;
}

/* offsets == NULL selects the uniform layout. Returns 0 on success. */
int or_batch_mt(const uint8_t *data, const uint64_t *offsets, uint64_t stride,
                uint32_t len, uint64_t n, int mode,
                const uint16_t *initial_arr, uint16_t initial,
                const uint8_t *addrs, uint16_t *out, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  if ((uint64_t)nthreads > n) nthreads = n ? (int)n : 1;
  pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
  or_job *jobs = (or_job *)calloc((size_t)nthreads, sizeof(or_job));
  if (!th || !jobs) {
    free(th);
    free(jobs);
    return -1;
  }
  uint64_t per = n / (uint64_t)nthreads, rem = n % (uint64_t)nthreads;
  uint64_t first = 0;
  int started = 0, rc = 0;
  for (int t = 0; t < nthreads; ++t) {
    uint64_t cnt = per + ((uint64_t)t < rem ? 1 : 0);
    or_job j = {data,  offsets,     stride,  len,   n,   mode,
                initial_arr, initial, addrs, out, first, cnt};
    jobs[t] = j;
    first += cnt;
    if (pthread_create(&th[t], NULL, or_worker, &jobs[t]) != 0) {
      rc = -1;
      break;
    }
    started++;
  }
  for (int t = 0; t < started; ++t) pthread_join(th[t], NULL);
  free(th);
  free(jobs);
  return rc;
}
