/*
 * yucsum.h — C ABI of the MI355X-native Internet-checksum engine.
 *
 * This is the drop-in boundary for yustack's `checksum` package
 * (reference: /root/reference/checksum/checksum.go). The reference exposes
 * three package-level Go functions and nothing else; every caller
 * (header/ipv4.go:177-179, header/tcp.go:165-173, header/udp.go:67-75,
 * types/route.go:90-92, transport/udp/endpoint.go:175,
 * transport/tcp/connect.go:314,580, network/ipv4/icmp.go:42,
 * checker/checker.go:32,84-88) reaches the hot path through them.
 *
 * Two groups of entry points:
 *
 *  1. Scalar, Go-signature entry points (yu_checksum, yu_checksum_combine,
 *     yu_pseudo_header_checksum). These are what a cgo shim binds so that the
 *     reference's callers compile unchanged. They run on the
 *     calling host thread: a cgo call costs ~100 ns, a GPU round trip costs
 *     microseconds, so per-call offload would be a pessimisation. They are
 *     total functions (never fail), reentrant and allocation-free.
 *
 *  2. Batched device entry points (yu_csum_batch_uniform,
 *     yu_csum_batch_ragged). These are the GPU hot path: one launch computes
 *     the per-packet sums of a whole device-resident batch with hand-written
 *     gfx950 HIP kernels. They are asynchronous on the given HIP stream,
 *     perform no allocation and no synchronisation (graph-capturable), and
 *     return a status code. There is no CPU fallback: without a usable GPU
 *     they return a negative status.
 *
 *  3. Batched host entry points (yu_csum_batch_host_uniform / _ragged / _iov,
 *     and their _multi forms over several GPUs): the path that starts and
 *     ends in host memory (tun / link-layer buffers). Batches up to 4 MiB are
 *     read and answered in place over PCIe by the kernel (one launch, one
 *     synchronisation); larger ones are staged through library-owned pinned
 *     buffers with H2D copy, kernel and D2H copy overlapped on separate
 *     streams. Synchronous.
 *
 * All arithmetic is unsigned integer. Results are bit-identical to the
 * reference Go code on the same bytes, including the reference's uint32
 * wrap-around for buffers longer than 131072 bytes (RAW mode).
 */
#ifndef YUCSUM_H
#define YUCSUM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define YUCSUM_ABI_VERSION 1

/* ------------------------------------------------------------------ */
/* Status codes (batched entry points).                               */
/* ------------------------------------------------------------------ */
#define YU_OK 0
#define YU_EINVAL (-22)         /* bad argument (mode, NULL pointer, len) */
#define YU_ENODEV (-19)         /* no HIP device / device index out of range */
#define YU_ENOMEM (-12)         /* pinned/device staging allocation failed */
#define YU_EHIP_BASE (-1000)    /* -(1000 + hipError_t) for any other HIP error */

/* ------------------------------------------------------------------ */
/* Preconditions: every YU_EINVAL the batched calls return.            */
/* Each `return YU_EINVAL` in the library is tagged with one of these   */
/* names, and tests/test_abi.py checks that the tags and this list      */
/* agree. All are checked before any device work; a call that returns  */
/* YU_EINVAL has read no packet byte and written nothing.               */
/*                                                                      */
/*  [mode]          mode is not 0 .. YU_MODE_COUNT-1 (every call).       */
/*  [out]           out == NULL in a yu_csum_batch_* call, or h_out ==   */
/*                  NULL in a yu_csum_batch_host_* call, with n > 0 (the */
/*                  fill calls take NULL: no result array; an empty     */
/*                  batch, n == 0, is a no-op returning YU_OK).          */
/*  [fill-mode]     a fill call (yu_csum_fill_*) with a mode that has no */
/*                  field to write: RAW, VERIFY_* (or no mode at all).   */
/*  [side-align]    device calls: initial_arr not 2-byte aligned, addrs  */
/*                  not 4-byte aligned, out not 2-byte aligned.          */
/*  [data]          data == NULL with n > 0 (device calls), h_data ==    */
/*                  NULL while the packets hold bytes (host calls), iov  */
/*                  == NULL while first_iov names views.                 */
/*  [len-transport] a packet of a mode other than RAW longer than        */
/*                  YU_MAX_TRANSPORT_LEN (uniform len; every host ragged */
/*                  or iov packet). Device ragged batches are not read   */
/*                  back on the host: see "Out of contract" below.       */
/*  [len-raw]       a RAW packet longer than YU_MAX_RAW_LEN (the same).  */
/*  [len-min]       uniform len below the mode's fixed header: UDP 8,    */
/*                  TCP 20, ICMP 4, IPV4 / VERIFY_IPV4 1 (the IHL byte). */
/*  [span]          uniform: data + (n-1)*stride + len wraps the address */
/*                  space.                                               */
/*  [offsets]       offsets == NULL, or (device) not 8-byte aligned, or  */
/*                  (host) decreasing; first_iov == NULL or decreasing.  */
/*  [iov-view]      a view with base == NULL and len > 0.                */
/*  [fill-align]    yu_csum_fill_uniform: data or stride not a multiple  */
/*                  of 4. The uniform writers store whole dwords of each */
/*                  packet's window, so no dword may hold bytes of two   */
/*                  packets.                                             */
/*  [fill-overlap]  yu_csum_fill_uniform: n > 1 and stride < len.        */
/*  [devices]       *_multi: devices == NULL, ndev < 1 or ndev > 64.     */
/*                  (A listed device that does not exist: YU_ENODEV.)    */
/*                                                                      */
/* Where the writers differ from the reference: Go's SetChecksum         */
/* (header/udp.go:60-62, header/tcp.go:156-158, header/ipv4.go:165-167,  */
/* header/icmpv4.go:46-48) has no alignment precondition, and neither do */
/* yu_csum_fill_ragged (device) and the yu_csum_fill_host_* calls: a     */
/* packed, unaligned tun burst (any data address, any offsets) is        */
/* written in place as it lies. Only the uniform device writer asks for  */
/* [fill-align]; an unaligned uniform batch goes through                 */
/* yu_csum_fill_ragged with offsets[i] = i * stride instead (same values,*/
/* same field stores). In the ragged writer a field at an even address   */
/* is one 16-bit store and one at an odd address two byte stores; from   */
/* 65536 packets on (the TXW kind, yu_ragged_fill_variant_n) the         */
/* 128-byte lines that lie wholly inside one 48-packet chunk's packets   */
/* and hold a field are stored whole from the bytes just read, the field */
/* patched in; a field straddling two lines keeps its byte stores.       */
/* Bytes outside the packets' fields are never changed.                  */
/*                                                                      */
/* Out of contract (device ragged batches only, whose offsets live in    */
/* device memory and are not checked here): a packet whose offsets       */
/* decrease, longer than the mode's limit (YU_MAX_TRANSPORT_LEN; RAW:    */
/* YU_MAX_RAW_LEN), or ending past offsets[n] (a call touches at most    */
/* data[0, offsets[n])). It gets an unspecified result, never a fault or */
/* a hang: every byte a ragged call reads or writes lies in the dwords   */
/* holding data[0, offsets[n]), whatever the other offsets say           */
/* (offsets[n] itself must be right, and data + offsets[i] must not wrap */
/* the address space). A kernel that takes a group of consecutive        */
/* packets at a time (k_seg's chunks                                    */
/* of 16 to 64 packets, k_hdr's steps of 64; yu_ragged_variant_n and    */
/* yu_ragged_fill_variant_n name the kernel) may give the other packets */
/* of the group holding one, [k*c, k*c + c) for group size c,           */
/* unspecified results too. A fill call never writes a byte outside the */
/* checksum fields of in-contract packets: no field of an out-of-       */
/* contract packet is stored, nor any field of its group. Every other   */
/* packet's result and field are exact. Validate first when the offsets */
/* come from outside (the host forms and the Python front end           */
/* batch.checksum_ragged(validate=True) do).                            */

/* ------------------------------------------------------------------ */
/* Scalar entry points (host CPU, Go-signature drop-ins).             */
/* ------------------------------------------------------------------ */

/* Replaces `func Checksum(buf []byte, initial uint16) uint16`
 * (checksum/checksum.go:4-18). Sum of big-endian 16-bit words of buf, odd
 * trailing byte as the high byte of a final word, plus `initial`, in a
 * uint32 accumulator that wraps mod 2^32, folded once by ChecksumCombine.
 * The result is NOT complemented. len==0 (buf may be NULL) returns
 * fold(initial) == initial. */
uint16_t yu_checksum(const uint8_t *buf, size_t len, uint16_t initial);

/* Replaces `func ChecksumCombine(a, b uint16) uint16`
 * (checksum/checksum.go:32-35): one end-around-carry add. */
uint16_t yu_checksum_combine(uint16_t a, uint16_t b);

/* Replaces `func PseudoHeaderChecksum(protocol uint32, srcAddr, dstAddr
 * string) uint16` (checksum/checksum.go:24-28). Go strings become
 * (pointer, length) pairs; the protocol is truncated to uint8 exactly as
 * `uint8(protocol)` does. The transport length is NOT included (callers add
 * it through {UDP,TCP}.CalculateChecksum, header/udp.go:67-75,
 * header/tcp.go:165-173). */
uint16_t yu_pseudo_header_checksum(uint32_t protocol,
                                   const uint8_t *src_addr, size_t src_len,
                                   const uint8_t *dst_addr, size_t dst_len);

/* ------------------------------------------------------------------ */
/* Batched modes. Each names the reference composition it reproduces.  */
/* "pseudo" = the per-packet pseudo-header partial sum: either the 8-byte */
/* {src[4], dst[4]} record from `addrs` (protocol fixed by the mode) or,  */
/* when addrs is NULL, the uint16 PseudoHeaderChecksum value from        */
/* `initial_arr[i]` (or the scalar `initial`).                           */
/* ------------------------------------------------------------------ */

/* out[i] = Checksum(pkt_i, initial_i)  — checksum/checksum.go:4-18.
 * Uncomplemented; exact for any length (uint32 wrap reproduced). */
#define YU_MODE_RAW 0
/* pkt_i = UDP header (8 B) + data. out[i] = the value sendUDP stores:
 * ^UDP.CalculateChecksum(Checksum(data, pseudo), len) with the header's
 * checksum field taken as 0 (Encode writes 0) —
 * transport/udp/endpoint.go:164-187, header/udp.go:67-83. Protocol 17. */
#define YU_MODE_UDP 1
/* pkt_i = TCP segment (header incl. options, then data). out[i] = the value
 * sendTCP stores: ^TCP.CalculateChecksum(Checksum(data, pseudo), len) with
 * the checksum field taken as 0 — transport/tcp/connect.go:556-586,
 * header/tcp.go:165-186. Protocol 6. As in every segment sendTCP encodes,
 * 20 <= DataOffset() <= len is required; other segments get an unspecified
 * value (never a fault). Data = the bytes past DataOffset() * 4. (Only
 * sendTCPWithOptions given options whose length is not a multiple of 4 —
 * no caller does: sendSynTCP passes 4 or 8, connect.go:266-284 — would sum
 * its header to the floored DataOffset() and leave the option bytes past it
 * out of the sum, a value the receiver's check rejects; this mode sums them
 * as data, as the receiver does. Measured by executing the reference,
 * DESIGN.md §2.) */
#define YU_MODE_TCP 2
/* pkt_i = IPv4 datagram. out[i] = ^IPv4.CalculateChecksum() over
 * b[:IHL*4] (clamped to len) with the header-checksum field taken as 0 —
 * network/ipv4/ipv4.go:80-97, header/ipv4.go:146-157,177-179. initial and
 * addrs are ignored. */
#define YU_MODE_IPV4 3
/* pkt_i = ICMPv4 message (4-byte header + data). out[i] =
 * ^Checksum(hdr, Checksum(data, 0)) with the checksum field taken as 0 —
 * network/ipv4/icmp.go:36-45. initial and addrs are ignored. */
#define YU_MODE_ICMP 4
/* Receive-side verification, checker semantics (checker/checker.go:25-40):
 * out[i] = Checksum(b[:IHL*4] clamped to len, 0) INCLUDING the stored field. The packet is
 * valid iff out[i] is 0x0000 or 0xFFFF. */
#define YU_MODE_VERIFY_IPV4 5
/* checker.TCP (checker/checker.go:71-99): out[i] = Checksum over
 * pseudo ‖ BE16(len) ‖ segment INCLUDING the stored field. Valid iff
 * out[i] ∈ {0, 0xFFFF}. Protocol 6. */
#define YU_MODE_VERIFY_TCP 6
/* The same verification for UDP datagrams (protocol 17). The reference
 * never verifies on receive (transport/udp/endpoint.go:191-229); this is
 * the checker.TCP formula applied to UDP. */
#define YU_MODE_VERIFY_UDP 7
/* Receive-side verification of whole IPv4 packets as a tun device delivers
 * them (link/tundev/tundev.go:78-114 -> network/ipv4/ipv4.go:62-77): the
 * composition of checker.IPv4 and checker.TCP's checksum test
 * (checker/checker.go:25-40,71-92), all inputs taken from the packet itself:
 *   valid  = len >= 20 && HeaderLength() <= TotalLength() <= len
 *            (IPv4.IsValid, header/ipv4.go:126-138)
 *   IP ok  = Checksum(b[:HeaderLength()], 0) in {0, 0xFFFF}
 *   L4     = valid && Protocol() in {6 TCP, 17 UDP, 1 ICMP}
 *   L4 ok  = Checksum(Payload(), Checksum(BE16(len(Payload())),
 *            PseudoHeaderChecksum(proto, src, dst))) in {0, 0xFFFF}, with
 *            Payload() = b[HeaderLength():TotalLength()]; ICMP without the
 *            pseudo-header and length (network/ipv4/icmp.go:36-45).
 * out[i] is a bit set of YU_RX_*. No side arrays; not a fill mode. */
#define YU_MODE_VERIFY_RX 8
/* Transmit side of whole IPv4 datagrams as the link endpoint writes them
 * (network/ipv4/ipv4.go:80-97 WritePacket after sendUDP
 * transport/udp/endpoint.go:164-187, sendTCP transport/tcp/connect.go:556-586
 * or sendICMPv4 network/ipv4/icmp.go:36-45; written out by
 * link/tundev/tundev.go:171-196): both checksum fields of a datagram in one
 * pass, all inputs taken from the datagram itself. TWO results per packet:
 *   out[2i]   = the IPv4 header checksum WritePacket stores: YU_MODE_IPV4's
 *               value, ^Checksum(b[:HeaderLength()]) with the field as 0;
 *   out[2i+1] = the transport checksum its sender stores, over the segment
 *               b[HeaderLength():TotalLength()] with the pseudo-header from
 *               the datagram's source, destination and protocol and the
 *               length TotalLength() - HeaderLength(): YU_MODE_UDP (17),
 *               YU_MODE_TCP (6) or YU_MODE_ICMP (1) on that segment, field as
 *               0; 0 when the protocol is another one or the segment is
 *               shorter than its header (8 / 20 / 4 bytes).
 * Datagrams must satisfy 20 <= HeaderLength() <= TotalLength() <= len (every
 * datagram WritePacket encodes: IHL 5); others get {0, 0} and, in place,
 * no write. TCP segments need 20 <= DataOffset() <= their length (as
 * YU_MODE_TCP). With fill, each field whose value is defined is stored
 * big-endian in place. No side arrays (initial / addrs are ignored). */
#define YU_MODE_TX_DATAGRAM 9
#define YU_MODE_COUNT 10

/* Results per packet in `out`: 2 for YU_MODE_TX_DATAGRAM, 1 otherwise. Every
 * out / h_out array below holds n * YU_MODE_OUTPUTS(mode) uint16 values. */
#define YU_MODE_OUTPUTS(mode) ((mode) == YU_MODE_TX_DATAGRAM ? 2 : 1)

#define YU_RX_IP_OK 1u   /* header checksum verifies */
#define YU_RX_L4 2u      /* transport (TCP/UDP/ICMP) present and checked */
#define YU_RX_L4_OK 4u   /* transport checksum verifies */
#define YU_RX_INVALID 8u /* IPv4.IsValid fails (nothing else is set) */

/* Packets handed to the transport/IPv4/ICMP modes must be <= 65535 bytes
 * (the IPv4 total-length limit; the reference's uint16 length arithmetic is
 * only defined there). RAW packets may be up to YU_MAX_RAW_LEN bytes
 * (4 GiB - 64 KiB; the reference's uint32 wrap is reproduced throughout).
 * The uniform calls reject longer packets with YU_EINVAL; a ragged batch
 * is not read back on the host, so a longer ragged packet gets an
 * unspecified value (never a fault or a hang). */
#define YU_MAX_TRANSPORT_LEN 65535u
#define YU_MAX_RAW_LEN 0xFFFF0000u

/* ------------------------------------------------------------------ */
/* Batched device entry points (the GPU hot path).                     */
/* All pointers are device pointers (hipMalloc / torch CUDA tensors).   */
/* `stream` is a hipStream_t (NULL = legacy default stream).            */
/* Asynchronous: returns after enqueueing the kernel.                   */
/* ------------------------------------------------------------------ */

/* Uniform-stride batch: packet i occupies data[i*stride, i*stride + len).
 * Packets may overlap (stride < len) — they are only read.
 *  initial_arr: NULL or n uint16 (per-packet initial / pseudo partial)
 *  initial:     used when initial_arr == NULL
 *  addrs:       NULL or n*8 bytes {src[4], dst[4]} (UDP/TCP/VERIFY_TCP/UDP)
 *  out:         n * YU_MODE_OUTPUTS(mode) uint16 results, written in host
 *               byte order as numbers (store one big-endian into the packet
 *               to set its field). */
int yu_csum_batch_uniform(const uint8_t *data, uint64_t stride, uint32_t len,
                          uint64_t n, int mode,
                          const uint16_t *initial_arr, uint16_t initial,
                          const uint8_t *addrs, uint16_t *out, void *stream);

/* Ragged batch (tun-style back-to-back packets, any byte alignment):
 * packet i occupies data[offsets[i], offsets[i+1]); offsets is a device
 * array of n+1 non-decreasing uint64 (the layout of buffer.VectorisedView
 * flattened, buffer/view.go:37-46). */
int yu_csum_batch_ragged(const uint8_t *data, const uint64_t *offsets,
                         uint64_t n, int mode,
                         const uint16_t *initial_arr, uint16_t initial,
                         const uint8_t *addrs, uint16_t *out, void *stream);

/* In-place field writer (TX modes UDP/TCP/IPV4/ICMP/TX_DATAGRAM only):
 * computes the same value as the matching batch call and stores it
 * big-endian into the packet's checksum field (UDP.SetChecksum
 * header/udp.go:60-62, TCP.SetChecksum header/tcp.go:156-158,
 * IPv4.SetChecksum header/ipv4.go:165-167, ICMPv4.SetChecksum
 * header/icmpv4.go:46-48; both fields of a datagram in TX_DATAGRAM).
 * `out` may be NULL. `data` is written: the fields only (see Preconditions
 * above: [fill-mode]; the uniform form also [fill-align], [fill-overlap];
 * the ragged form takes any alignment). */
int yu_csum_fill_uniform(uint8_t *data, uint64_t stride, uint32_t len,
                         uint64_t n, int mode,
                         const uint16_t *initial_arr, uint16_t initial,
                         const uint8_t *addrs, uint16_t *out, void *stream);
int yu_csum_fill_ragged(uint8_t *data, const uint64_t *offsets, uint64_t n,
                        int mode, const uint16_t *initial_arr,
                        uint16_t initial, const uint8_t *addrs, uint16_t *out,
                        void *stream);

/* ------------------------------------------------------------------ */
/* Batched host entry point (host memory in, host memory out).         */
/* ------------------------------------------------------------------ */

/* Same contract as yu_csum_batch_uniform but every pointer is a HOST
 * pointer (pageable or pinned). The batch is cut into slices that are
 * staged through library-owned pinned buffers on `device` and pipelined
 * (H2D of slice k+1 overlaps the kernel of slice k and the D2H of slice
 * k-1). Synchronous: returns when h_out is complete. Thread-safe: each call
 * borrows one staging context of `device` from a bounded pool and returns it
 * (see yu_host_staging_bytes below). */
int yu_csum_batch_host_uniform(const uint8_t *h_data, uint64_t stride,
                               uint32_t len, uint64_t n, int mode,
                               const uint16_t *h_initial_arr,
                               uint16_t initial, const uint8_t *h_addrs,
                               uint16_t *h_out, int device);

/* The same for a ragged host batch: packet i = h_data[h_offsets[i],
 * h_offsets[i+1]) (a tun read burst packed back to back). The offsets are
 * host memory and are validated here (non-decreasing, packet lengths within
 * the mode's limit), then shipped rebased with each slice. */
int yu_csum_batch_host_ragged(const uint8_t *h_data, const uint64_t *h_offsets,
                              uint64_t n, int mode,
                              const uint16_t *h_initial_arr, uint16_t initial,
                              const uint8_t *h_addrs, uint16_t *h_out,
                              int device);

/* Scatter-gather packets, as the tun endpoint reads them into several views
 * (link/tundev/tundev.go:116-125; buffer.VectorisedView, buffer/view.go:
 * 37-46): packet i is the concatenation of iov[first_iov[i]] ..
 * iov[first_iov[i+1] - 1]. The views are gathered into the library's pinned
 * staging while earlier slices are on the GPU. Layout-compatible with
 * struct iovec. */
typedef struct yu_iovec {
  const void *base;
  uint64_t len;
} yu_iovec;

int yu_csum_batch_host_iov(const yu_iovec *iov, const uint64_t *first_iov,
                           uint64_t n, int mode, const uint16_t *h_initial_arr,
                           uint16_t initial, const uint8_t *h_addrs,
                           uint16_t *h_out, int device);

/* Host-memory field writer: the matching yu_csum_batch_host_* call (TX modes
 * UDP/TCP/IPV4/ICMP/TX_DATAGRAM only), then each result stored big-endian into the
 * packet's checksum field in host memory, as the device writer does
 * (yu_csum_fill_uniform). `h_out` may be NULL. The iov form writes through
 * the views (their `base` must be writable memory). Synchronous. */
int yu_csum_fill_host_uniform(uint8_t *h_data, uint64_t stride, uint32_t len,
                              uint64_t n, int mode,
                              const uint16_t *h_initial_arr, uint16_t initial,
                              const uint8_t *h_addrs, uint16_t *h_out,
                              int device);
int yu_csum_fill_host_ragged(uint8_t *h_data, const uint64_t *h_offsets,
                             uint64_t n, int mode,
                             const uint16_t *h_initial_arr, uint16_t initial,
                             const uint8_t *h_addrs, uint16_t *h_out,
                             int device);
int yu_csum_fill_host_iov(const yu_iovec *iov, const uint64_t *first_iov,
                          uint64_t n, int mode, const uint16_t *h_initial_arr,
                          uint16_t initial, const uint8_t *h_addrs,
                          uint16_t *h_out, int device);

/* Multi-GPU host path (SURVEY.md §8b `yu_csum_batch_host(..., ngpu)`, §8e):
 * the same three calls with the batch split into ndev contiguous shards, one
 * per entry of `devices` (a device may be listed more than once), each shard
 * run through the single-device pipeline on that device by a persistent
 * per-device worker thread, all at once. Packets are independent, so there
 * is no exchange: shard i writes h_out[first_i, first_i + n_i). Uniform and
 * iovec batches split by packet count, ragged batches on the packet boundary
 * nearest an even split of the bytes (balanced PCIe traffic). Synchronous;
 * returns the first failing shard's status (YU_EINVAL for ndev < 1 or > 64,
 * YU_ENODEV for a device index out of range). */
int yu_csum_batch_host_uniform_multi(const uint8_t *h_data, uint64_t stride,
                                     uint32_t len, uint64_t n, int mode,
                                     const uint16_t *h_initial_arr,
                                     uint16_t initial, const uint8_t *h_addrs,
                                     uint16_t *h_out, const int *devices,
                                     int ndev);
int yu_csum_batch_host_ragged_multi(const uint8_t *h_data,
                                    const uint64_t *h_offsets, uint64_t n,
                                    int mode, const uint16_t *h_initial_arr,
                                    uint16_t initial, const uint8_t *h_addrs,
                                    uint16_t *h_out, const int *devices,
                                    int ndev);
int yu_csum_batch_host_iov_multi(const yu_iovec *iov, const uint64_t *first_iov,
                                 uint64_t n, int mode,
                                 const uint16_t *h_initial_arr,
                                 uint16_t initial, const uint8_t *h_addrs,
                                 uint16_t *h_out, const int *devices, int ndev);

/* ------------------------------------------------------------------ */
/* Host-path staging (the yu_csum_batch_host_* / yu_csum_fill_host_*   */
/* calls, and each shard of the _multi forms).                          */
/* ------------------------------------------------------------------ */

/* A host call borrows one staging context of its device for its own length
 * and returns it; a caller that finds every context in use waits for one.
 * There are two pools per device: bulk contexts (3 pipeline slots) and burst
 * contexts (1 slot) for the calls that take the direct path (one slice of at
 * most 4 MiB: a tun read burst), so a burst never waits behind bulk batches
 * that hold every bulk context. Contexts are created on first need, up to
 * yu_host_contexts() per pool and device: YU_HOST_CONTEXTS in the environment
 * (1..64, default 4; a product setting, read without the YU_TUNING gate). So
 * the staging grows with the calls the pools let run at once, not with the
 * number of OS threads that ever called (the Go consumer calls from many
 * goroutines, which migrate across OS threads: transport/tcp/accept.go:238,
 * transport/tcp/endpoint.go:229, network/ipv4/icmp.go:30-34).
 *
 * A bulk context holds 3 pipeline slots of at most one slice each: up to
 * YU_HOST_SLICE_BYTES of packet bytes and YU_HOST_SLICE_PACKETS packets'
 * side arrays; a burst context one slot of at most 4 MiB and as many
 * packets. Between calls a device's staging is therefore at most
 * yu_host_contexts() * (YU_HOST_CONTEXT_PINNED_MAX +
 * YU_HOST_BURST_CONTEXT_PINNED_MAX) bytes of pinned host memory and
 * yu_host_contexts() * (YU_HOST_CONTEXT_DEVICE_MAX +
 * YU_HOST_BURST_CONTEXT_DEVICE_MAX) of device memory (a packet longer than a
 * slice gets a slice of its own for that call; the context gives the extra
 * back when the call returns). */
#define YU_HOST_SLICE_BYTES (32ull << 20)
#define YU_HOST_SLICE_PACKETS (1ull << 18)
#define YU_HOST_CONTEXT_PINNED_MAX \
  (3ull * (YU_HOST_SLICE_BYTES + 26ull * YU_HOST_SLICE_PACKETS + 72ull))
#define YU_HOST_CONTEXT_DEVICE_MAX \
  (3ull * (YU_HOST_SLICE_BYTES + 22ull * YU_HOST_SLICE_PACKETS + 8ull))
#define YU_HOST_BURST_CONTEXT_PINNED_MAX \
  ((4ull << 20) + 26ull * YU_HOST_SLICE_PACKETS + 72ull)
#define YU_HOST_BURST_CONTEXT_DEVICE_MAX \
  ((4ull << 20) + 22ull * YU_HOST_SLICE_PACKETS + 8ull)

/* The pool bound K (YU_HOST_CONTEXTS, clamped to 1..64), per pool. */
int yu_host_contexts(void);
/* Pinned host bytes the host-path staging of `device` holds now (idle and
 * lent contexts); the device bytes go to *dev_bytes when it is not NULL.
 * 0 for a device never used or out of range. Never fails. */
uint64_t yu_host_staging_bytes(int device, uint64_t *dev_bytes);
/* Frees the staging of every idle context of `device` (a later call
 * allocates again). YU_ENODEV for a device out of range. */
int yu_host_staging_trim(int device);

/* ------------------------------------------------------------------ */
/* Introspection.                                                      */
/* ------------------------------------------------------------------ */
int yu_abi_version(void);
const char *yu_strerror(int status);
/* Number of HIP devices (0 when none / no driver). Never fails. */
int yu_device_count(void);
/* Path of the HIP runtime (libamdhip64) this library's HIP calls are bound
 * to, as the dynamic loader resolved them (dladdr of the library's own
 * reference to hipGetDevice); NULL if it cannot be told. No device needed.
 * A process with two HIP runtimes (PyTorch-ROCm bundles one) must have this
 * library bound to the runtime the rest of the process uses: the Python
 * loader checks it ("One HIP runtime per process"). */
const char *yu_hip_runtime_path(void);
/* Name of the kernel variant the uniform path would launch for this shape
 * (for profiling and tests; no device needed). Returns a static string. */
const char *yu_uniform_variant(uint64_t stride, uint32_t len, int mode,
                               uint64_t data_align16);
/* The same for a batch of n packets (the choice above 3 KiB depends on n;
 * yu_uniform_variant answers for n = 2). */
const char *yu_uniform_variant_n(uint64_t stride, uint32_t len, uint64_t n,
                                 int mode, uint64_t data_align16);
/* Name of the kernel variant the ragged path launches for this mode (static
 * string; "" for a bad mode), for a large batch; _n: for a batch of n
 * packets (bursts of up to 4096 packets take a wave per packet). */
const char *yu_ragged_variant(int mode);
const char *yu_ragged_variant_n(int mode, uint64_t n);
/* The kernel variant yu_csum_fill_ragged launches for a batch of n packets (the
 * TX modes write in place through their own k_seg form). */
const char *yu_ragged_fill_variant_n(int mode, uint64_t n);

#ifdef __cplusplus
}
#endif

#endif /* YUCSUM_H */
