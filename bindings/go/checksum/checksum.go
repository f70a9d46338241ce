// Package checksum is a drop-in replacement for yustack's package checksum
// (github.com/YaoZengzeng/yustack/checksum, reference checksum/checksum.go).
//
// The three package functions keep their exact signatures, so header/ipv4.go,
// header/tcp.go, header/udp.go, types/route.go, transport/udp/endpoint.go,
// transport/tcp/connect.go, network/ipv4/icmp.go and checker/checker.go build
// unchanged. They bind the scalar entry points of the C ABI (include/yucsum.h,
// libyucsum.so). Batches go to the GPU through BatchHostUniform, BatchHostRagged
// and BatchHostPackets (a tun read burst as [][]byte, no copy on the Go side).
//
// Status: written against the C ABI; not compiled in the build container (it
// has no Go toolchain). Needs Go >= 1.21 (runtime.Pinner, unsafe.Slice). See INTEGRATION.md for how to build and swap it in.
package checksum

/*
#cgo CFLAGS: -I${SRCDIR}/../../../include
#cgo LDFLAGS: -L${SRCDIR}/../../../yustack_amd -lyucsum -Wl,-rpath,${SRCDIR}/../../../yustack_amd
#include <stdlib.h>
#include "yucsum.h"
*/
import "C"

import (
	"errors"
	"fmt"
	"runtime"
	"unsafe"
)

// cgoMin is the buffer length below which the sum stays in Go: a cgo call
// costs ~100 ns, more than summing a 20-byte header.
const cgoMin = 256

// Checksum calculates the checksum of the bytes in the given byte array
// (reference checksum/checksum.go:4-18). Not complemented.
func Checksum(buf []byte, initial uint16) uint16 {
	if len(buf) < cgoMin {
		return goSum(buf, initial)
	}
	return uint16(C.yu_checksum((*C.uint8_t)(unsafe.Pointer(&buf[0])), C.size_t(len(buf)),
		C.uint16_t(initial)))
}

// goSum: the same uint32 accumulation (wrap included) for short buffers.
func goSum(buf []byte, initial uint16) uint16 {
	v := uint32(initial)
	n := len(buf)
	if n&1 != 0 {
		n--
		v += uint32(buf[n]) << 8
	}
	for i := 0; i < n; i += 2 {
		v += uint32(buf[i])<<8 | uint32(buf[i+1])
	}
	return ChecksumCombine(uint16(v), uint16(v>>16))
}

// PseudoHeaderChecksum calculates the pseudo header checksum for the given
// destination protocol and network addresses, ignoring the length field
// (reference checksum/checksum.go:24-28).
func PseudoHeaderChecksum(protocol uint32, srcAddr string, dstAddr string) uint16 {
	xsum := Checksum([]byte(srcAddr), 0)
	xsum = Checksum([]byte(dstAddr), xsum)
	return Checksum([]byte{0, uint8(protocol)}, xsum)
}

// ChecksumCombine combines the two uint16 to form their checksum
// (reference checksum/checksum.go:32-35).
func ChecksumCombine(a, b uint16) uint16 {
	v := uint32(a) + uint32(b)
	return uint16(v + v>>16)
}

// Mode selects the reference composition a batch reproduces (include/yucsum.h).
type Mode int

const (
	ModeRaw        Mode = C.YU_MODE_RAW
	ModeUDP        Mode = C.YU_MODE_UDP
	ModeTCP        Mode = C.YU_MODE_TCP
	ModeIPv4       Mode = C.YU_MODE_IPV4
	ModeICMP       Mode = C.YU_MODE_ICMP
	ModeVerifyIPv4 Mode = C.YU_MODE_VERIFY_IPV4
	ModeVerifyTCP  Mode = C.YU_MODE_VERIFY_TCP
	ModeVerifyUDP  Mode = C.YU_MODE_VERIFY_UDP
	ModeVerifyRX   Mode = C.YU_MODE_VERIFY_RX // out[i] = RX* bits
	// whole outgoing IPv4 datagrams: out[2i] = IPv4 header field, out[2i+1] =
	// transport field (two results per packet, see Outputs)
	ModeTxDatagram Mode = C.YU_MODE_TX_DATAGRAM
)

// Outputs is the number of results per packet a mode writes to out
// (include/yucsum.h YU_MODE_OUTPUTS): 2 for ModeTxDatagram, else 1.
func (m Mode) Outputs() uint64 {
	if m == ModeTxDatagram {
		return 2
	}
	return 1
}

// VERIFY_RX result bits (include/yucsum.h YU_RX_*).
const (
	RXIPOk    = C.YU_RX_IP_OK
	RXL4      = C.YU_RX_L4
	RXL4Ok    = C.YU_RX_L4_OK
	RXInvalid = C.YU_RX_INVALID
)

// ErrNoDevice is returned when no MI355X (HIP device) is usable.
var ErrNoDevice = errors.New("checksum: no HIP device")

// BatchHostUniform computes one result per packet of a uniform-stride batch in
// host memory (packet i = data[i*stride : i*stride+length]) on GPU `device`.
// initial (len n) and addrs (len 8n, {src[4], dst[4]}) are optional. The C
// side copies into its own pinned staging and retains no Go pointer.
func BatchHostUniform(data []byte, stride uint64, length uint32, n uint64, mode Mode,
	initial []uint16, addrs []byte, out []uint16, device int) error {
	if n == 0 {
		return nil
	}
	// overflow-safe form of (n-1)*stride+length <= len(data)
	if uint64(len(out))/mode.Outputs() < n || uint64(length) > uint64(len(data)) ||
		(n > 1 && stride > (uint64(len(data))-uint64(length))/(n-1)) {
		return errTooSmall
	}
	if err := checkSide(n, initial, addrs); err != nil {
		return err
	}
	var pd *C.uint8_t
	if len(data) > 0 {
		pd = (*C.uint8_t)(unsafe.Pointer(&data[0]))
	}
	pi, pa := sideArgs(initial, addrs)
	return status(C.yu_csum_batch_host_uniform(pd, C.uint64_t(stride),
		C.uint32_t(length), C.uint64_t(n), C.int(mode), pi, 0, pa,
		(*C.uint16_t)(unsafe.Pointer(&out[0])), C.int(device)))
}

var errTooSmall = errors.New("checksum: batch buffers too small")

// checkSide rejects optional side arrays shorter than the batch: the C calls
// read n initial values (2n bytes) and n address records (8n bytes).
func checkSide(n uint64, initial []uint16, addrs []byte) error {
	if len(initial) > 0 && uint64(len(initial)) < n {
		return fmt.Errorf("checksum: initial has %d values for %d packets", len(initial), n)
	}
	if len(addrs) > 0 && (n > uint64(len(addrs))/8) {
		return fmt.Errorf("checksum: addrs has %d bytes for %d packets (8 each)", len(addrs), n)
	}
	return nil
}

func status(rc C.int) error {
	switch {
	case rc == C.YU_OK:
		return nil
	case rc == C.YU_ENODEV:
		return ErrNoDevice
	default:
		return fmt.Errorf("checksum: %s (%d)", C.GoString(C.yu_strerror(rc)), int(rc))
	}
}

// sideArgs returns the optional per-packet side arrays as C pointers.
func sideArgs(initial []uint16, addrs []byte) (*C.uint16_t, *C.uint8_t) {
	var pi *C.uint16_t
	if len(initial) > 0 {
		pi = (*C.uint16_t)(unsafe.Pointer(&initial[0]))
	}
	var pa *C.uint8_t
	if len(addrs) > 0 {
		pa = (*C.uint8_t)(unsafe.Pointer(&addrs[0]))
	}
	return pi, pa
}

// deviceList turns the optional device list into the C (pointer, count) pair
// of the *_multi calls; a []C.int holds no Go pointers, so it may be passed.
func deviceList(devices []int) ([]C.int, int) {
	if len(devices) == 0 {
		devices = []int{0}
	}
	d := make([]C.int, len(devices))
	for i, v := range devices {
		d[i] = C.int(v)
	}
	return d, len(d)
}

// BatchHostRagged computes one result per packet of a burst packed back to
// back in host memory: packet i = data[offsets[i]:offsets[i+1]] (len(offsets)
// = n+1). initial (n) and addrs (8n) are optional. With several devices the
// burst is split into one shard per GPU (yu_csum_batch_host_ragged_multi).
func BatchHostRagged(data []byte, offsets []uint64, mode Mode, initial []uint16, addrs []byte,
	out []uint16, devices ...int) error {
	if len(offsets) < 2 {
		return nil
	}
	n := uint64(len(offsets) - 1)
	if uint64(len(out))/mode.Outputs() < n || offsets[n] > uint64(len(data)) {
		return errTooSmall
	}
	if err := checkSide(n, initial, addrs); err != nil {
		return err
	}
	var pd *C.uint8_t
	if len(data) > 0 {
		pd = (*C.uint8_t)(unsafe.Pointer(&data[0]))
	}
	pi, pa := sideArgs(initial, addrs)
	d, nd := deviceList(devices)
	return status(C.yu_csum_batch_host_ragged_multi(pd, (*C.uint64_t)(unsafe.Pointer(&offsets[0])),
		C.uint64_t(n), C.int(mode), pi, 0, pa, (*C.uint16_t)(unsafe.Pointer(&out[0])), &d[0], C.int(nd)))
}

// BatchHostPackets computes one result per packet of a burst given as one
// slice per packet (buffer.View, buffer/view.go:4), gathered by the library
// into its pinned staging (see withPackets).
func BatchHostPackets(pkts [][]byte, mode Mode, initial []uint16, addrs []byte, out []uint16,
	devices ...int) error {
	if len(pkts) == 0 {
		return nil
	}
	if uint64(len(out))/mode.Outputs() < uint64(len(pkts)) {
		return errTooSmall
	}
	if err := checkSide(uint64(len(pkts)), initial, addrs); err != nil {
		return err
	}
	pi, pa := sideArgs(initial, addrs)
	d, nd := deviceList(devices)
	return withPackets(pkts, func(iov *C.yu_iovec, first *C.uint64_t, n C.uint64_t) C.int {
		return C.yu_csum_batch_host_iov_multi(iov, first, n, C.int(mode), pi, 0, pa,
			(*C.uint16_t)(unsafe.Pointer(&out[0])), &d[0], C.int(nd))
	})
}

// FillHostPackets is the batched TX step of sendUDP / sendTCP / WritePacket /
// sendICMPv4: for each outgoing packet (one slice, as Encode left it, field 0)
// it computes the checksum and stores it big-endian into the packet's field
// in place, like SetChecksum (header/udp.go:60-62, header/tcp.go:156-158,
// header/ipv4.go:165-167, header/icmpv4.go:46-48). mode is ModeUDP, ModeTCP,
// ModeIPv4, ModeICMP or ModeTxDatagram (both fields of whole datagrams); out
// (n results, 2n for ModeTxDatagram) may be nil.
func FillHostPackets(pkts [][]byte, mode Mode, initial []uint16, addrs []byte, out []uint16,
	device int) error {
	if len(pkts) == 0 {
		return nil
	}
	var po *C.uint16_t
	if out != nil {
		if uint64(len(out))/mode.Outputs() < uint64(len(pkts)) {
			return errTooSmall
		}
		po = (*C.uint16_t)(unsafe.Pointer(&out[0]))
	}
	if err := checkSide(uint64(len(pkts)), initial, addrs); err != nil {
		return err
	}
	pi, pa := sideArgs(initial, addrs)
	return withPackets(pkts, func(iov *C.yu_iovec, first *C.uint64_t, n C.uint64_t) C.int {
		return C.yu_csum_fill_host_iov(iov, first, n, C.int(mode), pi, 0, pa, po, C.int(device))
	})
}

// withPackets passes one view per packet to call as a C iovec array. The
// views' Go memory is pinned (runtime.Pinner) for the call, because the
// C-allocated array holds pointers into it; the library keeps none of them.
func withPackets(pkts [][]byte, call func(*C.yu_iovec, *C.uint64_t, C.uint64_t) C.int) error {
	n := len(pkts)
	var pin runtime.Pinner
	defer pin.Unpin()
	iov := unsafe.Slice((*C.yu_iovec)(C.malloc(C.size_t(n)*C.size_t(unsafe.Sizeof(C.yu_iovec{})))), n)
	defer C.free(unsafe.Pointer(&iov[0]))
	first := make([]uint64, n+1)
	for i, p := range pkts {
		if len(p) > 0 {
			pin.Pin(&p[0])
			iov[i].base = unsafe.Pointer(&p[0])
		} else {
			iov[i].base = nil
		}
		iov[i].len = C.uint64_t(len(p))
		first[i+1] = uint64(i + 1)
	}
	return status(call(&iov[0], (*C.uint64_t)(unsafe.Pointer(&first[0])), C.uint64_t(n)))
}
