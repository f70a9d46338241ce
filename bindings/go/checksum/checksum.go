// Package checksum is a drop-in replacement for yustack's package checksum
// (github.com/YaoZengzeng/yustack/checksum, reference checksum/checksum.go).
//
// The three package functions keep their exact signatures, so header/ipv4.go,
// header/tcp.go, header/udp.go, types/route.go, transport/udp/endpoint.go,
// transport/tcp/connect.go, network/ipv4/icmp.go and checker/checker.go build
// unchanged. They bind the scalar entry points of the C ABI (include/yucsum.h,
// libyucsum.so). Batches go to the GPU through BatchHostUniform and
// BatchHostRagged (batch.go) and, from Go 1.21, BatchHostPackets /
// FillHostPackets (packets_go121.go: a tun burst as [][]byte, no copy on the
// Go side).
//
// Toolchain floors, per file: this file and batch.go use nothing past Go 1.10
// (cgo, unsafe.Pointer conversions), because the reference's unchanged callers
// need a Go of that era (INTEGRATION.md §2: sleep/sleep_unsafe.go:66-67 links
// runtime.gopark with its Go 1.10 signature); packets_go121.go needs Go 1.21
// (runtime.Pinner, unsafe.Slice) and is left out of older builds by its build
// constraint. Status: written against the C ABI; not compiled in the build
// container (it has no Go toolchain). See INTEGRATION.md for how to swap it in.
package checksum

/*
#cgo CFLAGS: -I${SRCDIR}/../../../include
#cgo LDFLAGS: -L${SRCDIR}/../../../yustack_amd -lyucsum -Wl,-rpath,${SRCDIR}/../../../yustack_amd
#include <stdlib.h>
#include "yucsum.h"
*/
import "C"

import "unsafe"

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

