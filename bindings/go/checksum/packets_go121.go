//go:build go1.21
// +build go1.21

package checksum

// Bursts given as one slice per packet. The C side receives an iovec array
// that holds pointers into Go memory, which cgo allows only while that memory
// is pinned (runtime.Pinner, Go 1.21); older toolchains build the package
// without this file (use BatchHostRagged on a packed burst there).

/*
#include <stdlib.h>
#include "yucsum.h"
*/
import "C"

import (
	"runtime"
	"unsafe"
)

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
// (n results, 2n for ModeTxDatagram) may be nil. Like SetChecksum it has no
// alignment precondition: the CPU stores each field wherever it lies. The
// errors it returns are include/yucsum.h's Preconditions ([fill-mode] for
// another mode; [len-transport] for a packet over 65535 bytes; [iov-view]).
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
