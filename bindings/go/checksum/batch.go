package checksum

// Batched calls on host memory that need nothing past Go 1.10: one Go pointer
// per argument (data, offsets, side arrays, out), each to memory that holds no
// Go pointers, so the cgo pointer rules of every Go release allow them. The
// #cgo flags are in checksum.go.

/*
#include <stdlib.h>
#include "yucsum.h"
*/
import "C"

import (
	"errors"
	"fmt"
	"unsafe"
)

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


// HostStaging reports the pinned host and device bytes the host path's staging
// holds for device now (include/yucsum.h yu_host_staging_bytes). Each call
// borrows one of at most HostContexts() contexts of its device and kind (bulk,
// or burst for the small direct calls), so between calls this stays within
// HostContexts() * HostContextPinnedMax pinned bytes however many OS threads a
// program's goroutines have run on.
func HostStaging(device int) (pinned, dev uint64) {
	var d C.uint64_t
	p := C.yu_host_staging_bytes(C.int(device), &d)
	return uint64(p), uint64(d)
}

// HostContextPinnedMax is the pinned bytes of one bulk and one burst staging
// context at most, between calls (include/yucsum.h YU_HOST_CONTEXT_PINNED_MAX +
// YU_HOST_BURST_CONTEXT_PINNED_MAX): HostContexts() of each per device.
// A plain literal, not an expression over the header's macros, which cgo would have
// to evaluate (the cgo build is unverified here, INTEGRATION.md §2):
// 3*(32 MiB + 26*2^18 + 72) + (4 MiB + 26*2^18 + 72). tests/test_bindings.py checks it
// against include/yucsum.h.
const HostContextPinnedMax uint64 = 132120864

// HostContexts is the bound on staging contexts per device (YU_HOST_CONTEXTS,
// default 4, read once from the environment).
func HostContexts() int { return int(C.yu_host_contexts()) }

// HostStagingTrim frees the staging of the device's idle contexts.
func HostStagingTrim(device int) error { return status(C.yu_host_staging_trim(C.int(device))) }
