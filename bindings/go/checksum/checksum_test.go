package checksum

import (
	"math/rand"
	"testing"
)

// refChecksum is the reference loop (checksum/checksum.go:4-18) restated for
// comparison; it is test-only.
func refChecksum(buf []byte, initial uint16) uint16 {
	v := uint32(initial)
	l := len(buf)
	if l&1 != 0 {
		l--
		v += uint32(buf[l]) << 8
	}
	for i := 0; i < l; i += 2 {
		v += (uint32(buf[i]) << 8) + uint32(buf[i+1])
	}
	return ChecksumCombine(uint16(v), uint16(v>>16))
}

func TestRFC1071(t *testing.T) {
	if got := Checksum([]byte{0x00, 0x01, 0xf2, 0x03, 0xf4, 0xf5, 0xf6, 0xf7}, 0); got != 0xddf2 {
		t.Fatalf("got 0x%x want 0xddf2", got)
	}
}

func TestAgainstReferenceLoop(t *testing.T) {
	r := rand.New(rand.NewSource(1))
	for i := 0; i < 2000; i++ {
		b := make([]byte, r.Intn(5000))
		r.Read(b)
		init := uint16(r.Intn(65536))
		if Checksum(b, init) != refChecksum(b, init) {
			t.Fatalf("len %d", len(b))
		}
	}
	ff := make([]byte, 131074)
	for i := range ff {
		ff[i] = 0xff
	}
	if Checksum(ff, 0xffff) != 65534 {
		t.Fatal("uint32 wrap")
	}
}

func BenchmarkChecksum1500(b *testing.B) {
	buf := make([]byte, 1500)
	b.SetBytes(1500)
	for i := 0; i < b.N; i++ {
		Checksum(buf, 0)
	}
}

// TestShortArgumentsRejected: too-short side arrays and a data slice that a
// wrapping size product would let through are errors, never reads past the Go
// allocation (no device needed: the checks run before any C call).
func TestShortArgumentsRejected(t *testing.T) {
	data := make([]byte, 4*100)
	out := make([]uint16, 4)
	if BatchHostUniform(data, 100, 100, 4, ModeRaw, make([]uint16, 3), nil, out, 0) == nil {
		t.Fatal("initial shorter than n accepted")
	}
	if BatchHostUniform(data, 100, 100, 4, ModeUDP, nil, make([]byte, 31), out, 0) == nil {
		t.Fatal("addrs shorter than 8n accepted")
	}
	if BatchHostUniform(data, 1<<63, 100, 3, ModeRaw, nil, nil, out, 0) == nil {
		t.Fatal("wrapping (n-1)*stride accepted")
	}
	if BatchHostUniform(data, 100, 500, 1, ModeRaw, nil, nil, out, 0) == nil {
		t.Fatal("length past data accepted")
	}
	offs := []uint64{0, 100, 200, 300, 400}
	if BatchHostRagged(data, offs, ModeRaw, make([]uint16, 2), nil, out) == nil {
		t.Fatal("ragged: short initial accepted")
	}
}

// TestStagingIsBounded: goroutines calling at once (the Go runtime spreads them
// over OS threads) share at most HostContexts() staging contexts, so the pinned
// staging held afterwards stays within that many contexts' bound
// (include/yucsum.h, Host-path staging), and a trim frees it.
func TestStagingIsBounded(t *testing.T) {
	const n, L = 12000, 1500 // 18 MB: the sliced pipeline
	data := make([]byte, n*L)
	for i := range data {
		data[i] = byte(i * 7)
	}
	errs := make(chan error, 32)
	for g := 0; g < 32; g++ {
		go func() {
			out := make([]uint16, n)
			errs <- BatchHostUniform(data, L, L, n, ModeRaw, nil, nil, out, 0)
		}()
	}
	for g := 0; g < 32; g++ {
		if err := <-errs; err == ErrNoDevice {
			t.Skip("no HIP device")
		} else if err != nil {
			t.Fatal(err)
		}
	}
	pinned, _ := HostStaging(0)
	if bound := uint64(HostContexts()) * HostContextPinnedMax; pinned == 0 || pinned > bound {
		t.Fatalf("pinned staging %d, bound %d", pinned, bound)
	}
	if err := HostStagingTrim(0); err != nil {
		t.Fatal(err)
	}
	if pinned, _ = HostStaging(0); pinned != 0 {
		t.Fatalf("%d pinned bytes after a trim", pinned)
	}
}
