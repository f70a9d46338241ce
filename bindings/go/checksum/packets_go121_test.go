//go:build go1.21
// +build go1.21

package checksum

import "testing"

// TestBatchHostPackets checks the GPU burst path against the scalar package
// (skipped without a HIP device).
func TestBatchHostPackets(t *testing.T) {
	pkts := make([][]byte, 1000)
	for i := range pkts {
		pkts[i] = make([]byte, 40+(i*37)%1461)
		for j := range pkts[i] {
			pkts[i][j] = byte(i*131 + j*7)
		}
	}
	out := make([]uint16, len(pkts))
	if err := BatchHostPackets(pkts, ModeRaw, nil, nil, out); err == ErrNoDevice {
		t.Skip("no HIP device")
	} else if err != nil {
		t.Fatal(err)
	}
	for i, p := range pkts {
		if want := Checksum(p, 0); out[i] != want {
			t.Fatalf("packet %d: got %#x want %#x", i, out[i], want)
		}
	}
	var blob []byte
	offs := []uint64{0}
	for _, p := range pkts {
		blob = append(blob, p...)
		offs = append(offs, uint64(len(blob)))
	}
	out2 := make([]uint16, len(pkts))
	if err := BatchHostRagged(blob, offs, ModeRaw, nil, nil, out2, 0, 0); err != nil {
		t.Fatal(err)
	}
	for i := range out {
		if out2[i] != out[i] {
			t.Fatalf("ragged packet %d: got %#x want %#x", i, out2[i], out[i])
		}
	}
}

// FillHostPackets sets each ICMP echo's checksum field in place: afterwards every
// packet sums to 0xFFFF, as checker-style verification expects, and the value
// stored is the complement of the sum with the field zero (sendICMPv4,
// network/ipv4/icmp.go:36-45).
func TestFillHostPackets(t *testing.T) {
	pkts := make([][]byte, 500)
	want := make([]uint16, len(pkts))
	for i := range pkts {
		pkts[i] = make([]byte, 8+(i*29)%1400)
		for j := range pkts[i] {
			pkts[i][j] = byte(i*17 + j*3)
		}
		pkts[i][2], pkts[i][3] = 0, 0
		want[i] = ^Checksum(pkts[i], 0)
	}
	if err := FillHostPackets(pkts, ModeICMP, nil, nil, nil, 0); err == ErrNoDevice {
		t.Skip("no HIP device")
	} else if err != nil {
		t.Fatal(err)
	}
	for i, p := range pkts {
		if got := uint16(p[2])<<8 | uint16(p[3]); got != want[i] {
			t.Fatalf("packet %d: field %#x want %#x", i, got, want[i])
		}
		if s := Checksum(p, 0); s != 0xffff {
			t.Fatalf("packet %d: sums to %#x after fill", i, s)
		}
	}
}

// TestShortPacketArgumentsRejected: the per-packet calls check their side
// arrays before any C call, like TestShortArgumentsRejected.
func TestShortPacketArgumentsRejected(t *testing.T) {
	data := make([]byte, 4*100)
	out := make([]uint16, 4)
	pkts := [][]byte{data[:100], data[100:200]}
	if BatchHostPackets(pkts, ModeUDP, nil, make([]byte, 8), out) == nil {
		t.Fatal("packets: short addrs accepted")
	}
	if FillHostPackets(pkts, ModeUDP, make([]uint16, 1), nil, nil, 0) == nil {
		t.Fatal("fill: short initial accepted")
	}
}

// TestFillTxDatagram: ModeTxDatagram sets both fields of whole outgoing IPv4
// datagrams (header checksum at 10, UDP checksum at 20+6); out receives the two
// values per datagram. Afterwards the header sums to 0xFFFF and so does the UDP
// segment with its pseudo-header (checked with the scalar package, as
// network/ipv4/ipv4.go and transport/udp do on receive).
func TestFillTxDatagram(t *testing.T) {
	pkts := make([][]byte, 300)
	for i := range pkts {
		n := 28 + (i*41)%1400
		p := make([]byte, n)
		for j := range p {
			p[j] = byte(i*7 + j*13)
		}
		p[0], p[9] = 0x45, 17 // IPv4, IHL 5, UDP
		p[2], p[3] = byte(n>>8), byte(n)
		p[24], p[25] = byte((n-20)>>8), byte(n-20)
		pkts[i] = p
	}
	out := make([]uint16, 2*len(pkts))
	if FillHostPackets(pkts, ModeTxDatagram, nil, nil, out[:len(pkts)], 0) == nil {
		t.Fatal("out with one slot per datagram accepted")
	}
	if err := FillHostPackets(pkts, ModeTxDatagram, nil, nil, out, 0); err == ErrNoDevice {
		t.Skip("no HIP device")
	} else if err != nil {
		t.Fatal(err)
	}
	for i, p := range pkts {
		if s := Checksum(p[:20], 0); s != 0xffff {
			t.Fatalf("datagram %d: header sums to %#x", i, s)
		}
		if got := uint16(p[10])<<8 | uint16(p[11]); got != out[2*i] {
			t.Fatalf("datagram %d: header field %#x, out %#x", i, got, out[2*i])
		}
		ph := Checksum(p[12:20], 17+uint16(len(p)-20))
		if s := Checksum(p[20:], ph); s != 0xffff {
			t.Fatalf("datagram %d: UDP segment sums to %#x", i, s)
		}
		if got := uint16(p[26])<<8 | uint16(p[27]); got != out[2*i+1] {
			t.Fatalf("datagram %d: UDP field %#x, out %#x", i, got, out[2*i+1])
		}
	}
}
