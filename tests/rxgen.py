"""Received-packet batches for the VERIFY_RX mode (test data, not product).

Packets are whole IPv4 datagrams as a tun device delivers them
(link/tundev/tundev.go:78-114): an IPv4 header (IHL 5..15, options random) and a
TCP, UDP, ICMP or other payload, with both checksums filled the way the
reference's senders fill them (network/ipv4/ipv4.go:80-97 for the header;
transport/tcp/connect.go:556-586, transport/udp/endpoint.go:164-187,
network/ipv4/icmp.go:36-45 for the transport). A share of them is then damaged
— a flipped header or payload byte, a wrong total length, a truncated packet,
trailing bytes past the total length — so every YU_RX_* outcome occurs.
The expected flags always come from the oracle, never from this generator.
"""
import numpy as np

from oracle import oracle as O


def _fill16(buf, off, value):
    buf[off] = (value >> 8) & 0xFF
    buf[off + 1] = value & 0xFF


def make_packet(rng, plen, proto=None, ihl=None):
    proto = int(rng.choice([6, 17, 1, 47])) if proto is None else proto
    ihl = int(rng.integers(5, 16)) if ihl is None else ihl
    hl = 4 * ihl
    if proto == 6:
        plen = max(plen, 20)
    elif proto == 17:
        plen = max(plen, 8)
    elif proto == 1:
        plen = max(plen, 4)
    tl = hl + plen
    pkt = bytearray(rng.integers(0, 256, size=tl, dtype=np.uint8).tobytes())
    pkt[0] = 0x40 | ihl
    _fill16(pkt, 2, tl)
    pkt[9] = proto
    pkt[10] = pkt[11] = 0
    _fill16(pkt, 10, ~O.checksum(bytes(pkt[:hl]), 0) & 0xFFFF)
    src, dst = bytes(pkt[12:16]), bytes(pkt[16:20])
    seg = hl
    if proto == 6:
        pkt[seg + 12] = int(rng.integers(5, min(15, plen // 4) + 1)) << 4
        pkt[seg + 16] = pkt[seg + 17] = 0
        xs = O.pseudo_header_checksum(6, src, dst)
        xs = O.checksum(bytes([(plen >> 8) & 0xFF, plen & 0xFF]), xs)
        _fill16(pkt, seg + 16, ~O.checksum(bytes(pkt[seg:]), xs) & 0xFFFF)
    elif proto == 17:
        _fill16(pkt, seg + 4, plen)
        pkt[seg + 6] = pkt[seg + 7] = 0
        xs = O.pseudo_header_checksum(17, src, dst)
        xs = O.checksum(bytes([(plen >> 8) & 0xFF, plen & 0xFF]), xs)
        _fill16(pkt, seg + 6, ~O.checksum(bytes(pkt[seg:]), xs) & 0xFFFF)
    elif proto == 1:
        pkt[seg + 2] = pkt[seg + 3] = 0
        _fill16(pkt, seg + 2, ~O.checksum(bytes(pkt[seg:]), 0) & 0xFFFF)
    return pkt


def damage(rng, pkt):
    r = rng.random()
    hl = (pkt[0] & 0xF) * 4
    if r < 0.15:  # header byte
        i = int(rng.integers(0, hl))
        pkt[i] ^= 1 << int(rng.integers(0, 8))
    elif r < 0.30 and len(pkt) > hl:  # payload byte
        i = int(rng.integers(hl, len(pkt)))
        pkt[i] ^= 1 << int(rng.integers(0, 8))
    elif r < 0.35:  # total length beyond the packet
        _fill16(pkt, 2, len(pkt) + int(rng.integers(1, 100)))
    elif r < 0.38:  # truncated below the minimum header
        del pkt[int(rng.integers(0, 20)):]
    elif r < 0.41:  # total length below the header length
        _fill16(pkt, 2, int(rng.integers(0, hl)))
    elif r < 0.50:  # trailing bytes past the total length (IsValid accepts)
        pkt += bytes(rng.integers(0, 256, size=int(rng.integers(1, 64)), dtype=np.uint8))
    return pkt


def rx_batch(rng, n, lo=0, hi=1480, bad=0.5):
    """Ragged blob + offsets of n received packets with payloads in [lo, hi]."""
    pkts = []
    for _ in range(n):
        p = make_packet(rng, int(rng.integers(lo, hi + 1)))
        if rng.random() < bad:
            p = damage(rng, p)
        pkts.append(bytes(p))
    offs = np.zeros(n + 1, np.uint64)
    offs[1:] = np.cumsum([len(p) for p in pkts])
    return np.frombuffer(b"".join(pkts), dtype=np.uint8).copy(), offs


def short_header_packet(rng, total):
    """A received datagram of `total` >= 20 bytes whose IPv4 header length is under
    20 bytes (IHL 0..4, which IsValid accepts: header/ipv4.go:126-138), with a total
    length that is often under 20 too, so the header and transport end points both
    fall inside the first 20 bytes. Some have an IP sum that checks (IHL 0, or IHL
    >= 2 with the ID field set to make the sum 0xFFFF), some an ICMP payload that
    is empty (transport sum 0), some a total length past the packet (invalid)."""
    pkt = bytearray(rng.integers(0, 256, size=total, dtype=np.uint8).tobytes())
    ihl = int(rng.integers(0, 5))
    hl = 4 * ihl
    r = rng.random()
    if r < 0.3:
        tl = hl
    elif r < 0.7:
        tl = int(rng.integers(hl, 20))
    elif r < 0.9:
        tl = int(rng.integers(hl, total + 1))
    else:
        tl = total + int(rng.integers(1, 50))  # IsValid: tl > pktSize
    pkt[0] = 0x40 | ihl
    _fill16(pkt, 2, tl)
    pkt[9] = int(rng.choice([6, 17, 1, 47]))
    if hl >= 8 and rng.random() < 0.5:  # ID field chosen so the header sums to 0xFFFF
        pkt[4] = pkt[5] = 0
        _fill16(pkt, 4, (0xFFFF - O.checksum(bytes(pkt[:hl]), 0)) & 0xFFFF)
    return pkt


def filler_packet(rng, total):
    """A `total`-byte datagram with a plain IHL-5 header (tl = total, random
    protocol) and unfixed checksums: it only moves the next packet's start."""
    pkt = bytearray(rng.integers(0, 256, size=total, dtype=np.uint8).tobytes())
    if total >= 20:
        pkt[0] = 0x45
        _fill16(pkt, 2, total)
        pkt[9] = int(rng.choice([6, 17, 1, 47]))
    return pkt


def tx_packet(rng, plen, proto=None, ihl=None, pad4=False):
    """An outgoing datagram for TX_DATAGRAM: built like the reference's senders
    (make_packet), then both checksum fields overwritten with random bytes (the
    mode takes them as 0). pad4: trailing bytes up to a multiple of 4 (past
    TotalLength, which the contract allows), for the in-place writer's 4-aligned
    offsets."""
    pkt = make_packet(rng, plen, proto=proto, ihl=ihl)
    hl = (pkt[0] & 0xF) * 4
    pkt[10:12] = rng.integers(0, 256, size=2, dtype=np.uint8).tobytes()
    f = {17: 6, 6: 16, 1: 2}.get(pkt[9])
    if f is not None:
        pkt[hl + f: hl + f + 2] = rng.integers(0, 256, size=2, dtype=np.uint8).tobytes()
    if pad4 and len(pkt) % 4:
        pkt += rng.integers(0, 256, size=4 - len(pkt) % 4, dtype=np.uint8).tobytes()
    return pkt


def tcp_contract(pkt):
    """Keep a damaged outgoing datagram inside YU_MODE_TCP's contract (20 <=
    DataOffset <= segment length, as every segment sendTCP encodes): a flipped
    header byte can move the segment so that its DataOffset byte is payload. The
    datagram may still leave the IPv4 contract (its fields are then not set)."""
    if len(pkt) >= 20:
        hl, tl = (pkt[0] & 0xF) * 4, (pkt[2] << 8) | pkt[3]
        if 20 <= hl <= tl <= len(pkt) and pkt[9] == 6 and tl - hl >= 20:
            doff = (pkt[hl + 12] >> 4) * 4
            if doff < 20 or doff > tl - hl:
                pkt[hl + 12] = 0x50 | (pkt[hl + 12] & 0x0F)
    return pkt


def tx_batch(rng, n, lo=0, hi=1480, bad=0.1, pad4=False):
    """Ragged blob + offsets of n outgoing datagrams (tx_packet), a share of them
    damaged or malformed (damage: some leave the TX contract, some do not)."""
    pkts = []
    for _ in range(n):
        p = tx_packet(rng, int(rng.integers(lo, hi + 1)), pad4=pad4)
        if rng.random() < bad:
            p = tcp_contract(damage(rng, p))
            if pad4 and len(p) % 4:
                p += bytes(4 - len(p) % 4)
        pkts.append(bytes(p))
    offs = np.zeros(n + 1, np.uint64)
    offs[1:] = np.cumsum([len(p) for p in pkts])
    return np.frombuffer(b"".join(pkts), dtype=np.uint8).copy(), offs


def tile_edge_batch(rng, n, chunk, base_off, tile=4096, special=None):
    """Ragged RX batch whose short-header packets (short_header_packet, or
    `special(rng, total)`) start so that
    floor4(start) lies 4..20 bytes before a tile boundary of k_seg's chunk-relative
    tiling (b0 = floor4 of the chunk's first start; boundaries every `tile` bytes,
    both the 4 KiB and the 8 KiB ones). Each is preceded by a filler sized to put
    it there. Returns (blob incl. base_off leading bytes + 32 slack, offsets)."""
    pkts, offs = [], [base_off]
    pos = base_off
    b0 = 0
    special_next = False
    for i in range(n):
        if i % chunk == 0:
            b0 = pos & ~3
        if special_next:
            p = (special or short_header_packet)(rng, int(rng.integers(20, 81)))
            special_next = False
        else:
            d = 4 * int(rng.integers(1, 6))
            s = int(rng.integers(0, 4))
            m = -(-(pos + 40 - b0) // tile)  # first boundary leaving a >= 20-byte filler
            start = b0 + m * tile - d + s
            p = filler_packet(rng, start - pos)
            special_next = (i + 1) % chunk != 0  # the next packet stays in this chunk
        pkts.append(bytes(p))
        pos += len(p)
        offs.append(pos)
    blob = np.zeros(pos + 32, np.uint8)
    blob[base_off:pos] = np.frombuffer(b"".join(pkts), np.uint8)
    return blob, np.array(offs, np.uint64)
