"""tests/golden/goexec.py (the Go-subset interpreter the fixture generator runs the
reference's source with) on small Go programs of its own, so its semantics are
checked without the reference present: wrapping typed integers, slices, structs and
composite literals, pointer receivers, closures, variadics, range, nil slices, 3-index
slices and Go's bounds panics."""
import os
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
import goexec as G  # noqa: E402

SRC = r'''
package demo

import (
	"encoding/binary"
	"errors"
	"log"
	"unsafe"
)

type Counter struct {
	n    int
	name string
	buf  []byte
}

type Bytes []byte

const (
	first = iota * 2
	second
	third
)

func (c *Counter) Add(k int) int {
	c.n += k
	return c.n
}

func (b Bytes) Sum() uint16 {
	var s uint16
	for i := 0; i < len(b); i++ {
		s += uint16(b[i]) << 8
	}
	return s
}

func NewCounter(k int) *Counter {
	return &Counter{n: k, name: "c"}
}

func Apply(fs ...func(int) int) int {
	t := 0
	for _, f := range fs {
		t = f(t)
	}
	return t
}

func Adder(k int) func(int) int {
	return func(x int) int { return x + k }
}

func Wrap8(a uint8, b uint8) uint8 {
	return a + b
}

func Cut(b []byte) int {
	c := b[1:3:4]
	return cap(c)*10 + len(c)
}

func BE(b []byte) uint32 {
	binary.BigEndian.PutUint16(b[2:], 0xBEEF)
	log.Printf("ignored")
	return binary.BigEndian.Uint32(b)
}

func NilLen(b []byte) int {
	if b == nil {
		return -1
	}
	return len(b)
}

func Third() int {
	return third
}

type Kind int

func (k Kind) Double() int {
	return int(k) * 2
}

var table = []int{5, 7, 9}

var errShort = errors.New("short")

func Classify(x int) string {
	switch {
	case x < 0:
		return "neg"
	case x == 0, x == 100:
		return "edge"
	default:
		return "pos"
	}
}

func Tag(k Kind) int {
	switch k {
	case 1, 2:
		return 10
	case 3:
		return 30
	}
	return -1
}

func Pair(a, b int) (int, int) {
	return b, a
}

func Swap(a, b int) int {
	x, y := Pair(a, b)
	return x*10 + y
}

func Words(n int) int {
	w := make([]uint16, n)
	w[n-1] = 65535
	w[n-1]++
	return len(w) + int(w[n-1]) + table[2]
}

func Check(b []byte) error {
	if len(b) < 2 {
		return errShort
	}
	return nil
}

func Addr(b []byte) *uint8 {
	return (*uint8)(unsafe.Pointer(&b[1]))
}
'''


class _Err:
    def __init__(self, m):
        self.m = m


@pytest.fixture(scope="module")
def it(tmp_path_factory):
    d = tmp_path_factory.mktemp("gosrc") / "demo"
    d.mkdir()
    (d / "demo.go").write_text(SRC)
    i = G.Interp(str(d.parent))
    i.stubs.update({"errors.New": lambda m: _Err(m.b), "unsafe.Pointer": lambda x: x})
    i.load("demo")
    return i


def test_structs_pointer_receivers_and_literals(it):
    c = it.call("demo", "NewCounter", G.Int(5, "int"))
    assert isinstance(c, G.Struct) and c.f["n"].v == 5 and c.f["buf"] is None
    assert it.method("demo", c, "Add", G.Int(7, "int")).v == 12
    assert c.f["n"].v == 12  # the pointer receiver changed the value in place


def test_closures_variadics_and_range(it):
    fs = [it.call("demo", "Adder", G.Int(k, "int")) for k in (1, 10, 100)]
    assert it.call("demo", "Apply", *fs).v == 111
    assert it.call("demo", "Apply").v == 0


def test_typed_wrap_slices_and_binary(it):
    assert it.call("demo", "Wrap8", G.Int(200, "uint8"), G.Int(100, "uint8")).v == 44
    assert it.method("demo", G.from_bytes(b"\x01\x02", "Bytes"), "Sum").v == 0x0300
    assert it.call("demo", "Cut", G.from_bytes(b"abcdef")).v == 32  # cap 3, len 2
    assert it.call("demo", "BE", G.from_bytes(b"\x12\x34\x00\x00")).v == 0x1234BEEF
    assert it.call("demo", "NilLen", None).v == -1
    assert it.call("demo", "NilLen", G.from_bytes(b"")).v == 0
    assert it.call("demo", "Third").v == 4


def test_bounds_panic(it):
    with pytest.raises(G.GoPanic):
        it.call("demo", "Cut", G.from_bytes(b"ab"))


def test_switch_vars_named_types_multi_assign(it):
    """cgo-shim constructs: tagless and tagged switch, package-level vars (initialised
    on first use), methods on a named integer type, multi-value assignment and
    `make([]uint16, n)` with uint16 wrap."""
    assert [it.call("demo", "Classify", G.Int(x, "int")).b for x in (-3, 0, 100, 5)] == \
        [b"neg", b"edge", b"edge", b"pos"]
    assert [it.call("demo", "Tag", G.Int(k, "Kind")).v for k in (1, 2, 3, 4)] == [10, 10, 30, -1]
    k = it.call("demo", "Tag", G.Int(3, "Kind"))
    assert k.v == 30
    assert it.method("demo", G.Int(21, "Kind"), "Double").v == 42
    assert it.call("demo", "Swap", G.Int(1, "int"), G.Int(2, "int")).v == 21
    assert it.call("demo", "Words", G.Int(3, "int")).v == 3 + 0 + 9
    e = it.call("demo", "Check", G.from_bytes(b"a"))
    assert isinstance(e, _Err) and e is it.call("demo", "Check", G.from_bytes(b""))  # one var, one value
    assert it.call("demo", "Check", G.from_bytes(b"ab")) is None


def test_element_reference_and_pointer_conversion(it):
    """`&b[1]` is a reference into the slice (what a cgo call is handed), passed through
    `unsafe.Pointer` and a `(*T)(x)` conversion unchanged; `&b[1]` of a 1-byte slice
    panics, as Go's bounds check does."""
    b = G.from_bytes(b"xyz")
    r = it.call("demo", "Addr", b)
    assert isinstance(r, G.Ref) and r.s.buf is b.buf and r.i == 1 and r.s.get(r.i).v == ord("y")
    with pytest.raises(G.GoPanic):
        it.call("demo", "Addr", G.from_bytes(b"x"))
