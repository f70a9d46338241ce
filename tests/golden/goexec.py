"""A minimal interpreter for the Go subset yustack's checksum path is written in.

TEST INFRASTRUCTURE ONLY (fixture generation). The reference is Go and this image
has no Go toolchain, so the reference cannot be compiled. This module executes the
reference's own source files (read from /root/reference at generation time, never
copied) with Go's semantics for the constructs they use:

* typed integer arithmetic that wraps at the type's width (uint8/16/32/64, int);
  untyped constants; Go's operator precedence (`<<`, `>>`, `&` bind tighter than `+`);
* slices over shared backing arrays, with Go's bounds checks (a panic is an exception);
* strings and `[]byte(s)` conversions, `[]byte{...}` literals, `make([]byte, n)`;
* named slice types with methods (`type TCP []byte`, `func (b TCP) ...`);
* `const` blocks with `iota`, `:=`, `=`, `op=`, `++`, `--`, `if`, 3-clause `for`,
  `for k, v := range`, `return`, package-qualified calls across the loaded packages,
  and `encoding/binary.BigEndian` (stdlib, restated);
* struct types (zero values per field type), keyed and positional composite literals,
  `&T{...}`, pointer receivers, field reads and stores, 3-index slices, slices of
  non-byte values (`[]header.Network{ipv4}`), function literals (closures over their
  scope), variadic parameters, and calls through interface values (dispatch on the
  concrete value, as Go does at run time).

Struct values are shared, not copied, on assignment: the code the path executes never
copies a struct and then changes both copies. Values from outside the loaded packages
(a `*testing.T`, a link endpoint, `log.Printf`) are Python stubs the caller supplies.

For cgo code (this repo's own Go shim, bindings/go/checksum, run by
tests/test_go_shim_exec.py): package-level `var`s (initialised on first use), `switch`,
`make([]T, n)` for non-byte T, multi-value assignment, `&s[i]` as a reference into the
slice, and `(*T)(x)` conversions; `C.*` names and `unsafe.Pointer` are stubs the caller
supplies (the test binds them to the C ABI through ctypes).

Function bodies are parsed lazily, when first called, so code the path does not reach
(options parsing, the TCP state machine, ...) is only skipped over.
tests/golden/make_refexec.py uses it to produce known-answer vectors "from the
reference itself": checksum/checksum.go, header/{ipv4,tcp,udp,icmpv4}.go, the senders
(transport/udp/endpoint.go sendUDP, transport/tcp/connect.go sendTCP /
sendTCPWithOptions, network/ipv4/icmp.go sendICMPv4, network/ipv4/ipv4.go
WritePacket, types/route.go, buffer/prependable.go) and checker/checker.go.
"""
from __future__ import annotations

import os
import re

WIDTH = {"uint8": 8, "byte": 8, "uint16": 16, "uint32": 32, "uint64": 64, "uint": 64,
         "int8": 8, "int16": 16, "int32": 32, "int64": 64, "int": 64}
SIGNED = {"int8", "int16", "int32", "int64", "int"}
# named integer types (`type Mode int`) -> their underlying type: an Int keeps the
# named type (methods dispatch on it) and wraps at the underlying width
NAMED_INT = {}


class GoPanic(Exception):
    pass


# ----------------------------------------------------------------------------- values
class Int:
    __slots__ = ("v", "t")

    def __init__(self, v, t="untyped"):
        if t == "byte":
            t = "uint8"
        self.t = t
        self.v = wrap(v, t)

    def __repr__(self):
        return f"{self.t}({self.v})"


def wrap(v, t):
    if t == "untyped":
        return v
    t = NAMED_INT.get(t, t)
    w = WIDTH[t]
    v &= (1 << w) - 1
    if t in SIGNED and v >= 1 << (w - 1):
        v -= 1 << w
    return v


class Slice:
    """A []byte (or named byte-slice type) over a shared bytearray."""
    __slots__ = ("buf", "off", "len", "cap", "t")

    def __init__(self, buf, off, n, cap, t="[]byte"):
        self.buf, self.off, self.len, self.cap, self.t = buf, off, n, cap, t

    def get(self, i):
        if not 0 <= i < self.len:
            raise GoPanic(f"index out of range [{i}] with length {self.len}")
        return Int(self.buf[self.off + i], "uint8")

    def set(self, i, x):
        if not 0 <= i < self.len:
            raise GoPanic(f"index out of range [{i}] with length {self.len}")
        self.buf[self.off + i] = x & 0xFF

    def sub(self, lo, hi):
        hi = self.len if hi is None else hi
        if not 0 <= lo <= hi <= self.cap:
            raise GoPanic(f"slice bounds out of range [{lo}:{hi}] with capacity {self.cap}")
        return Slice(self.buf, self.off + lo, hi - lo, self.cap - lo, self.t)

    def bytes(self):
        return bytes(self.buf[self.off:self.off + self.len])


def from_bytes(b, t="[]byte"):
    ba = bytearray(b)
    return Slice(ba, 0, len(ba), len(ba), t)


class Str:
    __slots__ = ("b", "t")

    def __init__(self, b, t="string"):
        self.b, self.t = bytes(b), t


class Struct:
    """A struct value (or the value a pointer to it points at): fields by name."""
    __slots__ = ("t", "pkg", "f")

    def __init__(self, t, pkg, fields):
        self.t, self.pkg, self.f = t, pkg, fields

    def __repr__(self):
        return f"{self.t}{self.f}"


class GoList:
    """A slice of non-byte values ([]header.Network, variadic parameters)."""
    __slots__ = ("items", "t")

    def __init__(self, items, t="[]"):
        self.items, self.t = list(items), t

    @property
    def len(self):
        return len(self.items)

    def get(self, i):
        if not 0 <= i < len(self.items):
            raise GoPanic(f"index out of range [{i}] with length {len(self.items)}")
        return self.items[i]

    def set(self, i, x):
        self.get(i)
        self.items[i] = x


class Ref:
    """`&s[i]`: element i of a slice (the start of the memory a cgo call is handed)."""
    __slots__ = ("s", "i")

    def __init__(self, s, i):
        self.s, self.i = s, i


class Closure:
    """A function literal with the scopes it closes over; `owner` names the function
    it was created in (for Interp.watch)."""
    __slots__ = ("params", "body", "env", "pkg", "owner")

    def __init__(self, params, body, env, pkg, owner):
        self.params, self.body, self.env, self.pkg, self.owner = params, body, env, pkg, owner


class GoFatal(Exception):
    """t.Fatalf from a stub *testing.T: ends the checker, as runtime.Goexit does."""


# ----------------------------------------------------------------------------- lexer
TOK = re.compile(r"""
 (?P<ws>[ \t\r]+) | (?P<nl>\n) | (?P<lc>//[^\n]*) | (?P<bc>/\*.*?\*/)
|(?P<num>0[xX][0-9a-fA-F_]+|0[bB][01_]+|0[oO][0-7_]+|[0-9][0-9_]*)
|(?P<str>"(?:[^"\\\n]|\\.)*"|`[^`]*`)
|(?P<chr>'(?:[^'\\\n]|\\.)*')
|(?P<id>[A-Za-z_][A-Za-z0-9_]*)
|(?P<op>&\^=|<<=|>>=|\.\.\.|&&|\|\||<-|\+\+|--|==|!=|<=|>=|:=|\+=|-=|\*=|/=|%=|&=|\|=|\^=|<<|>>|&\^|[-+*/%&|^<>=!()\[\]{},;.:~])
""", re.S | re.X)
SEMI_AFTER = {"break", "continue", "fallthrough", "return", "++", "--", ")", "]", "}"}


def lex(src):
    out = []
    pos = 0
    while pos < len(src):
        m = TOK.match(src, pos)
        if not m:
            raise SyntaxError(f"bad token at {src[pos:pos + 20]!r}")
        pos = m.end()
        k = m.lastgroup
        if k in ("ws", "lc"):
            continue
        if k == "nl" or (k == "bc" and "\n" in m.group()):
            if out and (out[-1][0] in ("id", "num", "str", "chr") or out[-1][1] in SEMI_AFTER):
                out.append(("op", ";"))
            continue
        if k == "bc":
            continue
        out.append((k, m.group()))
    out.append(("op", ";"))
    out.append(("eof", ""))
    return out


# ----------------------------------------------------------------------------- parser
PREC = {"||": 1, "&&": 2, "==": 3, "!=": 3, "<": 3, "<=": 3, ">": 3, ">=": 3,
        "+": 4, "-": 4, "|": 4, "^": 4, "*": 5, "/": 5, "%": 5, "<<": 5, ">>": 5, "&": 5, "&^": 5}


class Parser:
    def __init__(self, toks, i=0):
        self.t, self.i = toks, i
        self.nolit = False  # inside an if / for header: `x {` opens the block

    def peek(self, k=0):
        return self.t[self.i + k]

    def val(self, k=0):
        return self.t[self.i + k][1]

    def next(self):
        tok = self.t[self.i]
        self.i += 1
        return tok

    def expect(self, v):
        tok = self.next()
        if tok[1] != v:
            raise SyntaxError(f"expected {v!r}, got {tok[1]!r} near token {self.i}")
        return tok

    def accept(self, v):
        if self.val() == v:
            self.i += 1
            return True
        return False

    def skip_balanced(self):
        """Skip one balanced (...)/[...]/{...} group starting at the current token."""
        pairs = {"(": ")", "[": "]", "{": "}"}
        depth = []
        while True:
            v = self.next()[1]
            if v in pairs:
                depth.append(pairs[v])
            elif depth and v == depth[-1]:
                depth.pop()
                if not depth:
                    return

    # --- types: names, qualified names, []T, [N]T, *T, ...T; map / chan / func /
    # struct / interface types are skipped over (only their name is kept)
    def parse_type(self):
        if self.accept("..."):
            return "..." + self.parse_type()
        if self.accept("["):
            if self.accept("]"):
                return "[]" + self.parse_type()
            n = self.expr()
            self.expect("]")
            return "[" + (str(n[1].v) if n[0] == "lit" else "?") + "]" + self.parse_type()
        if self.accept("*"):
            return "*" + self.parse_type()
        if self.val() == "map":
            self.next()
            self.skip_balanced()
            self.parse_type()
            return "map"
        if self.val() == "chan":
            self.next()
            self.parse_type()
            return "chan"
        if self.val() == "func":
            self.next()
            self.skip_balanced()
            if self.val() == "(":
                self.skip_balanced()
            elif self.peek()[0] == "id" or self.val() in ("[", "*"):
                self.parse_type()
            return "func"
        if self.val() in ("struct", "interface"):
            self.next()
            self.skip_balanced()
            return "struct{}"
        name = self.next()[1]
        if self.val() == "." and self.peek(1)[0] == "id":
            self.next()
            name = name + "." + self.next()[1]
        return name

    def struct_fields(self):
        """`struct { a, b T; C }` after the keyword: [(name, type)]."""
        self.expect("{")
        out = []
        while not self.accept("}"):
            if self.accept(";"):
                continue
            names = [self.next()[1]]
            while self.accept(","):
                names.append(self.next()[1])
            if self.val() in (";", "}") or self.peek()[0] == "str":  # embedded field
                t = names[0]
            else:
                t = self.parse_type()
            if self.peek()[0] == "str":  # field tag
                self.next()
            out += [(nm, t) for nm in names]
        return out

    def params(self):
        """A parameter list after its "(": [(name or None, type)]."""
        params, pending = [], []
        while not self.accept(")"):
            if self.peek()[0] != "id" and self.val() not in ("...",):
                pending.append(self.parse_type())  # unnamed: a type
                self.accept(",")
                continue
            nm = self.next()[1]
            if self.val() in (",", ")"):
                pending.append(nm)
                self.accept(",")
                continue
            if self.val() == ".":  # a qualified type with no name
                self.i -= 1
                pending.append(self.parse_type())
                self.accept(",")
                continue
            t = self.parse_type()
            for q in pending + [nm]:
                params.append((q, t))
            pending = []
            self.accept(",")
        for q in pending:  # unnamed params: types only
            params.append((None, q))
        return params

    # --- expressions
    def expr(self, prec=1):
        lhs = self.unary()
        while True:
            op = self.val()
            p = PREC.get(op)
            if p is None or p < prec or self.peek()[0] != "op":
                return lhs
            self.next()
            rhs = self.expr(p + 1)
            lhs = ("bin", op, lhs, rhs)

    def unary(self):
        v = self.val()
        if self.peek()[0] == "op" and v in ("-", "+", "!", "^", "&", "*"):
            self.next()
            return ("un", v, self.unary())
        return self.primary()

    def primary(self):
        kind, v = self.next()
        if kind == "num":
            x = ("lit", Int(int(v.replace("_", ""), 0)))
        elif kind == "str":
            s = v[1:-1] if v[0] == "`" else bytes(v[1:-1], "utf-8").decode("unicode_escape").encode("latin-1")
            x = ("lit", Str(s if isinstance(s, bytes) else s.encode()))
        elif kind == "chr":
            x = ("lit", Int(ord(bytes(v[1:-1], "utf-8").decode("unicode_escape"))))
        elif v == "(":
            x = self.expr()
            self.expect(")")
        elif v == "[":  # []byte{...} literal or []byte(x) conversion
            self.expect("]")
            t = "[]" + self.parse_type()
            if self.val() == "{":
                self.next()
                elems = []
                while not self.accept("}"):
                    elems.append(self.expr())
                    self.accept(",")
                x = ("slicelit", t, elems)
            else:
                x = ("name", t)
        elif v == "func":  # function literal
            self.expect("(")
            params = self.params()
            while self.val() != "{":
                if self.val() == "(":
                    self.skip_balanced()
                else:
                    self.parse_type()
            x = ("funclit", params, self.block())
        elif kind == "id":
            x = ("name", v)
        else:
            raise SyntaxError(f"unexpected {v!r}")
        while True:
            v = self.val()
            if v == "{" and not self.nolit and self._typeish(x):  # composite literal
                x = ("complit", x, self.complit_body())
                continue
            if v == ".":
                self.next()
                x = ("sel", x, self.next()[1])
            elif v == "(":
                self.next()
                args = []
                while not self.accept(")"):
                    args.append(self.expr())
                    self.accept(",")
                x = ("call", x, args)
            elif v == "[":
                self.next()
                lo = None if self.val() == ":" else self.expr()
                if self.accept(":"):
                    hi = None if self.val() in ("]", ":") else self.expr()
                    mx = self.expr() if self.accept(":") else None
                    self.expect("]")
                    x = ("slice", x, lo, hi, mx)
                else:
                    self.expect("]")
                    x = ("index", x, lo)
            else:
                return x

    @staticmethod
    def _typeish(x):
        """A composite literal's type: a name starting with a capital or lower letter
        that is a type (resolved at run time), or pkg.Name."""
        return x[0] == "name" and not x[1].startswith("[]") or (x[0] == "sel" and x[1][0] == "name")

    def complit_body(self):
        """`{k: v, ...}` or `{v, ...}`: [(key or None, expr)]."""
        self.expect("{")
        out = []
        while not self.accept("}"):
            if self.accept(";"):
                continue
            e = self.expr()
            if self.accept(":"):
                out.append((e[1], self.expr()))
            else:
                out.append((None, e))
            self.accept(",")
        return out

    # --- statements
    def block(self):
        self.expect("{")
        saved, self.nolit = self.nolit, False
        out = []
        while not self.accept("}"):
            if self.accept(";"):
                continue
            out.append(self.stmt())
        self.nolit = saved
        return out

    def simple(self):
        lhs = [self.expr()]
        while self.accept(","):
            lhs.append(self.expr())
        v = self.val()
        if v in (":=", "=") or (v.endswith("=") and v[:-1] in PREC):
            self.next()
            rhs = [self.expr()]
            while self.accept(","):
                rhs.append(self.expr())
            return ("assign", v, lhs, rhs)
        if v in ("++", "--"):
            self.next()
            return ("assign", "+=" if v == "++" else "-=", lhs, [("lit", Int(1))])
        return ("expr", lhs[0])

    def stmt(self):
        v = self.val()
        if v == "return":
            self.next()
            vals = []
            if self.val() not in (";", "}"):
                vals.append(self.expr())
                while self.accept(","):
                    vals.append(self.expr())
            return ("return", vals)
        if v == "if":
            self.next()
            init = None
            self.nolit = True
            s = self.simple()
            if self.accept(";"):
                init, s = s, self.simple()
            self.nolit = False
            body = self.block()
            els = None
            if self.accept("else"):
                els = [self.stmt()] if self.val() == "if" else self.block()
            return ("if", init, s[1], body, els)
        if v == "for":
            self.next()
            init = cond = post = None
            self.nolit = True
            j = self.i  # `for k, v := range x {`
            while self.t[j][1] not in ("{", ";", "range"):
                j += 1
            if self.t[j][1] == "range":
                keys = [] if self.val() == "range" else [self.expr()]
                while self.accept(","):
                    keys.append(self.expr())
                define = self.accept(":=")
                if not define:
                    self.accept("=")
                self.expect("range")
                x = self.expr()
                self.nolit = False
                return ("range", keys, define, x, self.block())
            if self.val() != "{":
                s = self.simple()
                if self.accept(";"):
                    init = s
                    cond = None if self.val() == ";" else self.simple()[1]
                    self.expect(";")
                    post = None if self.val() == "{" else self.simple()
                else:
                    cond = s[1]
            self.nolit = False
            return ("for", init, cond, post, self.block())
        if v == "switch":  # switch [init;] [tag] { case a, b: ... default: ... }
            self.next()
            init = tag = None
            self.nolit = True
            if self.val() != "{":
                s = self.simple()
                if self.accept(";"):
                    init = s
                    s = None if self.val() == "{" else self.simple()
                tag = s[1] if s else None
            self.nolit = False
            self.expect("{")
            clauses = []
            while not self.accept("}"):
                if self.accept(";"):
                    continue
                if self.accept("default"):
                    conds = None
                else:
                    self.expect("case")
                    conds = [self.expr()]
                    while self.accept(","):
                        conds.append(self.expr())
                self.expect(":")
                body = []
                while self.val() not in ("case", "default", "}"):
                    if self.accept(";"):
                        continue
                    body.append(self.stmt())
                clauses.append((conds, body))
            return ("switch", init, tag, clauses)
        if v == "var":
            self.next()
            name = self.next()[1]
            t = self.parse_type() if self.val() != "=" else None
            val = self.expr() if self.accept("=") else None
            return ("var", name, t, val)
        if v == "{":
            return ("block", self.block())
        s = self.simple()
        self.accept(";")
        return s


# ----------------------------------------------------------------------------- loader
class Func:
    def __init__(self, pkg, name, recv, params, toks, body_at):
        self.pkg, self.name, self.recv, self.params = pkg, name, recv, params
        self.toks, self.body_at, self.body = toks, body_at, None


class Package:
    def __init__(self, name):
        self.name = name
        self.funcs, self.methods, self.consts, self.types, self.imports = {}, {}, {}, {}, {}
        self.structs = {}  # name -> [(field, type)]
        self.vars = {}  # package-level var: name -> [type, init expr, done, value]


class Return(Exception):
    def __init__(self, vals):
        self.vals = vals


class Interp:
    """Loads Go packages from a source tree (module path prefix -> directory)."""

    def __init__(self, root, module="github.com/YaoZengzeng/yustack"):
        self.root, self.module, self.pkgs = root, module, {}
        # packages outside the loaded tree, as Python callables: "pkg.Func" -> f(*args)
        self.stubs = {"log.Printf": lambda *a: None, "log.Println": lambda *a: None}
        # functions whose locals to keep when they return (or end in a panic / Fatalf):
        # (package, name) or (package, "Outer.func") for a function literal in Outer
        self.watch, self.frames = set(), {}
        self._fn_stack = []  # names of the functions being run (a literal's owner)

    def load(self, rel_dir, files=None):
        d = os.path.join(self.root, rel_dir)
        names = files or sorted(f for f in os.listdir(d) if f.endswith(".go") and not f.endswith("_test.go"))
        pkg = None
        for f in names:
            pkg = self._load_file(os.path.join(d, f), pkg)
        self.pkgs[rel_dir.split("/")[-1]] = pkg
        return pkg

    def _load_file(self, path, pkg):
        toks = lex(open(path).read())
        p = Parser(toks)
        p.expect("package")
        name = p.next()[1]
        pkg = pkg or Package(name)
        imports = {}
        while p.peek()[0] != "eof":
            v = p.val()
            if v == ";":
                p.next()
            elif v == "import":
                p.next()
                specs = []
                if p.accept("("):
                    while not p.accept(")"):
                        if p.accept(";"):
                            continue
                        alias = p.next()[1] if p.peek()[0] == "id" else None
                        specs.append((alias, p.next()[1].strip('"')))
                else:
                    alias = p.next()[1] if p.peek()[0] == "id" else None
                    specs.append((alias, p.next()[1].strip('"')))
                for alias, path_ in specs:
                    imports[alias or path_.split("/")[-1]] = path_.split("/")[-1]
            elif v == "const":
                p.next()
                self._consts(p, pkg)
            elif v == "type":
                p.next()
                tname = p.next()[1]
                if p.val() == "[" and p.val(1) == "]":
                    p.next()
                    p.next()
                    pkg.types[tname] = "[]" + p.parse_type()
                elif p.val() == "struct":
                    p.next()
                    pkg.structs[tname] = p.struct_fields()
                elif p.val() == "interface":
                    p.next()
                    p.skip_balanced()
                else:
                    pkg.types[tname] = p.parse_type()
                    if pkg.types[tname] in WIDTH:
                        NAMED_INT[tname] = pkg.types[tname]
            elif v == "var":
                p.next()
                at = p.i
                try:
                    specs = []
                    if p.accept("("):
                        while not p.accept(")"):
                            if p.accept(";"):
                                continue
                            specs.append(self._var_spec(p))
                    else:
                        specs.append(self._var_spec(p))
                    for nm, t, e in specs:
                        pkg.vars[nm] = [t, e, False, None]
                except (SyntaxError, IndexError, KeyError, ValueError):
                    p.i = at  # not in the subset: skipped, as it is never used on the path
                    if p.val() == "(":
                        p.skip_balanced()
                    else:
                        while p.val() != ";":
                            if p.val() in "([{":
                                p.skip_balanced()
                            else:
                                p.next()
            elif v == "func":
                p.next()
                recv = None
                if p.accept("("):
                    rname = p.next()[1]
                    recv = (rname, p.parse_type().lstrip("*"))
                    p.expect(")")
                fname = p.next()[1]
                p.expect("(")
                params = p.params()
                while p.val() != "{":  # results
                    if p.val() == "(":
                        p.skip_balanced()
                    else:
                        p.next()
                fn = Func(pkg, fname, recv, params, toks, p.i)
                p.skip_balanced()
                if recv:
                    pkg.methods[(recv[1], fname)] = fn
                else:
                    pkg.funcs[fname] = fn
            else:
                raise SyntaxError(f"{path}: unexpected top-level {v!r}")
        pkg.imports.update(imports)
        return pkg

    @staticmethod
    def _var_spec(p):
        nm = p.next()[1]
        t = p.parse_type() if p.val() not in ("=", ";", ")") else None
        e = p.expr() if p.accept("=") else None
        if p.val() not in (";", ")"):
            raise SyntaxError("var spec")
        return nm, t, e

    def _var(self, pkg, n):
        slot = pkg.vars[n]
        if not slot[2]:
            t, e = slot[0], slot[1]
            v = self._eval(e, [{}], pkg) if e is not None else self._zero(t, pkg)
            slot[2], slot[3] = True, self._convert(v, t, pkg) if t else v
        return slot[3]

    def _consts(self, p, pkg):
        specs = []
        if p.accept("("):
            iota, last = 0, None
            while not p.accept(")"):
                if p.accept(";"):
                    continue
                nm = p.next()[1]
                typ = None
                if p.val() not in ("=", ";", ")"):
                    typ = p.parse_type()
                if p.accept("="):
                    e = p.expr()
                    last = (e, typ)
                else:
                    e, typ = last
                specs.append((nm, e, typ, iota))
                iota += 1
        else:
            nm = p.next()[1]
            typ = p.parse_type() if p.val() != "=" else None
            p.expect("=")
            specs.append((nm, p.expr(), typ, 0))
        for nm, e, typ, iota in specs:
            pkg.consts[nm] = (e, typ, iota)

    # ------------------------------------------------------------------ evaluation
    def call(self, pkg_name, fname, *args):
        return self._invoke(self.pkgs[pkg_name].funcs[fname], None, list(args))

    def method(self, pkg_name, recv, mname, *args):
        return self._invoke(self.pkgs[pkg_name].methods[(recv.t, mname)], recv, list(args))

    def _bind(self, params, args, scope, pkg):
        """Parameters into scope; a final ...T parameter takes the remaining
        arguments as a slice."""
        for k, (nm, t) in enumerate(params):
            if t.startswith("..."):
                v = GoList(args[k:], "[]" + t[3:])
            else:
                v = self._convert(args[k], t, pkg) if k < len(args) else self._zero(t, pkg)
            if nm is not None and nm != "_":
                scope[nm] = v

    def _run(self, body, env, pkg, key):
        sink = {} if key in self.watch else None
        try:
            self._exec_block(body, env, pkg, sink)
        except Return as r:
            return r.vals[0] if len(r.vals) == 1 else tuple(r.vals)
        finally:
            if sink is not None:
                self.frames[key] = sink
        return None

    def _invoke(self, fn, recv, args):
        if fn.body is None:
            fn.body = Parser(fn.toks, fn.body_at).block()
        env = [{}]
        if fn.recv:
            env[0][fn.recv[0]] = recv
        self._bind(fn.params, args, env[0], fn.pkg)
        self._fn_stack.append(fn.name)
        try:
            return self._run(fn.body, env, fn.pkg, (fn.pkg.name, fn.name))
        finally:
            self._fn_stack.pop()

    def _invoke_closure(self, c, args):
        env = c.env + [{}]
        self._bind(c.params, args, env[-1], c.pkg)
        return self._run(c.body, env, c.pkg, (c.pkg.name, c.owner + ".func"))

    def _exec_block(self, stmts, env, pkg, sink=None):
        env.append({})
        try:
            for s in stmts:
                self._exec(s, env, pkg)
        finally:
            if sink is not None:
                for scope in env[1:]:
                    sink.update(scope)
            env.pop()

    def _lookup(self, name, env):
        for scope in reversed(env):
            if name in scope:
                return scope
        return None

    def _exec(self, s, env, pkg):
        k = s[0]
        if k == "expr":
            self._eval(s[1], env, pkg)
        elif k == "return":
            raise Return([self._eval(e, env, pkg) for e in s[1]])
        elif k == "var":
            _, nm, t, val = s
            v = self._eval(val, env, pkg) if val is not None else self._zero(t, pkg)
            env[-1][nm] = self._convert(v, t, pkg) if t else v
        elif k == "assign":
            _, op, lhs, rhs = s
            vals = [self._eval(e, env, pkg) for e in rhs]
            if len(lhs) > 1 and len(vals) == 1 and isinstance(vals[0], tuple):  # a, b := f()
                vals = list(vals[0])
            for target, v in zip(lhs, vals):
                if op == ":=":
                    if target[1] != "_":
                        env[-1][target[1]] = v
                    continue
                if op != "=":
                    v = self._binop(op[:-1], self._eval(target, env, pkg), v)
                self._store(target, v, env, pkg)
        elif k == "if":
            _, init, cond, body, els = s
            env.append({})
            try:
                if init:
                    self._exec(init, env, pkg)
                if self._eval(cond, env, pkg):
                    self._exec_block(body, env, pkg)
                elif els:
                    self._exec_block(els, env, pkg)
            finally:
                env.pop()
        elif k == "for":
            _, init, cond, post, body = s
            env.append({})
            try:
                if init:
                    self._exec(init, env, pkg)
                while cond is None or self._eval(cond, env, pkg):
                    self._exec_block(body, env, pkg)
                    if post:
                        self._exec(post, env, pkg)
            finally:
                env.pop()
        elif k == "range":
            _, keys, define, x, body = s
            seq = self._eval(x, env, pkg)
            n = seq.len if isinstance(seq, (Slice, GoList)) else len(seq.b)
            for i in range(n):
                vals = [Int(i, "int"), seq.get(i) if not isinstance(seq, Str) else Int(seq.b[i], "uint8")]
                env.append({})
                try:
                    for key, v in zip(keys, vals):
                        if key[0] == "name" and key[1] == "_":
                            continue
                        if define:
                            env[-1][key[1]] = v
                        else:
                            self._store(key, v, env, pkg)
                    self._exec_block(body, env, pkg)
                finally:
                    env.pop()
        elif k == "block":
            self._exec_block(s[1], env, pkg)
        elif k == "switch":
            _, init, tag, clauses = s
            env.append({})
            try:
                if init:
                    self._exec(init, env, pkg)
                tv = self._eval(tag, env, pkg) if tag is not None else True
                chosen = None
                for conds, body in clauses:
                    if conds is None:
                        continue
                    for c in conds:
                        cv = self._eval(c, env, pkg)
                        if (cv is True and tag is None) or (tag is not None and self._binop("==", tv, cv)):
                            chosen = body
                            break
                    if chosen is not None:
                        break
                if chosen is None:
                    chosen = next((b for c, b in clauses if c is None), None)
                if chosen is not None:
                    self._exec_block(chosen, env, pkg)
            finally:
                env.pop()
        else:
            raise NotImplementedError(k)

    def _store(self, target, v, env, pkg):
        if target[0] == "name":
            scope = self._lookup(target[1], env)
            old = scope[target[1]]
            scope[target[1]] = self._convert(v, old.t, pkg) if isinstance(old, Int) else v
        elif target[0] == "index":
            base = self._eval(target[1], env, pkg)
            if isinstance(base, GoList) and isinstance(v, Int) and base.t.startswith("[]"):
                v = self._convert(v, base.t[2:], pkg)  # the element type's width
            base.set(self._int(self._eval(target[2], env, pkg)), v if isinstance(base, GoList) else v.v)
        elif target[0] == "sel":
            st = self._eval(target[1], env, pkg)
            if not isinstance(st, Struct):
                raise NotImplementedError(target)
            old = st.f[target[2]]
            st.f[target[2]] = self._convert(v, old.t, st.pkg) if isinstance(old, Int) else v
        elif target[0] == "un" and target[1] == "*":
            self._store(target[2], v, env, pkg)
        else:
            raise NotImplementedError(target)

    @staticmethod
    def _int(x):
        return x.v if isinstance(x, Int) else int(x)

    def _struct_def(self, t, pkg):
        """(fields, package) of struct type t (plain or pkg-qualified), or None."""
        if "." in t:
            q, n = t.split(".", 1)
            other = self.pkgs.get(pkg.imports.get(q, q))
            return (other.structs[n], other, n) if other and n in other.structs else None
        for p in [pkg] + list(self.pkgs.values()):
            if t in p.structs:
                return p.structs[t], p, t
        return None

    def _zero(self, t, pkg):
        if t is None or t.startswith("*") or t in ("map", "chan", "func"):
            return None
        if t == "bool":
            return False
        sd = self._struct_def(t, pkg)
        if sd is not None:
            fields, spkg, name = sd
            return Struct(name, spkg, {f: self._zero(ft, spkg) for f, ft in fields})
        rt = self._resolve_type(t, pkg)
        u = self._underlying(rt, pkg)
        if u in WIDTH:
            return Int(0, u)
        if u == "string":
            return Str(b"", rt)
        if u.startswith("[") and u[1] != "]":  # [N]T
            n = u[1:u.index("]")]
            if n.isdigit() and u.endswith("byte"):
                return Slice(bytearray(int(n)), 0, int(n), int(n), rt)
            return None
        return None  # nil: slices, pointers, interfaces, maps, channels, funcs

    def _resolve_type(self, t, pkg):
        if t in WIDTH or t in ("string", "bool") or t.startswith("[]"):
            return t
        if "." in t:
            q, n = t.split(".", 1)
            other = self.pkgs.get(pkg.imports.get(q, q))
            if other and n in other.types:
                return n
            return t
        return t

    def _underlying(self, t, pkg):
        for p in [pkg] + list(self.pkgs.values()):
            if t in p.types:
                return p.types[t]
        return t

    def _convert(self, v, t, pkg):
        if t is None:
            return v
        t = self._resolve_type(t, pkg)
        u = self._underlying(t, pkg)
        if u in WIDTH:
            return Int(v.v if isinstance(v, Int) else int(v), t if t in NAMED_INT else u)
        if u == "[]byte" or u == "[]uint8":
            if isinstance(v, Str):
                return from_bytes(v.b, t if t != u else "[]byte")
            if isinstance(v, Slice):
                return Slice(v.buf, v.off, v.len, v.cap, t if t != u else "[]byte")
        if u == "string":
            if isinstance(v, Slice):
                return Str(v.bytes(), t)
            if isinstance(v, Str):
                return Str(v.b, t)
        return v

    def _binop(self, op, a, b):
        if op in ("&&", "||"):
            raise NotImplementedError
        if a is None or b is None:  # x == nil / x != nil (nil slices, pointers, errors)
            if op not in ("==", "!="):
                raise GoPanic("invalid memory address or nil pointer dereference")
            return (a is b) if op == "==" else (a is not b)
        if isinstance(a, Int) and isinstance(b, Int):
            t = a.t if a.t != "untyped" else b.t
            if op in ("<<", ">>"):
                t = a.t
                r = a.v << b.v if op == "<<" else a.v >> b.v
                return Int(r, t)
            x, y = a.v, b.v
            if op == "+":
                return Int(x + y, t)
            if op == "-":
                return Int(x - y, t)
            if op == "*":
                return Int(x * y, t)
            if op == "/":
                if y == 0:
                    raise GoPanic("integer divide by zero")
                q = abs(x) // abs(y)
                return Int(q if (x >= 0) == (y >= 0) else -q, t)
            if op == "%":
                if y == 0:
                    raise GoPanic("integer divide by zero")
                r = abs(x) % abs(y)
                return Int(r if x >= 0 else -r, t)
            if op == "&":
                return Int(x & y, t)
            if op == "|":
                return Int(x | y, t)
            if op == "^":
                return Int(x ^ y, t)
            if op == "&^":
                return Int(x & ~y, t)
            return {"==": x == y, "!=": x != y, "<": x < y, "<=": x <= y, ">": x > y, ">=": x >= y}[op]
        if isinstance(a, Str) and isinstance(b, Str):
            return {"==": a.b == b.b, "!=": a.b != b.b, "+": Str(a.b + b.b, a.t)}[op]
        if isinstance(a, bool) and isinstance(b, bool):
            return {"==": a == b, "!=": a != b}[op]
        raise NotImplementedError((op, a, b))

    def _eval(self, e, env, pkg):
        k = e[0]
        if k == "lit":
            return e[1]
        if k == "name":
            n = e[1]
            scope = self._lookup(n, env)
            if scope is not None:
                return scope[n]
            if n in ("true", "false"):
                return n == "true"
            if n == "nil":
                return None
            if n in pkg.consts:
                return self._const(pkg, n)
            if n in pkg.vars:
                return self._var(pkg, n)
            raise NameError(n)
        if k == "bin":
            op = e[1]
            if op == "&&":
                return bool(self._eval(e[2], env, pkg)) and bool(self._eval(e[3], env, pkg))
            if op == "||":
                return bool(self._eval(e[2], env, pkg)) or bool(self._eval(e[3], env, pkg))
            return self._binop(op, self._eval(e[2], env, pkg), self._eval(e[3], env, pkg))
        if k == "un":
            if e[1] == "&" and e[2][0] == "index":  # &s[i]: a reference into the slice
                base = self._eval(e[2][1], env, pkg)
                if isinstance(base, (Slice, GoList)):
                    i = self._int(self._eval(e[2][2], env, pkg))
                    base.get(i)  # bounds check, as Go's
                    return Ref(base, i)
            x = self._eval(e[2], env, pkg)
            if e[1] in ("&", "*"):  # pointers: the value itself (shared, see module doc)
                return x
            if e[1] == "!":
                return not x
            if e[1] == "-":
                return Int(-x.v, x.t)
            if e[1] == "^":
                if x.t == "untyped":
                    return Int(~x.v)
                return Int(~x.v, x.t)
            return x
        if k == "index":
            return self._eval(e[1], env, pkg).get(self._int(self._eval(e[2], env, pkg)))
        if k == "slice":
            s = self._eval(e[1], env, pkg)
            lo = 0 if e[2] is None else self._int(self._eval(e[2], env, pkg))
            hi = None if e[3] is None else self._int(self._eval(e[3], env, pkg))
            if isinstance(s, Str):
                hi = len(s.b) if hi is None else hi
                if not 0 <= lo <= hi <= len(s.b):
                    raise GoPanic(f"slice bounds out of range [{lo}:{hi}] with length {len(s.b)}")
                return Str(s.b[lo:hi], s.t)
            r = s.sub(lo, hi)
            if e[4] is not None:  # 3-index slice: the capacity is cut too
                mx = self._int(self._eval(e[4], env, pkg))
                if not r.len + lo <= mx <= s.cap:
                    raise GoPanic(f"slice bounds out of range [::{mx}] with capacity {s.cap}")
                r.cap = mx - lo
            return r
        if k == "slicelit":
            vals = [self._eval(x, env, pkg) for x in e[2]]
            if e[1] in ("[]byte", "[]uint8"):
                return from_bytes(bytes(v.v & 0xFF for v in vals))
            return GoList(vals, e[1])
        if k == "funclit":
            owner = self._fn_stack[-1] if self._fn_stack else "?"
            return Closure(e[1], e[2], list(env), pkg, owner)
        if k == "complit":
            return self._complit(e, env, pkg)
        if k == "call":
            return self._call(e, env, pkg)
        if k == "sel":
            base = e[1]
            if base[0] == "name" and self._lookup(base[1], env) is None and base[1] in pkg.imports:
                other = self.pkgs.get(pkg.imports[base[1]])
                if other is not None and e[2] in other.consts:
                    return self._const(other, e[2])
                stub = self.stubs.get(f"{pkg.imports[base[1]]}.{e[2]}")
                if stub is not None and not callable(stub):  # a stub constant (C.YU_OK)
                    return stub
                raise NameError(f"{base[1]}.{e[2]}")
            st = self._eval(base, env, pkg)
            if isinstance(st, Struct):
                return st.f[e[2]]
            return getattr(st, e[2])  # a Python stub's attribute
        raise NotImplementedError(k)

    def _complit(self, e, env, pkg):
        """T{...} / pkg.T{...}: a struct (keyed or positional fields) or a named slice."""
        tx, items = e[1], e[2]
        t = tx[1] if tx[0] == "name" else f"{tx[1][1]}.{tx[2]}"
        sd = self._struct_def(t, pkg)
        if sd is None:
            rt = self._resolve_type(t, pkg)
            u = self._underlying(rt, pkg)
            vals = [self._eval(x, env, pkg) for _, x in items]
            if u in ("[]byte", "[]uint8"):
                return from_bytes(bytes(v.v & 0xFF for v in vals), rt)
            return GoList(vals, rt)
        fields, spkg, name = sd
        st = self._zero(t, pkg)
        types = dict(fields)
        for k, (key, x) in enumerate(items):
            f = key if key is not None else fields[k][0]
            st.f[f] = self._convert(self._eval(x, env, pkg), types[f], spkg)
        return st
        raise NotImplementedError(k)

    def _const(self, pkg, n):
        expr, typ, iota = pkg.consts[n]
        env = [{"iota": Int(iota)}]
        v = self._eval(expr, env, pkg)
        return self._convert(v, typ, pkg) if typ and self._underlying(self._resolve_type(typ, pkg), pkg) in WIDTH else v

    def _call(self, e, env, pkg):
        fexpr, args = e[1], e[2]
        if fexpr[0] == "name":
            n = fexpr[1]
            if self._lookup(n, env) is None:
                if n == "len":
                    x = self._eval(args[0], env, pkg)
                    if x is None:  # a nil slice
                        return Int(0, "int")
                    return Int(x.len if isinstance(x, (Slice, GoList)) else len(x.b), "int")
                if n == "cap":
                    return Int(self._eval(args[0], env, pkg).cap, "int")
                if n == "make":
                    t = args[0][1]
                    size = self._int(self._eval(args[1], env, pkg))
                    if t in ("[]byte", "[]uint8") or self._underlying(t, pkg) in ("[]byte", "[]uint8"):
                        return Slice(bytearray(size), 0, size, size, t)
                    et = t[2:]
                    return GoList([Int(0, et) if et in WIDTH else None for _ in range(size)], t)
                if n == "copy":
                    dst, src = self._eval(args[0], env, pkg), self._eval(args[1], env, pkg)
                    b = src.bytes() if isinstance(src, Slice) else src.b
                    m = min(dst.len, len(b))
                    dst.buf[dst.off:dst.off + m] = b[:m]
                    return Int(m, "int")
                if n in WIDTH or n == "string" or n.startswith("[]") or n in pkg.types:
                    return self._convert(self._eval(args[0], env, pkg), n, pkg)
                if n in pkg.funcs:
                    return self._invoke(pkg.funcs[n], None, [self._eval(a, env, pkg) for a in args])
            else:
                f = self._lookup(n, env)[n]
                if isinstance(f, Closure):
                    return self._invoke_closure(f, [self._eval(a, env, pkg) for a in args])
                if callable(f):
                    return f(*[self._eval(a, env, pkg) for a in args])
            raise NameError(n)
        if fexpr[0] == "sel":
            base, name = fexpr[1], fexpr[2]
            # encoding/binary.BigEndian (stdlib, restated)
            if base == ("sel", ("name", "binary"), "BigEndian"):
                vals = [self._eval(a, env, pkg) for a in args]
                b = vals[0]
                if name == "Uint16":
                    return Int((b.get(0).v << 8) | b.get(1).v, "uint16")
                if name == "Uint32":
                    return Int(int.from_bytes(bytes(b.get(i).v for i in range(4)), "big"), "uint32")
                if name == "PutUint16":
                    b.get(1)
                    b.set(0, vals[1].v >> 8)
                    b.set(1, vals[1].v)
                    return None
                if name == "PutUint32":
                    b.get(3)
                    for i in range(4):
                        b.set(i, vals[1].v >> (24 - 8 * i))
                    return None
                raise NotImplementedError(name)
            if base[0] == "name" and self._lookup(base[1], env) is None and base[1] in pkg.imports:
                vals = [self._eval(a, env, pkg) for a in args]
                stub = self.stubs.get(f"{pkg.imports[base[1]]}.{name}")
                if stub is not None:
                    return stub(*vals)
                other = self.pkgs[pkg.imports[base[1]]]
                if name in other.funcs:
                    return self._invoke(other.funcs[name], None, vals)
                if name in other.types:
                    return self._convert(vals[0], name, other)
                raise NameError(f"{base[1]}.{name}")
            recv = self._eval(base, env, pkg)
            vals = [self._eval(a, env, pkg) for a in args]
            if not isinstance(recv, (Int, Slice, Str, Struct, GoList)):  # a Python stub
                return getattr(recv, name)(*vals)
            if isinstance(recv, Struct) and isinstance(recv.f.get(name), Closure):  # a func-typed field
                return self._invoke_closure(recv.f[name], vals)
            home = [recv.pkg] if isinstance(recv, Struct) else []
            for p in home + [pkg] + list(self.pkgs.values()):
                fn = p.methods.get((recv.t, name))
                if fn is not None:
                    return self._invoke(fn, recv, vals)
            raise NameError(f"method {recv.t}.{name}")
        if fexpr[0] == "un" and fexpr[1] == "*" and len(args) == 1:  # (*T)(x): a pointer conversion
            return self._eval(args[0], env, pkg)
        raise NotImplementedError(fexpr)


def load_reference(root="/root/reference"):
    """The packages on the checksum path: checksum, header (ipv4, tcp, udp)."""
    it = Interp(root)
    it.load("checksum", ["checksum.go"])
    it.load("header", ["ipv4.go", "tcp.go", "udp.go"])
    return it


def load_path(root="/root/reference", checksum=None):
    """Everything from the senders to the checker: the packages above, the buffers and
    route the senders use, the senders themselves (sendUDP, sendTCP /
    sendTCPWithOptions, sendICMPv4, ipv4 endpoint.WritePacket) and checker.go. Only the
    files that hold them are read; bodies are parsed when first run.
    checksum: (directory, files) of another package checksum to load in place of the
    reference's, e.g. the cgo shim (bindings/go/checksum): every caller above then
    resolves `checksum.X` to it, unchanged (the caller supplies the shim's `C.*` stubs)."""
    it = Interp(root)
    if checksum is None:
        it.load("checksum", ["checksum.go"])
    else:
        d, files = checksum
        assert os.path.basename(os.path.normpath(d)) == "checksum"
        it.load(os.path.abspath(d), files)
    it.load("seqnum", ["seqnum.go"])
    it.load("buffer", ["view.go", "prependable.go"])
    it.load("types", ["types.go", "route.go", "transport.go", "network.go"])
    it.load("header", ["ipv4.go", "tcp.go", "udp.go", "icmpv4.go"])
    it.load("transport/udp", ["endpoint.go", "protocol.go"])
    it.load("transport/tcp", ["connect.go", "protocol.go"])
    it.load("network/ipv4", ["ipv4.go", "icmp.go"])
    it.load("checker", ["checker.go"])
    return it
