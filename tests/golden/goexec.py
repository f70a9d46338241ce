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
  `return`, package-qualified calls across the loaded packages, and
  `encoding/binary.BigEndian` (stdlib, restated).

Function bodies are parsed lazily, when first called, so code the path does not reach
(struct types, options parsing, ...) is only skipped over. tests/golden/make_golden.py
uses it to produce known-answer vectors "from the reference itself" for the functions
on the path (checksum/checksum.go, header/{ipv4,tcp,udp}.go), pinning the C oracle.
"""
from __future__ import annotations

import os
import re

WIDTH = {"uint8": 8, "byte": 8, "uint16": 16, "uint32": 32, "uint64": 64, "uint": 64,
         "int8": 8, "int16": 16, "int32": 32, "int64": 64, "int": 64}
SIGNED = {"int8", "int16", "int32", "int64", "int"}


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

    # --- types (only what the path needs: names, []T, qualified names)
    def parse_type(self):
        if self.accept("["):
            self.expect("]")
            return "[]" + self.parse_type()
        if self.accept("*"):
            return "*" + self.parse_type()
        name = self.next()[1]
        if self.val() == "." and self.peek(1)[0] == "id":
            self.next()
            name = name + "." + self.next()[1]
        return name

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
        if self.peek()[0] == "op" and v in ("-", "+", "!", "^"):
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
        elif kind == "id":
            x = ("name", v)
        else:
            raise SyntaxError(f"unexpected {v!r}")
        while True:
            v = self.val()
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
                    hi = None if self.val() == "]" else self.expr()
                    self.expect("]")
                    x = ("slice", x, lo, hi)
                else:
                    self.expect("]")
                    x = ("index", x, lo)
            else:
                return x

    # --- statements
    def block(self):
        self.expect("{")
        out = []
        while not self.accept("}"):
            if self.accept(";"):
                continue
            out.append(self.stmt())
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
            s = self.simple()
            if self.accept(";"):
                init, s = s, self.simple()
            body = self.block()
            els = None
            if self.accept("else"):
                els = [self.stmt()] if self.val() == "if" else self.block()
            return ("if", init, s[1], body, els)
        if v == "for":
            self.next()
            init = cond = post = None
            if self.val() != "{":
                s = self.simple()
                if self.accept(";"):
                    init = s
                    cond = None if self.val() == ";" else self.simple()[1]
                    self.expect(";")
                    post = None if self.val() == "{" else self.simple()
                else:
                    cond = s[1]
            return ("for", init, cond, post, self.block())
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


class Return(Exception):
    def __init__(self, vals):
        self.vals = vals


class Interp:
    """Loads Go packages from a source tree (module path prefix -> directory)."""

    def __init__(self, root, module="github.com/YaoZengzeng/yustack"):
        self.root, self.module, self.pkgs = root, module, {}

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
                elif p.val() in ("struct", "interface"):
                    p.next()
                    p.skip_balanced()
                else:
                    pkg.types[tname] = p.parse_type()
            elif v == "var":
                p.next()
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
                params, pending = [], []
                while not p.accept(")"):
                    nm = p.next()[1]
                    if p.val() in (",", ")"):
                        pending.append(nm)
                        p.accept(",")
                        continue
                    t = p.parse_type()
                    for q in pending + [nm]:
                        params.append((q, t))
                    pending = []
                    p.accept(",")
                for q in pending:  # unnamed params: types only
                    params.append((None, q))
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

    def _invoke(self, fn, recv, args):
        if fn.body is None:
            fn.body = Parser(fn.toks, fn.body_at).block()
        env = [{}]
        if fn.recv:
            env[0][fn.recv[0]] = recv
        for (nm, t), a in zip(fn.params, args):
            if nm is not None:
                env[0][nm] = self._convert(a, t, fn.pkg)
        try:
            self._exec_block(fn.body, env, fn.pkg)
        except Return as r:
            return r.vals[0] if len(r.vals) == 1 else tuple(r.vals)
        return None

    def _exec_block(self, stmts, env, pkg):
        env.append({})
        try:
            for s in stmts:
                self._exec(s, env, pkg)
        finally:
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
            for target, v in zip(lhs, vals):
                if op == ":=":
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
        elif k == "block":
            self._exec_block(s[1], env, pkg)
        else:
            raise NotImplementedError(k)

    def _store(self, target, v, env, pkg):
        if target[0] == "name":
            scope = self._lookup(target[1], env)
            old = scope[target[1]]
            scope[target[1]] = self._convert(v, old.t, pkg) if isinstance(old, Int) else v
        elif target[0] == "index":
            self._eval(target[1], env, pkg).set(self._int(self._eval(target[2], env, pkg)), v.v)
        else:
            raise NotImplementedError(target)

    @staticmethod
    def _int(x):
        return x.v if isinstance(x, Int) else int(x)

    def _zero(self, t, pkg):
        return Int(0, t) if t in WIDTH else None

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
            return Int(v.v if isinstance(v, Int) else int(v), u)
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
            if n in pkg.consts:
                return self._const(pkg, n)
            raise NameError(n)
        if k == "bin":
            op = e[1]
            if op == "&&":
                return bool(self._eval(e[2], env, pkg)) and bool(self._eval(e[3], env, pkg))
            if op == "||":
                return bool(self._eval(e[2], env, pkg)) or bool(self._eval(e[3], env, pkg))
            return self._binop(op, self._eval(e[2], env, pkg), self._eval(e[3], env, pkg))
        if k == "un":
            x = self._eval(e[2], env, pkg)
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
                return Str(s.b[lo:hi], s.t)
            return s.sub(lo, hi)
        if k == "slicelit":
            vals = [self._eval(x, env, pkg) for x in e[2]]
            return from_bytes(bytes(v.v & 0xFF for v in vals))
        if k == "call":
            return self._call(e, env, pkg)
        if k == "sel":
            base = e[1]
            if base[0] == "name" and self._lookup(base[1], env) is None and base[1] in pkg.imports:
                other = self.pkgs.get(pkg.imports[base[1]])
                if other is not None and e[2] in other.consts:
                    return self._const(other, e[2])
            raise NotImplementedError(e)
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
                    return Int(x.len if isinstance(x, Slice) else len(x.b), "int")
                if n == "make":
                    t = args[0][1]
                    size = self._int(self._eval(args[1], env, pkg))
                    return Slice(bytearray(size), 0, size, size, t)
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
                other = self.pkgs[pkg.imports[base[1]]]
                vals = [self._eval(a, env, pkg) for a in args]
                if name in other.funcs:
                    return self._invoke(other.funcs[name], None, vals)
                if name in other.types:
                    return self._convert(vals[0], name, other)
                raise NameError(f"{base[1]}.{name}")
            recv = self._eval(base, env, pkg)
            for p in [pkg] + list(self.pkgs.values()):
                fn = p.methods.get((recv.t, name))
                if fn is not None:
                    return self._invoke(fn, recv, [self._eval(a, env, pkg) for a in args])
            raise NameError(f"method {recv.t}.{name}")
        raise NotImplementedError(fexpr)


def load_reference(root="/root/reference"):
    """The packages on the checksum path: checksum, header (ipv4, tcp, udp)."""
    it = Interp(root)
    it.load("checksum", ["checksum.go"])
    it.load("header", ["ipv4.go", "tcp.go", "udp.go"])
    return it
