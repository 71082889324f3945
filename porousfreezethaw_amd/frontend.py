"""Params front end: the reference's parameter files, evaluated as the reference
evaluates them.

The reference reads `Params` with pparse (modules/pparser/pparser.c:35-108): every line goes
first to the command parser (modules/cparser/cparser.c; intertrack.c:975-1037 registers `set`,
`icond`, `grid`, `mnemonic`, `continue_if`, `break`, the slice_* no-ops); comment and empty lines
are skipped; any other line is `name expression`, evaluated by the Digithell expression
evaluator (libsource/exprsion/exp_all.cc + the extensions of ee_wrapper.cc:304-335) and defined
as a variable for the following lines.  The driver then reads the values it needs
(intertrack.c:1491-1575) and evaluates the `icond` formulas at every grid node
(intertrack.c:1831-2012).

This module restates that evaluator -- its tokenizer, operator table, precedences and
evaluation order (a shunting-yard whose stack is reduced while the stacked operator's
precedence number is <= the incoming one) -- so that the values are bit-identical: numbers
go through float_val (str_fval.c), functions are C's libm through Python's math module.  The
icond formulas are compiled to the postfix program the evaluator executes and run per grid node
by libpft (pft_ic_eval, host C, the reference's node coordinates and multi-pass order).
"""
import math
import os
import re

import numpy as np

from .params import float_val, to_int

# --------------------------------------------------------------------------------------------
# the expression evaluator (exp_all.cc)

VAR, UNARY, POSTFIX, BINARY, L_PAR, R_PAR, NUMBER = range(7)   # exprsion.h:155


class EvalError(ValueError):
    pass


def _power(x, y):
    # exp_all.cc:53-64 (__Power__)
    if x == 0 and y <= 0:
        raise EvalError("domain")
    if x < 0 and y != math.floor(y):
        if math.fmod(1 / y - 1, 2) != 0:
            raise EvalError("domain")
        return -math.pow(-x, y)
    try:
        return math.pow(x, y)
    except OverflowError as e:
        raise EvalError("overflow") from e


def _div(x, y):
    if y == 0:
        raise EvalError("division by zero")
    return x / y


def _dom(pred, f):
    def g(x):
        if not pred(x):
            raise EvalError("domain")
        return f(x)
    return g


def _round(x):
    r = math.floor(x)
    if x - r >= 0.5:
        r += 1
    return float(r)


def _fact(x):
    if x < 0 or x != math.floor(x):
        raise EvalError("domain")
    if x > 170:
        raise EvalError("overflow")
    r = 1.0
    while x:
        r *= x
        x -= 1
    return r


def _comb(x, y, perm):
    if x < 0 or x != math.floor(x) or y < 0 or y != math.floor(y) or x < y:
        raise EvalError("domain")
    r = 1.0
    while y:
        r *= x
        x -= 1
        if not perm:
            r /= y
        y -= 1
    return r


def _ovf(f):
    def g(x):
        try:
            return f(x)
        except OverflowError as e:
            raise EvalError("overflow") from e
    return g


# (name, kind, precedence, function, opcode for pft_ic_eval) in the registration order of
# exp_all.cc:409-446 and ee_wrapper.cc:320-334 (the order matters: the first entry of a name is
# found first, its other version second)
_OPS = [
    ("-", BINARY, 22, lambda x, y: x - y, 1), ("+", BINARY, 22, lambda x, y: x + y, 2),
    ("*", BINARY, 20, lambda x, y: x * y, 3), ("/", BINARY, 20, _div, 4),
    ("C", BINARY, 18, lambda x, y: _comb(x, y, False), 5), ("P", BINARY, 18, lambda x, y: _comb(x, y, True), 6),
    ("-", UNARY, 16, lambda x: -x, 20), ("+", UNARY, 16, lambda x: x, 21),
    ("int", UNARY, 16, lambda x: float(math.floor(x)) if x > 0 else float(math.ceil(x)), 22),
    ("floor", UNARY, 16, lambda x: float(math.floor(x)), 23), ("ceil", UNARY, 16, lambda x: float(math.ceil(x)), 24),
    ("round", UNARY, 16, _round, 25), ("abs", UNARY, 16, math.fabs, 26),
    ("sin", UNARY, 16, _dom(lambda x: abs(x) <= 1e12, math.sin), 27),
    ("cos", UNARY, 16, _dom(lambda x: abs(x) <= 1e12, math.cos), 28),
    ("tan", UNARY, 16, _dom(lambda x: abs(x) <= 1e12 and math.cos(x) != 0, math.tan), 29),
    ("asin", UNARY, 16, _dom(lambda x: abs(x) <= 1, math.asin), 30),
    ("acos", UNARY, 16, _dom(lambda x: abs(x) <= 1, math.acos), 31),
    ("atan", UNARY, 16, math.atan, 32),
    ("sinh", UNARY, 16, _ovf(math.sinh), 33), ("cosh", UNARY, 16, _ovf(math.cosh), 34),
    ("tanh", UNARY, 16, math.tanh, 35),
    ("asinh", UNARY, 16, _ovf(lambda x: math.log(x + math.sqrt(math.pow(x, 2) + 1))), 36),
    ("acosh", UNARY, 16, _dom(lambda x: x >= 1, _ovf(lambda x: math.log(x + math.sqrt(math.pow(x, 2) - 1)))), 37),
    ("atanh", UNARY, 16, _dom(lambda x: abs(x) < 1, lambda x: math.log((1 + x) / (1 - x)) / 2), 38),
    ("log", UNARY, 16, _dom(lambda x: x > 0, math.log10), 39), ("ln", UNARY, 16, _dom(lambda x: x > 0, math.log), 40),
    ("sqrt", UNARY, 16, _dom(lambda x: x >= 0, math.sqrt), 41), ("exp", UNARY, 16, _ovf(math.exp), 42),
    ("pow10", UNARY, 16, _dom(lambda x: x <= 308, lambda x: math.pow(10, x)), 43),
    ("^", BINARY, 14, _power, 7), ("root", BINARY, 14, lambda x, y: _power(y, 1 / x) if x != 0 else _power(0, -1), 8),
    ("!", POSTFIX, 12, _fact, 44),
    ("toDeg", UNARY, 10, lambda x: x / math.pi * 180, 45), ("toRad", UNARY, 10, lambda x: x / 180 * math.pi, 46),
    # ee_wrapper.cc extensions
    ("sgn", UNARY, 16, lambda x: 1.0 if x > 0 else (-1.0 if x < 0 else 0.0), 47),
    ("max", BINARY, 16, lambda x, y: x if x > y else y, 9), ("min", BINARY, 16, lambda x, y: x if x < y else y, 10),
    ("<", BINARY, 24, lambda x, y: 1.0 if x < y else 0.0, 11), (">", BINARY, 24, lambda x, y: 1.0 if x > y else 0.0, 12),
    ("=", BINARY, 24, lambda x, y: 1.0 if x == y else 0.0, 13),
    ("and", BINARY, 26, lambda x, y: 1.0 if (x != 0 and y != 0) else 0.0, 14),
    ("or", BINARY, 26, lambda x, y: 1.0 if (x != 0 or y != 0) else 0.0, 15),
    ("not", UNARY, 25, lambda x: 0.0 if x != 0 else 1.0, 48),
]
# the opcode numbering is the ABI of pft_ic_eval (include/pft_frontend.h)
OP_PUSH_CONST, OP_PUSH_VAR = 100, 101


def _is_digit(c):
    return ("0" <= c <= "9") or c == "."


def _is_alpha(c):
    c = c.upper()
    return ("A" <= c <= "Z") or c == "_"


def _is_special(c):
    return not (_is_digit(c) or _is_alpha(c) or c == " " or c in "()")


def _is_identifier(s):
    if len(s) == 1 and _is_special(s):
        return True
    if not s or not _is_alpha(s[0]):
        return False
    return all(_is_alpha(c) or _is_digit(c) for c in s[1:])


class Evaluator:
    """exp_all.cc EXPRESSION with the ee_wrapper.cc extensions installed (the shared instance
    intertrack.c:1287 uses).  Variables: pi, e, then whatever is defined."""

    def __init__(self):
        self.ident = []                                     # [name, kind, prec, f|value, opcode]
        for name, kind, prec, f, code in _OPS:
            self.ident.append([name, kind, prec, f, code])
        self.ident.insert(0, ["e", VAR, 0, math.e, None])
        self.ident.insert(0, ["pi", VAR, 0, math.pi, None])

    # -- symbol table (exp_all.cc:265-340) ------------------------------------------------
    def _defined(self, s, start=0):
        if len(s) > 32 or not _is_identifier(s):
            return -2
        for q in range(start, len(self.ident)):
            if self.ident[q][0] == s:
                return q
        return -1

    def _var(self, s):
        q = self._defined(s)
        return self.ident[q] if q >= 0 and self.ident[q][1] == VAR else None

    def _unary(self, s):
        q = self._defined(s)
        if q < 0:
            return None
        if self.ident[q][1] in (UNARY, POSTFIX):
            return self.ident[q]
        if self.ident[q][1] != BINARY:
            return None
        q = self._defined(s, q + 1)
        return self.ident[q] if q >= 0 else None

    def _binary(self, s):
        q = self._defined(s)
        if q < 0:
            return None
        if self.ident[q][1] == BINARY:
            return self.ident[q]
        if self.ident[q][1] not in (UNARY, POSTFIX):
            return None
        q = self._defined(s, q + 1)
        return self.ident[q] if q >= 0 else None

    def define(self, name, value):
        """ev_def_var (exp_all.cc:500-530): define or redefine a variable"""
        if not _is_identifier(name):
            raise EvalError(f"invalid identifier {name!r}")
        q = self._defined(name)
        if q >= 0:
            if self.ident[q][1] != VAR:
                raise EvalError(f"{name!r} is an operator")
            self.ident[q][3] = float(value)
        else:
            self.ident.append([name, VAR, 0, float(value), None])

    def value(self, name):
        v = self._var(name)
        if v is None:
            raise EvalError(f"undefined variable {name!r}")
        return v[3]

    # -- lexical analysis (exp_all.cc:660-777) ----------------------------------------------
    def parse(self, expr):
        out = []
        loc, n = 0, len(expr)
        last = BINARY
        parenths = 0
        while loc < n:
            buf, q = "", 0
            while True:
                if loc >= n:
                    break
                c = expr[loc]
                loc += 1
                if c == " ":
                    break
                if _is_special(c) or c in "()":
                    if q == 0:
                        buf += c
                        q += 1
                        break
                    if not _is_identifier(buf) and buf[q - 1].lower() == "e" and c in "+-":
                        buf += c
                    else:
                        loc -= 1
                        break
                if _is_alpha(c) or _is_digit(c):
                    buf += c
                q += 1
                if q > 32:
                    raise EvalError("syntax: element too long")
            if not buf:
                if loc >= n:
                    break
                continue
            if _is_identifier(buf):
                if self._defined(buf) < 0:
                    raise EvalError(f"syntax: undefined symbol {buf!r}")
                i = self._binary(buf)
                kind = None
                if i is not None:
                    if last in (L_PAR, BINARY, UNARY):
                        i = self._unary(buf)
                        if i is None:
                            raise EvalError(f"syntax at {buf!r}")
                    else:
                        kind = BINARY
                elif (i := self._unary(buf)) is None:
                    i = self._var(buf)
                    if last in (POSTFIX, NUMBER, R_PAR, VAR):
                        raise EvalError(f"syntax at {buf!r}")
                    kind = VAR
                if kind is None:                              # the unary/postfix path
                    if i[2] < 0 or i[1] == POSTFIX:
                        if last in (L_PAR, BINARY, UNARY):
                            raise EvalError(f"syntax at {buf!r}")
                        kind = POSTFIX
                    else:
                        if last in (POSTFIX, NUMBER, R_PAR, VAR):
                            raise EvalError(f"syntax at {buf!r}")
                        kind = UNARY
                last = kind
                out.append((kind, i))
            elif buf == "(":
                if last in (POSTFIX, NUMBER, R_PAR, VAR):
                    raise EvalError("syntax at '('")
                parenths += 1
                last = L_PAR
                out.append((L_PAR, None))
            elif buf == ")":
                if last in (BINARY, UNARY, L_PAR):
                    raise EvalError("syntax at ')'")
                parenths -= 1
                if parenths < 0:
                    raise EvalError("syntax: unbalanced ')'")
                last = R_PAR
                out.append((R_PAR, None))
            else:
                if last in (POSTFIX, NUMBER, R_PAR, VAR):
                    raise EvalError(f"syntax at {buf!r}")
                last = NUMBER
                out.append((NUMBER, float_val(buf)))
        if last in (UNARY, BINARY, L_PAR):
            raise EvalError("syntax: incomplete expression")
        return out

    # -- evaluation (exp_all.cc:229-256, 779-859), optionally emitting the postfix program ----
    def run(self, tokens, emit=None, symbolic=()):
        """evaluate parsed tokens; `emit` (a list) receives the postfix program; variables named
        in `symbolic` are program inputs (their current value is used for the evaluation)"""
        vst, ost = [], []

        def apply(op):
            if op[0] == UNARY:
                vst[-1] = op[1][3](vst[-1])
            else:
                y = vst.pop()
                vst[-1] = op[1][3](vst[-1], y)
            if emit is not None:
                emit.append((op[1][4], 0.0))

        def reduce(prec):
            while ost:
                op = ost[-1]
                if op[0] != L_PAR and op[1][2] > prec:
                    break
                if op[0] == L_PAR and prec < 32:
                    break
                ost.pop()
                if op[0] == L_PAR and prec == 32:
                    break
                if op[0] in (UNARY, BINARY):
                    apply(op)

        for kind, x in tokens:
            if kind == BINARY:
                reduce(x[2])
                ost.append((BINARY, x))
            elif kind == POSTFIX:
                reduce(-x[2] if x[2] < 0 else x[2])
                vst[-1] = x[3](vst[-1])
                if emit is not None:
                    emit.append((x[4], 0.0))
            elif kind == UNARY:
                ost.append((UNARY, x))
            elif kind == VAR:
                vst.append(x[3])
                if emit is not None:
                    emit.append((OP_PUSH_VAR, float(symbolic.index(x[0]))) if x[0] in symbolic
                                else (OP_PUSH_CONST, x[3]))
            elif kind == L_PAR:
                ost.append((L_PAR, None))
            elif kind == R_PAR:
                reduce(32)
            else:
                vst.append(x)
                if emit is not None:
                    emit.append((OP_PUSH_CONST, x))
        reduce(33)
        return vst[0]

    def eval(self, expr):
        return self.run(self.parse(expr))

    def compile(self, expr, inputs):
        """postfix program of `expr` with `inputs` as per-node variables (their values must be
        defined, any value); constants folded to their current values"""
        prog = []
        self.run(self.parse(expr), emit=prog, symbolic=tuple(inputs))
        return prog


# --------------------------------------------------------------------------------------------
# the parameter file (pparser.c + the intertrack command set)

_COMMANDS = ("set", "icond", "grid", "mnemonic", "continue_if", "break", "slice_output", "slice_along",
             "slice_reverse_order")


def _cp_options(rest):
    """cparser.c option syntax: `opt[=value] ...`, value up to the next whitespace or quoted
    ("..." with \\" escapes); everything after # is a comment"""
    opts, i, n = [], 0, len(rest)
    while i < n:
        while i < n and rest[i] in " \t\n\r":
            i += 1
        if i >= n or rest[i] == "#":
            break
        j = i
        while j < n and rest[j] not in " \t\n\r=#":
            j += 1
        name = rest[i:j]
        i = j
        while i < n and rest[i] in " \t":
            i += 1
        value = None
        if i < n and rest[i] == "=":
            i += 1
            while i < n and rest[i] in " \t":
                i += 1
            value = ""
            while i < n and rest[i] not in " \t\n\r":
                if rest[i] == '"':
                    i += 1
                    while i < n and rest[i] != '"':
                        if rest[i] == "\\" and i + 1 < n and rest[i + 1] == '"':
                            i += 1
                        value += rest[i]
                        i += 1
                    i += 1
                elif rest[i] == "#":
                    break
                else:
                    value += rest[i]
                    i += 1
        opts.append((name, value))
    return opts


def _substitute(s, env):
    """evsubst: $NAME / ${NAME} from the environment"""
    return re.sub(r"\$\{(\w+)\}|\$(\w+)", lambda m: env.get(m.group(1) or m.group(2), ""), s)


class Case:
    """One parameter file evaluated the way intertrack.c reads it."""

    def __init__(self, ev, icond, settings, order):
        self.ev = ev
        self.icond = icond            # {"u": formula, ...}
        self.settings = settings      # `set` options (after $VAR substitution)
        self.defined = order          # variable names in definition order
        g = ev.value
        self.L = (g("L1"), g("L2"), g("L3"))                              # intertrack.c:1491-1497
        from . import PARAM_NAMES
        self.params = np.array([g(n) for n in PARAM_NAMES])                # :1502-1516
        self.calc_mode = to_int(self._d("calc_mode", 0))                   # :1523
        self.n = (to_int(self._d("n1", 0)), to_int(self._d("n2", 0)), to_int(self._d("n3", 0)))  # :1528-1542
        self.saved_files = to_int(g("saved_files"))                        # :1562
        self.tau, self.final_time, self.delta = g("tau"), g("final_time"), g("delta")   # :1565-1571
        self.tau_min = self._d("tau_min", 0.0)                             # :1574

    def _d(self, name, default):
        try:
            return self.ev.value(name)
        except EvalError:
            return default

    def values(self):
        return {n: self.ev.value(n) for n in self.defined}

    def simulation(self, nprocs=1, rank=0, beads=None, **kw):
        """the slab `rank` of this case, set up as intertrack.c does: grid, parameters, the
        icond formulas evaluated at every node, glass beads (`beads`: the unit-cube centres of
        data/spheres_positions.txt), t = 0, h = tau, h_min = tau_min, delta"""
        from . import Simulation
        return Simulation(*self.n, self.L, self.calc_mode, self.params, nprocs=nprocs, rank=rank, beads=beads,
                          icond=self.icond_programs(), tau=self.tau, tau_min=self.tau_min, delta=self.delta, **kw)

    def icond_programs(self):
        """postfix programs of the icond formulas in the multi-pass order of intertrack.c:1935-2006:
        [(variable index, program)], inputs x, y, z, _x, _y, _z, u, p, gl"""
        inputs = ("x", "y", "z", "_x", "_y", "_z", "u", "p", "gl")
        ev = self.ev
        for v in ("x", "y", "z", "_x", "_y", "_z"):
            ev.define(v, 0.5)
        names = ("u", "p", "gl")
        done, out = [False] * 3, []
        while not all(done):
            progress = False
            for q in range(3):
                if done[q]:
                    continue
                if names[q] not in self.icond:
                    raise EvalError(f"no icond formula for {names[q]}")
                try:
                    prog = ev.compile(self.icond[names[q]], inputs)
                except EvalError:
                    continue                    # refers to a quantity not yet defined: next pass
                out.append((q, prog))
                done[q] = progress = True
            for q in range(3):                  # completed quantities become variables (:1994-1998)
                if done[q]:
                    ev.define(names[q], 0.0)
            if not progress:
                raise EvalError("icond formulas cannot be evaluated (undefined symbols)")
        return out


def load_params(path=None, text=None, env=None, overrides=None):
    """Evaluate a parameter file (pparser.c:35-108 with intertrack.c's handler).  `overrides`
    replaces a variable's value right after its defining line (e.g. {"grid_nodes": 400})."""
    if text is None:
        with open(path) as f:
            text = f.read()
    env = dict(os.environ if env is None else env)
    overrides = dict(overrides or {})
    ev = Evaluator()
    icond, settings, order = {}, {}, []
    for lineno, line in enumerate(text.splitlines(True), 1):
        s = line.lstrip(" \t\n")
        cmd = re.match(r"[^ \t\n=#]*", s).group(0)
        if s[len(cmd):len(cmd) + 1] == "=":     # cparser.c:67-69: a command never contains '='
            raise EvalError(f"line {lineno}: invalid command")
        if cmd == "":                           # empty line or comment (cparser.c:76)
            continue
        if cmd in _COMMANDS:
            opts = _cp_options(s[len(cmd):])
            if cmd == "icond":
                for name, val in opts:
                    icond[name] = val
            elif cmd == "set":
                for name, val in opts:
                    settings[name] = _substitute(val, env) if val is not None else True
            elif cmd == "break":
                break
            continue
        m = re.match(r"\s*(\S+)\s+([^\n]*)", line)              # sscanf("%s %[^\n]")
        if not m:
            raise EvalError(f"line {lineno}: invalid line format")
        name, expr = m.group(1), m.group(2).rstrip("\r")
        try:
            val = ev.eval(expr)
        except EvalError as e:
            raise EvalError(f"line {lineno} ({name}): {e}") from None
        if name in overrides:
            val = float(overrides[name])
        ev.define(name, val)
        if name not in order:
            order.append(name)
    return Case(ev, icond, settings, order)
