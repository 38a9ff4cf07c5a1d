"""SiddhiQL subset parser: app text -> AST.

Covers what the pattern/sequence hot path needs: `define stream`,
`partition with (attr of S, ...) begin ... end`, pattern (`->`, `every`, `and`/`or`,
`<m:n>`, `not ... for T`, `within T`) and sequence (`,`, `*`, `?`, `+`) inputs, filters,
`select` lists and `insert into`.  Grammar reference:
/root/reference/modules/siddhi-query-compiler/src/main/antlr4/io/siddhi/query/compiler/SiddhiQL.g4
(partition :155-174, query :176-178, pattern :200-289, sequence :291-340, math_operation :456-471
for operator precedence, literals :717-740, time units :838-845).  The AST shapes follow the
visitor (SiddhiQLBaseVisitorImpl.java:783-886): `a -> b -> c` is left-associative NEXT,
`every x` binds one pattern source, `every (chain)` a parenthesised chain.
"""
from __future__ import annotations

import re
from dataclasses import dataclass, field
from typing import List, Optional, Tuple, Union


class SiddhiParserException(Exception):
    """Raised for text outside the supported SiddhiQL subset (mirrors SiddhiParserException)."""


# ----------------------------------------------------------------------------------------------
# AST
# ----------------------------------------------------------------------------------------------

TYPE_NAMES = {"string": "STRING", "int": "INT", "long": "LONG", "float": "FLOAT",
              "double": "DOUBLE", "bool": "BOOL", "object": "OBJECT"}


@dataclass
class Annotation:
    name: str                      # e.g. "info", "app:playback"
    elements: List[Tuple[Optional[str], str]] = field(default_factory=list)

    def get(self, key, default=None):
        for k, v in self.elements:
            if k is not None and k.lower() == key.lower():
                return v
        return default


@dataclass
class StreamDef:
    name: str
    attrs: List[Tuple[str, str]]   # (name, TYPE)
    annotations: List[Annotation] = field(default_factory=list)

    def attr_index(self, name):
        for i, (a, _) in enumerate(self.attrs):
            if a == name:
                return i
        return -1


# expressions -----------------------------------------------------------------------------------
@dataclass
class Const:
    type: str                      # INT LONG FLOAT DOUBLE BOOL STRING (None value = null)
    value: object


@dataclass
class Var:
    attr: str
    stream: Optional[str] = None   # e1 / Stream1 / None
    index: Optional[int] = None    # k >= 0, or LAST (-2), LAST-1 (-3) ... as in Variable.streamIndex


LAST = -2


@dataclass
class BinOp:
    op: str                        # + - * / % == != > >= < <= and or
    left: object
    right: object


@dataclass
class Not:
    expr: object


@dataclass
class IsNull:
    expr: object                   # Var / Func


@dataclass
class IsNullStream:
    stream: str
    index: Optional[int] = None


@dataclass
class Func:
    namespace: Optional[str]
    name: str
    args: list


# state elements ---------------------------------------------------------------------------------
@dataclass
class EStream:
    stream: str
    ref: Optional[str] = None
    filters: list = field(default_factory=list)
    absent: bool = False
    for_ms: Optional[int] = None


@dataclass
class ENext:
    current: object
    next: object


@dataclass
class EEvery:
    child: object


@dataclass
class ELogical:
    type: str                      # AND / OR
    e1: object
    e2: object


@dataclass
class ECount:
    child: EStream
    min: int                       # -1 = ANY
    max: int                       # -1 = ANY


@dataclass
class StateInput:
    kind: str                      # PATTERN / SEQUENCE
    element: object
    within_ms: Optional[int] = None


@dataclass
class StandardInput:
    stream: str
    filters: list = field(default_factory=list)


@dataclass
class OutputAttr:
    expr: object
    rename: Optional[str]


@dataclass
class Query:
    input: Union[StateInput, StandardInput]
    select: Optional[List[OutputAttr]]          # None = select *
    output_stream: Optional[str]
    output_event_type: str = "CURRENT"
    annotations: List[Annotation] = field(default_factory=list)
    group_by: list = field(default_factory=list)
    having: object = None
    partition: Optional["Partition"] = None

    @property
    def name(self):
        for a in self.annotations:
            if a.name.lower() == "info":
                n = a.get("name")
                if n is not None:
                    return n
        return None


@dataclass
class Partition:
    keys: List[Tuple[str, str]]              # (attr, stream)
    queries: List[Query] = field(default_factory=list)
    annotations: List[Annotation] = field(default_factory=list)


@dataclass
class App:
    annotations: List[Annotation]
    streams: dict
    queries: List[Query]
    partitions: List[Partition]


# ----------------------------------------------------------------------------------------------
# Lexer
# ----------------------------------------------------------------------------------------------

_TOKEN_RE = re.compile(r"""
    (?P<ws>\s+|--[^\n]*|/\*.*?\*/)
  | (?P<str>'[^']*'|"[^"]*")
  | (?P<num>(?:\d+(?:\.\d*)?|\.\d+)(?:[eE][-+]?\d+)?[fFdDlL]?)
  | (?P<id>`[A-Za-z_][A-Za-z0-9_]*`|[A-Za-z_][A-Za-z0-9_]*)
  | (?P<op>->|==|!=|>=|<=|\.\.\.|[-+*/%<>=(),;\[\]:.@#!?{}])
""", re.X | re.S)

_TIME_UNITS = [
    (re.compile(r"^years?$", re.I), 365 * 24 * 3600 * 1000),
    (re.compile(r"^months?$", re.I), 30 * 24 * 3600 * 1000),
    (re.compile(r"^weeks?$", re.I), 7 * 24 * 3600 * 1000),
    (re.compile(r"^days?$", re.I), 24 * 3600 * 1000),
    (re.compile(r"^hours?$", re.I), 3600 * 1000),
    (re.compile(r"^min(utes?)?$", re.I), 60 * 1000),
    (re.compile(r"^sec(onds?)?$", re.I), 1000),
    (re.compile(r"^millisec(onds?)?$", re.I), 1),
]


def _time_unit(word):
    for rx, mult in _TIME_UNITS:
        if rx.match(word):
            return mult
    return None


@dataclass
class Tok:
    kind: str
    text: str
    pos: int


def tokenize(text):
    toks = []
    i = 0
    while i < len(text):
        m = _TOKEN_RE.match(text, i)
        if not m:
            raise SiddhiParserException(f"unexpected character {text[i]!r} at {i}")
        i = m.end()
        kind = m.lastgroup
        if kind == "ws":
            continue
        t = m.group(kind)
        if kind == "id" and t.startswith("`"):
            t = t[1:-1]
        toks.append(Tok(kind, t, m.start()))
    toks.append(Tok("eof", "", len(text)))
    return toks


# ----------------------------------------------------------------------------------------------
# Parser
# ----------------------------------------------------------------------------------------------

class Parser:
    def __init__(self, text):
        self.text = text
        self.toks = tokenize(text)
        self.i = 0

    # helpers
    def peek(self, k=0):
        return self.toks[min(self.i + k, len(self.toks) - 1)]

    def at(self, text, k=0):
        t = self.peek(k)
        if t.kind in ("id",):
            return t.text.lower() == text.lower()
        return t.kind == "op" and t.text == text

    def take(self):
        t = self.toks[self.i]
        self.i += 1
        return t

    def expect(self, text):
        t = self.take()
        ok = (t.text.lower() == text.lower()) if t.kind == "id" else (t.kind == "op" and t.text == text)
        if not ok:
            raise SiddhiParserException(f"expected {text!r} but found {t.text!r} at {t.pos}: "
                                        f"...{self.text[max(0, t.pos - 40):t.pos + 40]}...")
        return t

    def accept(self, text):
        if self.at(text):
            return self.take()
        return None

    def name(self):
        t = self.take()
        if t.kind != "id":
            raise SiddhiParserException(f"expected a name but found {t.text!r} at {t.pos}")
        return t.text

    # app ----------------------------------------------------------------------------------------
    def parse_app(self):
        app_annotations = []
        streams = {}
        queries = []
        partitions = []
        pending = []
        while self.peek().kind != "eof":
            if self.accept(";"):
                continue
            if self.at("@"):
                ann = self.annotation()
                if ann.name.lower().startswith("app:"):
                    app_annotations.append(ann)
                else:
                    pending.append(ann)
                continue
            if self.at("define"):
                d = self.definition(pending)
                pending = []
                if d is not None:
                    streams[d.name] = d
                continue
            if self.at("partition"):
                p = self.partition(pending)
                pending = []
                partitions.append(p)
                for q in p.queries:
                    q.partition = p
                    queries.append(q)
                continue
            if self.at("from"):
                queries.append(self.query(pending))
                pending = []
                continue
            t = self.peek()
            raise SiddhiParserException(f"unsupported statement starting at {t.text!r} ({t.pos})")
        return App(app_annotations, streams, queries, partitions)

    def annotation(self):
        self.expect("@")
        nm = self.name()
        while self.accept(":"):
            nm += ":" + self.name()
        elems = []
        if self.accept("("):
            while not self.at(")"):
                if self.peek().kind == "str":
                    elems.append((None, self.take().text[1:-1]))
                else:
                    key = self.name()
                    while self.at(".") or self.at(":") or self.at("-"):
                        key += self.take().text + self.name()
                    if self.accept("="):
                        v = self.take()
                        elems.append((key, v.text[1:-1] if v.kind == "str" else v.text))
                    else:
                        elems.append((None, key))
                if not self.accept(","):
                    break
            self.expect(")")
        return Annotation(nm, elems)

    def definition(self, annotations):
        self.expect("define")
        kind = self.name().lower()
        if kind != "stream":
            raise SiddhiParserException(f"'define {kind}' is outside the pattern path (only streams)")
        nm = self.name()
        self.expect("(")
        attrs = []
        while True:
            an = self.name()
            ty = self.name().lower()
            if ty not in TYPE_NAMES:
                raise SiddhiParserException(f"unknown attribute type {ty}")
            attrs.append((an, TYPE_NAMES[ty]))
            if not self.accept(","):
                break
        self.expect(")")
        return StreamDef(nm, attrs, annotations)

    def partition(self, annotations):
        self.expect("partition")
        self.expect("with")
        self.expect("(")
        keys = []
        while True:
            # partition_with_stream: attribute OF stream_id   (range partitions are out of scope)
            attr = self.name()
            if not self.at("of"):
                raise SiddhiParserException("range partitions (`expr as 'label' or ...`) are not supported")
            self.expect("of")
            keys.append((attr, self.name()))
            if not self.accept(","):
                break
        self.expect(")")
        self.expect("begin")
        qs = []
        pending = []
        while not self.at("end"):
            if self.accept(";"):
                continue
            if self.at("@"):
                pending.append(self.annotation())
                continue
            qs.append(self.query(pending))
            pending = []
        self.expect("end")
        return Partition(keys, qs, annotations)

    # query --------------------------------------------------------------------------------------
    def query(self, annotations):
        self.expect("from")
        inp = self.query_input()
        select = None
        group_by = []
        having = None
        if self.accept("select"):
            if self.accept("*"):
                select = None
            else:
                select = []
                while True:
                    e = self.expr()
                    rename = None
                    if self.accept("as"):
                        rename = self.name()
                    select.append(OutputAttr(e, rename))
                    if not self.accept(","):
                        break
            if self.at("group"):
                self.expect("group")
                self.expect("by")
                while True:
                    group_by.append(self.expr())
                    if not self.accept(","):
                        break
            if self.accept("having"):
                having = self.expr()
        if self.at("output"):
            raise SiddhiParserException("output rate limiting is outside the pattern path")
        out = None
        etype = "CURRENT"
        if self.accept("insert"):
            if self.accept("all"):
                self.expect("events")
                etype = "ALL"
            elif self.accept("current"):
                self.expect("events")
            elif self.accept("expired"):
                self.expect("events")
                etype = "EXPIRED"
            self.expect("into")
            hash_ = self.accept("#")
            out = ("#" if hash_ else "") + self.name()
        elif self.accept("return"):
            out = None
        else:
            raise SiddhiParserException(f"expected 'insert into' at {self.peek().pos}")
        return Query(inp, select, out, etype, annotations, group_by, having)

    def _scan_input_kind(self):
        """Decide pattern / sequence / standard by scanning the input tokens up to `select`/`insert`."""
        depth = 0
        k = self.i
        has_arrow = has_comma = has_state = False
        while True:
            t = self.toks[k]
            if t.kind == "eof":
                break
            if t.kind == "id" and depth == 0 and t.text.lower() in ("select", "insert", "return", "output"):
                break
            if t.kind == "op" and t.text in ("(", "["):
                depth += 1
            elif t.kind == "op" and t.text in (")", "]"):
                depth -= 1
            elif t.kind == "op" and t.text == "->":
                has_arrow = True
            elif t.kind == "op" and t.text == "," and depth == 0:
                has_comma = True
            elif t.kind == "id" and t.text.lower() in ("every", "not", "within"):
                has_state = True
            elif t.kind == "op" and t.text == "=" and depth == 0:
                has_state = True
            k += 1
        if has_comma:
            return "SEQUENCE"
        if has_arrow or has_state:
            return "PATTERN"
        return "STANDARD"

    def query_input(self):
        kind = self._scan_input_kind()
        if kind == "STANDARD":
            s = self.name()
            filters = []
            while self.at("[") or (self.at("#") and self.at("[", 1)):
                self.accept("#")
                self.expect("[")
                filters.append(self.expr())
                self.expect("]")
            if self.at("#"):
                raise SiddhiParserException("windows / stream functions are outside the pattern path")
            return StandardInput(s, filters)
        if kind == "PATTERN":
            el = self.pattern_chain()
        else:
            el = self.sequence_chain_top()
        within = None
        if self.accept("within"):
            within = self.time_value()
        return StateInput(kind, el, within)

    # time values --------------------------------------------------------------------------------
    def time_value(self):
        total = 0
        seen = False
        while self.peek().kind == "num" and self.peek(1).kind == "id" and _time_unit(self.peek(1).text):
            v = int(self.take().text)
            total += v * _time_unit(self.take().text)
            seen = True
        if not seen:
            raise SiddhiParserException(f"expected a time value at {self.peek().pos}")
        return total

    # pattern ------------------------------------------------------------------------------------
    def pattern_chain(self):
        left = self.pattern_term()
        while self.accept("->"):
            right = self.pattern_term()
            left = ENext(left, right)
        return left

    def pattern_term(self):
        if self.accept("every"):
            if self.at("("):
                self.expect("(")
                inner = self.pattern_chain()
                self.expect(")")
                return EEvery(inner)
            return EEvery(self.pattern_source())
        if self.at("(") and not self._paren_is_expression():
            self.expect("(")
            inner = self.pattern_chain()
            self.expect(")")
            return inner
        return self.pattern_source()

    def _paren_is_expression(self):
        return False

    def pattern_source(self, allow_collect_ops=False):
        """pattern_source / sequence_source: logical, counting or plain stateful source."""
        first = self.stateful_source(allow_collect_ops)
        if self.at("and") or self.at("or"):
            typ = self.take().text.upper()
            second = self.stateful_source(allow_collect_ops)
            for s in (first, second):
                if not isinstance(s, EStream):
                    raise SiddhiParserException("logical states combine plain stream states only")
            if second.absent and not first.absent:
                # the visitor puts the absent element first: State.logicalNotAnd(absent, present) /
                # State.logicalOr(absent, present) (SiddhiQLBaseVisitorImpl.java:1019-1042)
                first, second = second, first
            return ELogical(typ, first, second)
        return first

    def stateful_source(self, allow_collect_ops):
        if self.accept("not"):
            src = self.basic_source(None)
            src.absent = True
            if self.accept("for"):
                src.for_ms = self.time_value()
            return src
        ref = None
        if self.peek().kind == "id" and self.at("=", 1):
            ref = self.name()
            self.expect("=")
        src = self.basic_source(ref)
        if self.at("<"):
            self.expect("<")
            mn, mx = self.collect()
            self.expect(">")
            return ECount(src, mn, mx)
        if allow_collect_ops:
            if self.accept("*"):
                return ECount(src, 0, -1)
            if self.accept("?"):
                return ECount(src, 0, 1)
            if self.accept("+"):
                return ECount(src, 1, -1)
        return src

    def collect(self):
        # collect: INT ':' INT | INT ':' | ':' INT | INT
        if self.accept(":"):
            return -1, int(self.take().text)
        a = int(self.take().text)
        if self.accept(":"):
            if self.peek().kind == "num":
                return a, int(self.take().text)
            return a, -1
        return a, a

    def basic_source(self, ref):
        self.accept("#")
        s = self.name()
        filters = []
        while self.at("[") or (self.at("#") and self.at("[", 1)):
            self.accept("#")
            self.expect("[")
            filters.append(self.expr())
            self.expect("]")
        if self.at("#"):
            raise SiddhiParserException("stream functions inside pattern states are not supported")
        return EStream(s, ref, filters)

    # sequence -----------------------------------------------------------------------------------
    def sequence_chain_top(self):
        # every_sequence_source_chain: EVERY? sequence_source ',' sequence_source_chain
        every = bool(self.accept("every"))
        if self.at("("):
            self.expect("(")
            first = self.sequence_chain()
            self.expect(")")
        else:
            first = self.pattern_source(allow_collect_ops=True)
        if every:
            first = EEvery(first)
        self.expect(",")
        rest = self.sequence_chain()
        return self._seq_join(first, rest)

    def _seq_join(self, first, rest):
        # the visitor builds NextStateElement(first, chain); chain itself is left-assoc
        return ENext(first, rest)

    def sequence_chain(self):
        left = self.sequence_term()
        while self.accept(","):
            right = self.sequence_term()
            left = ENext(left, right)
        return left

    def sequence_term(self):
        if self.at("("):
            self.expect("(")
            inner = self.sequence_chain()
            self.expect(")")
            return inner
        return self.pattern_source(allow_collect_ops=True)

    # expressions (precedence per SiddhiQL.g4:456-471) -------------------------------------------
    def expr(self):
        return self.or_expr()

    def or_expr(self):
        left = self.and_expr()
        while self.accept("or"):
            left = BinOp("or", left, self.and_expr())
        return left

    def and_expr(self):
        left = self.in_expr()
        while self.accept("and"):
            left = BinOp("and", left, self.in_expr())
        return left

    def in_expr(self):
        left = self.eq_expr()
        if self.at("in"):
            raise SiddhiParserException("`in <table>` is outside the pattern path")
        return left

    def eq_expr(self):
        left = self.rel_expr()
        while self.at("==") or self.at("!="):
            op = self.take().text
            left = BinOp(op, left, self.rel_expr())
        return left

    def rel_expr(self):
        left = self.add_expr()
        while self.at(">=") or self.at("<=") or self.at(">") or self.at("<"):
            op = self.take().text
            left = BinOp(op, left, self.add_expr())
        return left

    def add_expr(self):
        left = self.mul_expr()
        while self.at("+") or self.at("-"):
            op = self.take().text
            left = BinOp(op, left, self.mul_expr())
        return left

    def mul_expr(self):
        left = self.unary()
        while self.at("*") or self.at("/") or self.at("%"):
            op = self.take().text
            left = BinOp(op, left, self.unary())
        return left

    def unary(self):
        if self.accept("not"):
            return Not(self.unary())
        return self.primary()

    def primary(self):
        t = self.peek()
        if self.accept("("):
            e = self.expr()
            self.expect(")")
            return self._maybe_is_null(e)
        if t.kind == "op" and t.text in ("-", "+") and self.peek(1).kind == "num":
            sign = self.take().text
            c = self.number(self.take().text)
            if sign == "-":
                c = Const(c.type, -c.value)
            return c
        if t.kind == "num":
            # time constants are long constants (Expression.Time.* -> TimeConstant extends LongConstant)
            if self.peek(1).kind == "id" and _time_unit(self.peek(1).text) and not self.at("(", 2):
                return Const("LONG", self.time_value())
            return self.number(self.take().text)
        if t.kind == "str":
            self.take()
            return Const("STRING", t.text[1:-1])
        if t.kind == "id" and t.text.lower() in ("true", "false"):
            self.take()
            return Const("BOOL", t.text.lower() == "true")
        if t.kind == "id" and t.text.lower() == "null":
            self.take()
            return Const("OBJECT", None)
        if t.kind == "op" and t.text in ("#", "!"):
            raise SiddhiParserException("inner/fault stream references are outside the pattern path")
        if t.kind == "id":
            # function call?
            if self.at("(", 1) or (self.at(":", 1) and self.peek(2).kind == "id" and self.at("(", 3)):
                ns = None
                nm = self.name()
                if self.accept(":"):
                    ns, nm = nm, self.name()
                self.expect("(")
                args = []
                if self.accept("*"):
                    args = ["*"]
                else:
                    while not self.at(")"):
                        args.append(self.expr())
                        if not self.accept(","):
                            break
                self.expect(")")
                return self._maybe_is_null(Func(ns, nm, args))
            nm = self.name()
            idx = None
            if self.at("["):
                self.expect("[")
                if self.accept("last"):
                    idx = LAST
                    if self.accept("-"):
                        idx = LAST - int(self.take().text)
                else:
                    idx = int(self.take().text)
                self.expect("]")
            if self.accept("."):
                attr = self.name()
                return self._maybe_is_null(Var(attr, nm, idx))
            if idx is not None or self.at("is"):
                # stream reference (null_check: stream_reference IS NULL)
                if self.at("is"):
                    self.expect("is")
                    self.expect("null")
                    return IsNullStream(nm, idx)
            return self._maybe_is_null(Var(nm))
        raise SiddhiParserException(f"unexpected token {t.text!r} at {t.pos}")

    def _maybe_is_null(self, e):
        if self.at("is") and self.at("null", 1):
            self.take()
            self.take()
            return IsNull(e)
        return e

    @staticmethod
    def number(text):
        suf = text[-1].lower()
        if suf == "l":
            return Const("LONG", int(text[:-1]))
        if suf == "f":
            return Const("FLOAT", float(text[:-1]))
        if suf == "d":
            return Const("DOUBLE", float(text[:-1]))
        if "." in text or "e" in text.lower():
            return Const("DOUBLE", float(text))
        v = int(text)
        if v > 2 ** 31 - 1:
            raise SiddhiParserException(f"int literal out of range: {text}")
        return Const("INT", v)


def parse_app(text: str) -> App:
    return Parser(text).parse_app()
