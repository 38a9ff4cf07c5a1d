"""Lowering of one pattern/sequence query to the engine IR (include/siddhi_gpu_ir.h).

What it restates from the reference (all paths under
/root/reference/modules/siddhi-core/src/main/java/io/siddhi/core/):

* slot numbering = the order in which StateInputStreamParser.parse visits stream states
  (util/parser/StateInputStreamParser.java:167-403; next: current then next :229-242,
  logical: element 2 before element 1 :349-361);
* variable resolution in filters and in the select list (util/parser/ExpressionParser.java:1255-1440:
  filters default to the CURRENT (= last) event of a slot's chain, SingleInputStreamParser.java:185-197;
  the selector defaults to index 0, SelectorParser.java:215; `e[last]` -> index -1, `e[last-k]` -> -1-k,
  and the self-reference rule for counting states :1377-1386);
* the typed condition executors: compare domains (executor/condition/compare/*/*.java, note that
  Equal/NotEqual of FLOAT with LONG compare as double while >,>=,<,<= use Java promotion) and the
  arithmetic result type (ExpressionParser.java:1489-1507).
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from typing import List, Optional

from . import siddhiql as q

# IR constants (keep in sync with include/siddhi_gpu_ir.h) --------------------------------------
SG_IR_MAGIC = 0x52494753
SG_IR_VERSION = 1
SG_IR_HDR_WORDS = 14
SG_IR_F_PARTITIONED = 1
SG_IR_F_PLAYBACK = 2
SG_COUNT_ANY = 0x7FFFFFFF

TYPE_CODE = {"STRING": 0, "INT": 1, "LONG": 2, "FLOAT": 3, "DOUBLE": 4, "BOOL": 5}
# projection roles (include/siddhi_gpu_ir.h)
AGG_CODE = {"count": 1, "sum": 2, "avg": 3, "min": 4, "max": 5, "minForever": 4, "maxForever": 5}
PROJ_AGG_ITEM, PROJ_HAVING = 0x10000, 0x20000
PROJ_SLOT_AGG, PROJ_SLOT_OUT = 0xFD, 0xFE
CODE_TYPE = {v: k for k, v in TYPE_CODE.items()}

N_STREAM, N_NEXT, N_EVERY, N_LOGICAL, N_COUNT = 1, 2, 3, 4, 5
L_AND, L_OR = 1, 2

OP_VAR, OP_CONST, OP_CVT = 1, 2, 3
OP_ARITH = {"+": 10, "-": 11, "*": 12, "/": 13, "%": 14}
OP_CMP = {"==": 20, "!=": 21, ">": 22, ">=": 23, "<": 24, "<=": 25}
OP_AND, OP_OR, OP_NOT, OP_ISNULL, OP_ISNULL_EV = 30, 31, 32, 33, 34
OP_IFELSE = 40

NUMERIC = ("INT", "LONG", "FLOAT", "DOUBLE")
_RANK = {"INT": 0, "LONG": 1, "FLOAT": 2, "DOUBLE": 3}


class SiddhiAppCreationException(Exception):
    """Mirrors io.siddhi.core.exception.SiddhiAppCreationException for unsupported / invalid apps."""


def compare_domain(op, lt, rt):
    """Domain in which `lt op rt` is compared (executor/condition/compare/<op>/*.java)."""
    if lt in ("STRING", "BOOL") or rt in ("STRING", "BOOL"):
        if lt == rt and op in ("==", "!="):
            return lt
        raise SiddhiAppCreationException(f"cannot compare {lt} {op} {rt}")
    if lt not in NUMERIC or rt not in NUMERIC:
        raise SiddhiAppCreationException(f"cannot compare {lt} {op} {rt}")
    if "DOUBLE" in (lt, rt):
        return "DOUBLE"
    if {lt, rt} == {"FLOAT", "LONG"}:
        # EqualCompareConditionExpressionExecutorFloatLong.java / LongFloat: doubleValue() == doubleValue()
        return "DOUBLE" if op in ("==", "!=") else "FLOAT"
    if "FLOAT" in (lt, rt):
        return "FLOAT"
    if "LONG" in (lt, rt):
        return "LONG"
    return "INT"


def arith_type(lt, rt):
    """ExpressionParser.parseArithmeticOperationResultType (ExpressionParser.java:1489-1507)."""
    if lt not in NUMERIC or rt not in NUMERIC:
        raise SiddhiAppCreationException(f"arithmetic between {lt} and {rt} cannot be executed")
    return lt if _RANK[lt] >= _RANK[rt] else rt


# ------------------------------------------------------------------------------------------------
@dataclass
class SlotInfo:
    slot: int
    ref: Optional[str]
    stream: str
    stream_idx: int
    multi_value: bool          # belongs to a counting state (chains several events)
    element: object = None


@dataclass
class ResolvedVar:
    slot: int
    attr_idx: int
    attr: str
    type: str
    chain_index: int           # >= 0 k-th, -1 last, -2 second to last ...
    multi_value: bool = False  # selector: whole chain as a list (MultiValueVariableFunctionExecutor)


@dataclass
class CompiledQuery:
    name: Optional[str]
    kind: str                            # PATTERN / SEQUENCE
    ir: bytes
    streams: List[q.StreamDef]           # IR stream table order
    slots: List[SlotInfo]
    within_ms: Optional[int]
    partition_keys: dict                 # stream name -> attr name (partitioned queries); None: the
                                         # stream is not keyed, its events go to every known key
    select: list                         # [(name, type, expr-tree with ResolvedVar leaves)]
    output_stream: Optional[str]
    query: q.Query
    element: object = None
    receiver_kinds: dict = field(default_factory=dict)
    aggregators: list = field(default_factory=list)   # [_Typed("agg")] in QuerySelector order
    group_by: list = field(default_factory=list)      # typed group-by expressions
    having: object = None                             # typed having condition (may read output names)

    @property
    def partitioned(self):
        return bool(self.partition_keys)

    def stream_index(self, name):
        for i, s in enumerate(self.streams):
            if s.name == name:
                return i
        return -1


class _Ctx:
    def __init__(self, app: q.App, stream_defs, strings):
        self.app = app
        self.stream_defs = stream_defs
        self.strings = strings           # StringDictionary (host-side id assignment)
        self.slots: List[SlotInfo] = []
        self.streams: List[q.StreamDef] = []
        self.code: List[int] = []

    def stream_idx(self, name):
        for i, s in enumerate(self.streams):
            if s.name == name:
                return i
        if name not in self.stream_defs:
            raise SiddhiAppCreationException(f"stream {name} is not defined")
        self.streams.append(self.stream_defs[name])
        return len(self.streams) - 1


# ------------------------------------------------------------------------------------------------
# variable resolution
# ------------------------------------------------------------------------------------------------

def _chain_index(var: q.Var, default):
    if var.index is None:
        return default
    if var.index <= q.LAST:
        return var.index + 1          # ExpressionParser.java:1263-1265
    return var.index


def resolve_filter_var(ctx: _Ctx, var: q.Var, cur: SlotInfo, visible: List[SlotInfo]):
    """parseVariable with currentState = cur.slot and defaultStreamEventIndex = CURRENT."""
    chain = _chain_index(var, -1)
    if var.stream is None:
        sd = ctx.stream_defs[cur.stream]
        ai = sd.attr_index(var.attr)
        if ai < 0:
            raise SiddhiAppCreationException(f"attribute {var.attr} not in stream {cur.stream}")
        return ResolvedVar(cur.slot, ai, var.attr, sd.attrs[ai][1], chain)
    target = None
    for s in visible:
        if s.ref is None:
            if s.stream == var.stream:
                target = s
                break
        elif s.ref == var.stream:
            target = s
            # a counting state referring to itself with [last..] keeps the raw index
            # (ExpressionParser.java:1377-1386)
            if cur.ref is not None and var.index is not None and var.index <= q.LAST and \
                    var.stream == cur.ref:
                chain = var.index
            break
    if target is None:
        raise SiddhiAppCreationException(
            f"Stream with reference '{var.stream}' not found for attribute '{var.attr}'")
    sd = ctx.stream_defs[target.stream]
    ai = sd.attr_index(var.attr)
    if ai < 0:
        raise SiddhiAppCreationException(f"attribute {var.attr} not in stream {target.stream}")
    return ResolvedVar(target.slot, ai, var.attr, sd.attrs[ai][1], chain)


def resolve_select_var(ctx: _Ctx, var: q.Var):
    """parseVariable with currentState = UNKNOWN and defaultStreamEventIndex = 0 (selector)."""
    chain = _chain_index(var, 0)
    if var.stream is None:
        found = None
        for s in ctx.slots:
            sd = ctx.stream_defs[s.stream]
            ai = sd.attr_index(var.attr)
            if ai >= 0:
                if found is not None:
                    raise SiddhiAppCreationException(
                        f"{found[0].stream} and {s.stream} both contain attribute '{var.attr}'")
                found = (s, ai)
        if found is None:
            raise SiddhiAppCreationException(f"No matching stream reference found for attribute '{var.attr}'")
        s, ai = found
        return ResolvedVar(s.slot, ai, var.attr, ctx.stream_defs[s.stream].attrs[ai][1], chain)
    for s in ctx.slots:
        if (s.ref is None and s.stream == var.stream) or (s.ref is not None and s.ref == var.stream):
            sd = ctx.stream_defs[s.stream]
            ai = sd.attr_index(var.attr)
            if ai < 0:
                raise SiddhiAppCreationException(f"attribute {var.attr} not in stream {s.stream}")
            multi = s.multi_value and var.index is None
            return ResolvedVar(s.slot, ai, var.attr, sd.attrs[ai][1], chain, multi)
    raise SiddhiAppCreationException(f"Stream with reference '{var.stream}' not found for attribute '{var.attr}'")


# ------------------------------------------------------------------------------------------------
# typing + bytecode
# ------------------------------------------------------------------------------------------------

class _Typed:
    """Expression tree annotated with result types; leaves are ResolvedVar / Const."""

    def __init__(self, kind, type_, **kw):
        self.kind = kind
        self.type = type_
        self.__dict__.update(kw)


def type_expr(ctx: _Ctx, e, resolve, funcs=None):
    """funcs: typer of function calls (select / having only; filters on the device path take none)"""
    if isinstance(e, q.Const):
        if e.type == "OBJECT":
            return _Typed("const", "OBJECT", value=None)
        return _Typed("const", e.type, value=e.value)
    if isinstance(e, q.Var):
        rv = resolve(e)
        if isinstance(rv, _Typed):   # a having clause naming an output attribute
            return rv
        return _Typed("var", "OBJECT" if rv.multi_value else rv.type, var=rv)
    if isinstance(e, q.IsNullStream):
        # `e1 is null` inside a state query: the stream event itself (IsNullStreamConditionExpressionExecutor)
        try:
            v = resolve(q.Var("__stream__", e.stream, e.index))
        except SiddhiAppCreationException:
            if e.index is not None:
                raise
            # not a stream reference: `<attribute> is null` (e.g. an output attribute in `having`)
            return _Typed("isnull", "BOOL", arg=type_expr(ctx, q.Var(e.stream, None, None), resolve, funcs))
        return _Typed("isnull_ev", "BOOL", slot=v.slot, chain=v.chain_index)
    if isinstance(e, q.IsNull):
        inner = type_expr(ctx, e.expr, resolve, funcs)
        return _Typed("isnull", "BOOL", arg=inner)
    if isinstance(e, q.Not):
        inner = type_expr(ctx, e.expr, resolve, funcs)
        if inner.type != "BOOL":
            raise SiddhiAppCreationException("NOT needs a BOOL operand")
        return _Typed("not", "BOOL", arg=inner)
    if isinstance(e, q.BinOp):
        lt = type_expr(ctx, e.left, resolve, funcs)
        rt = type_expr(ctx, e.right, resolve, funcs)
        if e.op in ("and", "or"):
            if lt.type != "BOOL" or rt.type != "BOOL":
                raise SiddhiAppCreationException(f"{e.op.upper()} needs BOOL operands")
            return _Typed(e.op, "BOOL", left=lt, right=rt)
        if e.op in OP_CMP:
            # null constants compare as null (always false / NE true); give them the other side's type
            if lt.type == "OBJECT" and lt.kind == "const":
                lt.type = rt.type
            if rt.type == "OBJECT" and rt.kind == "const":
                rt.type = lt.type
            dom = compare_domain(e.op, lt.type, rt.type)
            return _Typed("cmp", "BOOL", op=e.op, dom=dom, left=lt, right=rt)
        if e.op in OP_ARITH:
            t = arith_type(lt.type, rt.type)
            return _Typed("arith", t, op=e.op, left=lt, right=rt)
    if isinstance(e, q.Func) and e.namespace is None and e.name == "ifThenElse":
        # IfThenElseFunctionExecutor.init (C/executor/function/IfThenElseFunctionExecutor.java:101-121):
        # three arguments, a BOOL condition, then / else of the same type (the result type)
        if len(e.args) != 3:
            raise SiddhiAppCreationException("ifThenElse() needs 3 arguments")
        c, x, y = (type_expr(ctx, a, resolve, funcs) for a in e.args)
        if c.type != "BOOL":
            raise SiddhiAppCreationException(f"ifThenElse() condition must be BOOL, not {c.type}")
        if x.type != y.type:
            raise SiddhiAppCreationException(f"ifThenElse() then / else types differ: {x.type} and {y.type}")
        return _Typed("ifelse", x.type, cond=c, left=x, right=y)
    if isinstance(e, q.Func):
        if funcs is not None:
            return funcs(e)
        raise SiddhiAppCreationException(f"function {e.name}() is not supported on the pattern path")
    raise SiddhiAppCreationException(f"unsupported expression {e!r}")


class _Emitter:
    def __init__(self, strings):
        self.code: List[int] = []
        self.strings = strings

    def w(self, *words):
        for x in words:
            self.code.append(x & 0xFFFFFFFF)

    def hdr(self, op, a=0, b=0, c=0):
        self.w(op | (a << 8) | (b << 16) | (c << 24))

    def emit(self, t: _Typed, want: Optional[str] = None):
        k = t.kind
        if k == "const":
            ty = want if t.value is None and want else t.type
            if t.value is None:
                self.hdr(OP_CONST, TYPE_CODE.get(ty, 1), 1)
                self.w(0, 0)
            else:
                ty = t.type
                if ty == "STRING":
                    bits = self.strings.id_of(t.value)
                elif ty == "BOOL":
                    bits = 1 if t.value else 0
                elif ty == "INT":
                    bits = t.value & 0xFFFFFFFF
                elif ty == "LONG":
                    bits = t.value & 0xFFFFFFFFFFFFFFFF
                elif ty == "FLOAT":
                    bits = struct.unpack("<I", struct.pack("<f", t.value))[0]
                elif ty == "DOUBLE":
                    bits = struct.unpack("<Q", struct.pack("<d", t.value))[0]
                else:
                    raise SiddhiAppCreationException(f"constant of type {ty}")
                self.hdr(OP_CONST, TYPE_CODE[ty], 0)
                self.w(bits & 0xFFFFFFFF, (bits >> 32) & 0xFFFFFFFF)
                self.cvt(ty, want)
            return
        if k == "var":
            v = t.var
            self.hdr(OP_VAR, TYPE_CODE[v.type], v.slot)
            self.w(v.attr_idx, v.chain_index)
            self.cvt(v.type, want)
            return
        if k == "agg":   # the aggregator's current value (SG_PROJ_SLOT_AGG, after its processAdd)
            self.hdr(OP_VAR, TYPE_CODE[t.type], PROJ_SLOT_AGG)
            self.w(t.idx, 0)
            self.cvt(t.type, want)
            return
        if k == "out":   # select item `idx` of the same output row (having over output attributes)
            self.hdr(OP_VAR, TYPE_CODE[t.type], PROJ_SLOT_OUT)
            self.w(t.idx, 0)
            self.cvt(t.type, want)
            return
        if k == "isnull_ev":
            self.hdr(OP_ISNULL_EV, 0, t.slot)
            self.w(t.chain)
            return
        if k == "isnull":
            self.emit(t.arg)
            self.hdr(OP_ISNULL)
            return
        if k == "not":
            self.emit(t.arg)
            self.hdr(OP_NOT)
            return
        if k in ("and", "or"):
            self.emit(t.left)
            self.emit(t.right)
            self.hdr(OP_AND if k == "and" else OP_OR)
            return
        if k == "ifelse":
            self.emit(t.cond)
            self.emit(t.left)
            self.emit(t.right)
            self.hdr(OP_IFELSE, TYPE_CODE[t.type])
            self.cvt(t.type, want)
            return
        if k == "cmp":
            self.emit(t.left, t.dom)
            self.emit(t.right, t.dom)
            self.hdr(OP_CMP[t.op], TYPE_CODE[t.dom])
            return
        if k == "arith":
            self.emit(t.left, t.type)
            self.emit(t.right, t.type)
            self.hdr(OP_ARITH[t.op], TYPE_CODE[t.type])
            self.cvt(t.type, want)
            return
        raise SiddhiAppCreationException(f"cannot emit {k}")

    def cvt(self, frm, to):
        if to is None or to == frm or frm in ("OBJECT",):
            return
        if frm in NUMERIC and to in NUMERIC and _RANK[to] > _RANK[frm]:
            self.hdr(OP_CVT, TYPE_CODE[frm], TYPE_CODE[to])
            return
        raise SiddhiAppCreationException(f"cannot convert {frm} to {to}")


# ------------------------------------------------------------------------------------------------
# lowering
# ------------------------------------------------------------------------------------------------

def _assign_slots(ctx: _Ctx, el, multi=False):
    """Slot order = StateInputStreamParser.parse visit order."""
    if isinstance(el, q.EStream):
        si = SlotInfo(len(ctx.slots), el.ref, el.stream, ctx.stream_idx(el.stream), multi, el)
        ctx.slots.append(si)
        el._slot = si
        return
    if isinstance(el, q.ENext):
        _assign_slots(ctx, el.current)
        _assign_slots(ctx, el.next)
        return
    if isinstance(el, q.EEvery):
        _assign_slots(ctx, el.child)
        return
    if isinstance(el, q.ELogical):
        _assign_slots(ctx, el.e2)
        _assign_slots(ctx, el.e1)
        return
    if isinstance(el, q.ECount):
        _assign_slots(ctx, el.child, True)
        return
    raise SiddhiAppCreationException(f"unsupported state element {el!r}")


def _compile_filters(ctx: _Ctx, em: _Emitter, el):
    if isinstance(el, q.EStream):
        si = el._slot
        visible = ctx.slots[: si.slot + 1]
        if not el.filters:
            el._filter = (0, 0)
            return
        resolve = lambda v: resolve_filter_var(ctx, v, si, visible)
        pc = len(em.code)
        for i, f in enumerate(el.filters):
            t = type_expr(ctx, f, resolve)
            if t.type != "BOOL":
                raise SiddhiAppCreationException("filter condition must be BOOL")
            em.emit(t)
            if i > 0:      # consecutive filters [a][b] behave as a and b
                em.hdr(OP_AND)
        el._filter = (pc, len(em.code) - pc)
        return
    if isinstance(el, q.ENext):
        _compile_filters(ctx, em, el.current)
        _compile_filters(ctx, em, el.next)
    elif isinstance(el, q.EEvery):
        _compile_filters(ctx, em, el.child)
    elif isinstance(el, q.ELogical):
        _compile_filters(ctx, em, el.e2)
        _compile_filters(ctx, em, el.e1)
    elif isinstance(el, q.ECount):
        _compile_filters(ctx, em, el.child)


def _encode_nodes(el, out: List[int]):
    if isinstance(el, q.EStream):
        pc, ln = el._filter
        for_ms = el.for_ms if el.for_ms is not None else -1
        out += [N_STREAM, el._slot.slot, el._slot.stream_idx, pc, ln, 1 if el.absent else 0,
                for_ms & 0xFFFFFFFF, (for_ms >> 32) & 0xFFFFFFFF]
    elif isinstance(el, q.ENext):
        out.append(N_NEXT)
        _encode_nodes(el.current, out)
        _encode_nodes(el.next, out)
    elif isinstance(el, q.EEvery):
        out.append(N_EVERY)
        _encode_nodes(el.child, out)
    elif isinstance(el, q.ELogical):
        out += [N_LOGICAL, L_AND if el.type == "AND" else L_OR]
        _encode_nodes(el.e1, out)
        _encode_nodes(el.e2, out)
    elif isinstance(el, q.ECount):
        mn = 0 if el.min < 0 else el.min
        mx = SG_COUNT_ANY if el.max < 0 else el.max
        out += [N_COUNT, mn, mx]
        _encode_nodes(el.child, out)


def _stream_counts(el, acc):
    if isinstance(el, q.EStream):
        acc[el.stream] = acc.get(el.stream, 0) + 1
    elif isinstance(el, q.ENext):
        _stream_counts(el.current, acc)
        _stream_counts(el.next, acc)
    elif isinstance(el, q.EEvery):
        _stream_counts(el.child, acc)
    elif isinstance(el, q.ELogical):
        _stream_counts(el.e1, acc)
        _stream_counts(el.e2, acc)
    elif isinstance(el, q.ECount):
        _stream_counts(el.child, acc)
    return acc


NUMERIC = ("INT", "LONG", "FLOAT", "DOUBLE")
INSTANCE_OF = {"instanceOfBoolean": "BOOL", "instanceOfDouble": "DOUBLE", "instanceOfFloat": "FLOAT",
               "instanceOfInteger": "INT", "instanceOfLong": "LONG", "instanceOfString": "STRING"}


def _type_select_func(ctx, f, resolve, funcs, aggs):
    """Function calls of a select / having clause.  Aggregators follow
    C/query/selector/attribute/aggregator/*AttributeAggregatorExecutor.java (return types from their
    init: count/distinctCount LONG, sum LONG for int/long and DOUBLE for float/double, avg DOUBLE,
    min/max the argument's type); instanceOf* follow C/executor/function/InstanceOf*FunctionExecutor.java
    (true iff the value is a non-null instance of that type)."""
    if f.namespace is not None:
        raise SiddhiAppCreationException(f"function {f.namespace}:{f.name}() is not supported")
    args = [type_expr(ctx, a, resolve, funcs) for a in f.args]
    for a in args:
        if _has_agg(a) and f.name not in INSTANCE_OF:
            raise SiddhiAppCreationException(f"aggregator inside {f.name}()")
    n = f.name
    if n in INSTANCE_OF:
        if len(args) != 1:
            raise SiddhiAppCreationException(f"{n}() takes one argument")
        return _Typed("instof", "BOOL", arg=args[0], want=INSTANCE_OF[n])
    if n == "count" and len(args) <= 1:
        t = "LONG"
    elif n == "distinctCount" and len(args) == 1:
        t = "LONG"
    elif n in ("sum", "avg", "min", "max", "minForever", "maxForever") and len(args) == 1:
        at = args[0].type
        if at not in NUMERIC:
            raise SiddhiAppCreationException(f"{n}() not supported for {at}")
        t = {"sum": "LONG" if at in ("INT", "LONG") else "DOUBLE", "avg": "DOUBLE"}.get(n, at)
    else:
        raise SiddhiAppCreationException(f"function {n}() is not supported in select")
    a = _Typed("agg", t, fn=n, arg=args[0] if args else None, idx=len(aggs))
    aggs.append(a)
    return a


def _has_agg(t):
    if t.kind == "agg":
        return True
    return any(_has_agg(getattr(t, k)) for k in ("left", "right", "arg")
               if isinstance(getattr(t, k, None), _Typed))


def compile_query(app: q.App, query: q.Query, strings) -> CompiledQuery:
    if not isinstance(query.input, q.StateInput):
        raise SiddhiAppCreationException("only pattern / sequence queries run on this engine")
    si = query.input
    ctx = _Ctx(app, app.streams, strings)
    _assign_slots(ctx, si.element)
    em = _Emitter(strings)
    _compile_filters(ctx, em, si.element)
    nodes: List[int] = []
    _encode_nodes(si.element, nodes)

    partition_keys = {}
    if query.partition is not None:
        for attr, stream in query.partition.keys:
            partition_keys[stream] = attr
        for s in ctx.streams:
            if s.name not in partition_keys:
                # a stream the partition does not key: each of its events goes to every partition key
                # known at that moment (PartitionStreamReceiver.receive with no partition executor ->
                # send(ComplexEvent), C/partition/PartitionStreamReceiver.java:83-92, 275-283)
                partition_keys[s.name] = None
                continue
            if s.attr_index(partition_keys[s.name]) < 0:
                raise SiddhiAppCreationException(f"partition attribute {partition_keys[s.name]} "
                                                 f"not in {s.name}")

    # select list (host-side projection, QuerySelector) -----------------------------------------
    select = []
    aggs: List[_Typed] = []
    resolve = lambda v: resolve_select_var(ctx, v)
    funcs = lambda f: _type_select_func(ctx, f, resolve, funcs, aggs)
    if query.select is None:
        names = set()
        for s in ctx.slots:
            for an, at in ctx.stream_defs[s.stream].attrs:
                if an in names:
                    raise SiddhiAppCreationException(f"Duplicate attribute '{an}' in select *")
                names.add(an)
                select.append((an, at, type_expr(ctx, q.Var(an), resolve)))
    else:
        for oa in query.select:
            t = type_expr(ctx, oa.expr, resolve, funcs)
            name = oa.rename
            if name is None:
                if isinstance(oa.expr, q.Var):
                    name = oa.expr.attr
                else:
                    raise SiddhiAppCreationException("select expressions need 'as <name>'")
            select.append((name, t.type, t))
    group_by = [type_expr(ctx, g, resolve) for g in query.group_by]
    having = None
    if query.having is not None:
        out_idx = {name: i for i, (name, _, _) in enumerate(select)}

        def resolve_having(v):
            # the output stream's attributes first (QueryParserHelper: having runs on the projected event)
            if v.stream is None and v.index is None and v.attr in out_idx:
                i = out_idx[v.attr]
                return _Typed("out", select[i][1], idx=i)
            return resolve(v)
        hfuncs = lambda f: _type_select_func(ctx, f, resolve_having, hfuncs, aggs)
        having = type_expr(ctx, query.having, resolve_having, hfuncs)
        if having.type != "BOOL":
            raise SiddhiAppCreationException("having needs a BOOL condition")

    # IR ---------------------------------------------------------------------------------------
    stream_words: List[int] = []
    for s in ctx.streams:
        stream_words.append(len(s.attrs))
        for _, at in s.attrs:
            if at not in TYPE_CODE:
                raise SiddhiAppCreationException(f"attribute type {at} is not supported on the engine")
            stream_words.append(TYPE_CODE[at])
    slot_words: List[int] = []
    for s in ctx.slots:
        slot_words += [s.stream_idx, 1 if s.multi_value else 0]
    within = -1 if si.within_ms is None else si.within_ms
    off_streams = SG_IR_HDR_WORDS
    off_slots = off_streams + len(stream_words)
    off_nodes = off_slots + len(slot_words)
    off_code = off_nodes + len(nodes)
    hdr = [SG_IR_MAGIC, SG_IR_VERSION, 0 if si.kind == "PATTERN" else 1, len(ctx.streams),
           len(ctx.slots), within & 0xFFFFFFFF, (within >> 32) & 0xFFFFFFFF,
           off_streams, off_nodes, len(nodes), off_code, len(em.code),
           (SG_IR_F_PARTITIONED if partition_keys else 0) |
           (SG_IR_F_PLAYBACK if any(a.name.lower() == "app:playback" for a in app.annotations) else 0),
           off_slots]
    words = hdr + stream_words + slot_words + nodes + em.code
    ir = struct.pack(f"<{len(words)}I", *[w & 0xFFFFFFFF for w in words])

    counts = _stream_counts(si.element, {})
    recv = {}
    for s in ctx.streams:
        multi = counts.get(s.name, 0) > 1
        recv[s.name] = ("SEQUENCE" if si.kind == "SEQUENCE" else "PATTERN") + ("_MULTI" if multi else "_SINGLE")

    return CompiledQuery(query.name, si.kind, ir, list(ctx.streams), list(ctx.slots), si.within_ms,
                         partition_keys, select, query.output_stream, query, si.element, recv,
                         aggs, group_by, having)


def _has_kind(t, kinds):
    if t.kind in kinds:
        return True
    return any(_has_kind(getattr(t, k), kinds) for k in ("left", "right", "arg", "cond")
               if isinstance(getattr(t, k, None), _Typed))


def projection_program(cq: CompiledQuery, strings):
    """The selector as device expression programs (sg_set_projection), or None when it must run on the
    host: group by (per-group aggregator states), distinctCount, multi-valued count attributes (OBJECT
    lists), instanceOf checks.  Items in QuerySelector order (siddhi_gpu_ir.h): one argument program per
    aggregator (empty for count()), the select list (reading aggregator values through
    SG_PROJ_SLOT_AGG), then `having` (reading output attributes through SG_PROJ_SLOT_OUT).
    Returns (code words, item pc, item len, item type codes, partition attribute per IR stream)."""
    if cq.group_by:
        return None
    em = _Emitter(strings)
    pcs, lens, types = [], [], []

    def item(t, code):
        pcs.append(len(em.code))
        if t is not None:
            em.emit(t)
        lens.append(len(em.code) - pcs[-1])
        types.append(code)

    for a in cq.aggregators:
        if a.fn not in AGG_CODE or (a.arg is not None and (a.arg.type not in TYPE_CODE or
                                                           _has_kind(a.arg, ("agg", "instof", "out")))):
            return None
        at = a.arg.type if a.arg is not None else "LONG"
        item(a.arg, TYPE_CODE[at] | (AGG_CODE[a.fn] << 8) | PROJ_AGG_ITEM)
    for name, typ, t in cq.select:
        if typ not in TYPE_CODE or _has_kind(t, ("instof", "out")):
            return None
        item(t, TYPE_CODE[typ])
    if cq.having is not None:
        if _has_kind(cq.having, ("instof",)):
            return None
        item(cq.having, TYPE_CODE["BOOL"] | PROJ_HAVING)
    part = []
    for s in cq.streams:
        attr = cq.partition_keys.get(s.name) if cq.partitioned else None
        part.append(s.attr_index(attr) if attr else -1)
    return em.code, pcs, lens, types, part