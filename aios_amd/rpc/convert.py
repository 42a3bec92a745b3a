"""protobuf <-> plain-dict conversion for the native cores, which take and return records keyed
by the proto field names.  `bytes` fields (the *_json payloads) cross as UTF-8 text."""
from __future__ import annotations

from google.protobuf import message_factory
from google.protobuf.descriptor import FieldDescriptor as FD

_BYTES = FD.TYPE_BYTES


def _is_repeated(f) -> bool:
    return f.is_repeated if hasattr(f, "is_repeated") else f.label == FD.LABEL_REPEATED


def to_dict(msg) -> dict:
    out = {}
    for f in msg.DESCRIPTOR.fields:
        v = getattr(msg, f.name)
        if f.message_type is not None and f.message_type.GetOptions().map_entry:
            out[f.name] = dict(v)
        elif _is_repeated(f):
            out[f.name] = [to_dict(x) if f.type == FD.TYPE_MESSAGE else x for x in v]
        elif f.type == FD.TYPE_MESSAGE:
            out[f.name] = to_dict(v) if msg.HasField(f.name) else {}
        elif f.type == _BYTES:
            out[f.name] = v.decode("utf-8", "replace")
        else:
            out[f.name] = v
    return out


_PLANS: dict = {}
_MAP, _RMSG, _REP, _MSG, _BYT, _FLT, _BOOL, _STR, _INT = range(9)


def _plan(cls) -> dict:
    """name -> (kind, sub-message class) for every field of `cls`, computed once per class."""
    plan = _PLANS.get(cls)
    if plan is None:
        plan = {}
        for f in cls.DESCRIPTOR.fields:
            mt = f.message_type
            is_map = mt is not None and mt.GetOptions().map_entry
            sub = message_factory.GetMessageClass(mt) if mt is not None and not is_map else None
            if is_map:
                kind = _MAP
            elif sub is not None and _is_repeated(f):
                kind = _RMSG
            elif _is_repeated(f):
                kind = _REP
            elif f.type == FD.TYPE_MESSAGE:
                kind = _MSG
            elif f.type == _BYTES:
                kind = _BYT
            elif f.type in (FD.TYPE_FLOAT, FD.TYPE_DOUBLE):
                kind = _FLT
            elif f.type == FD.TYPE_BOOL:
                kind = _BOOL
            elif f.type == FD.TYPE_STRING:
                kind = _STR
            else:
                kind = _INT
            plan[f.name] = (kind, sub)
        _PLANS[cls] = plan
    return plan


def from_dict(cls, d: dict):
    """`cls` built from a field-name dict in one constructor call (unknown keys and None values are
    skipped; the per-class field plan is cached -- the list RPCs convert hundreds of records per call)."""
    plan = _plan(cls)
    kw = {}
    for k, v in (d or {}).items():
        p = plan.get(k)
        if p is None or v is None:
            continue
        kind, sub = p
        if kind == _STR:
            kw[k] = v if isinstance(v, str) else str(v)
        elif kind == _INT:
            kw[k] = int(v)
        elif kind == _FLT:
            kw[k] = float(v)
        elif kind == _BOOL:
            kw[k] = bool(v)
        elif kind == _BYT:
            kw[k] = v.encode() if isinstance(v, str) else bytes(v)
        elif kind == _REP:
            kw[k] = v
        elif kind == _RMSG:
            kw[k] = [from_dict(sub, x) for x in v]
        elif kind == _MSG:
            kw[k] = from_dict(sub, v)
        else:
            kw[k] = {str(a): str(b) for a, b in v.items()}
    return cls(**kw)
