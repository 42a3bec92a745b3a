"""protobuf <-> plain-dict conversion for the native cores, which take and return records keyed
by the proto field names.  `bytes` fields (the *_json payloads) cross as UTF-8 text."""
from __future__ import annotations

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


def from_dict(cls, d: dict):
    msg = cls()
    fields = cls.DESCRIPTOR.fields_by_name
    for k, v in (d or {}).items():
        f = fields.get(k)
        if f is None or v is None:
            continue
        if f.message_type is not None and f.message_type.GetOptions().map_entry:
            getattr(msg, k).update({str(a): str(b) for a, b in v.items()})
        elif _is_repeated(f):
            if f.type == FD.TYPE_MESSAGE:
                sub = getattr(msg, k)
                for x in v:
                    sub.add().CopyFrom(from_dict(f.message_type._concrete_class, x))
            else:
                getattr(msg, k).extend(v)
        elif f.type == FD.TYPE_MESSAGE:
            getattr(msg, k).CopyFrom(from_dict(f.message_type._concrete_class, v))
        elif f.type == _BYTES:
            setattr(msg, k, v.encode() if isinstance(v, str) else bytes(v))
        elif f.type in (FD.TYPE_FLOAT, FD.TYPE_DOUBLE):
            setattr(msg, k, float(v))
        elif f.type == FD.TYPE_BOOL:
            setattr(msg, k, bool(v))
        elif f.type == FD.TYPE_STRING:
            setattr(msg, k, str(v))
        else:
            setattr(msg, k, int(v))
    return msg
