"""The gRPC contract must be wire-identical to the reference's .proto files.

The reference's own `agent-core/proto/*.proto` text is the oracle: every message field (name,
number, type, label) and every service method (request/response type, streaming) our runtime-
built descriptor pool defines is compared against it.  Skipped if the reference tree is absent.
"""
import os
import re

import pytest

from aios_amd.rpc import schema
from aios_amd.rpc.schema import build_pool, message, pb, service

REF = "/root/reference/agent-core/proto"
SCALAR = {"string", "int32", "int64", "uint32", "uint64", "bool", "bytes", "double", "float", "sint32", "sint64",
          "fixed32", "fixed64"}


def _strip_comments(t):
    t = re.sub(r"/\*.*?\*/", "", t, flags=re.S)
    return re.sub(r"//[^\n]*", "", t)


def _blocks(text, kind):
    """Yield (name, body) for top-level `message`/`service` blocks (nested braces handled)."""
    i = 0
    pat = re.compile(r"\b%s\s+(\w+)\s*\{" % kind)
    while True:
        m = pat.search(text, i)
        if not m:
            return
        depth, j = 1, m.end()
        while depth:
            depth += {"{": 1, "}": -1}.get(text[j], 0)
            j += 1
        yield m.group(1), text[m.end():j - 1]
        i = j


def _parse_ref(fname):
    text = _strip_comments(open(os.path.join(REF, fname)).read())
    pkg = re.search(r"\bpackage\s+([\w.]+)\s*;", text).group(1)
    msgs, svcs = {}, {}
    for name, body in _blocks(text, "message"):
        fields = {}
        for fm in re.finditer(r"(repeated\s+)?(map\s*<\s*\w+\s*,\s*[\w.]+\s*>|[\w.]+)\s+(\w+)\s*=\s*(\d+)\s*;", body):
            fields[fm.group(3)] = (bool(fm.group(1)), re.sub(r"\s", "", fm.group(2)), int(fm.group(4)))
        msgs[name] = fields
    for name, body in _blocks(text, "service"):
        svcs[name] = {m.group(1): (m.group(2), bool(m.group(3)), m.group(4)) for m in re.finditer(
            r"rpc\s+(\w+)\s*\(\s*([\w.]+)\s*\)\s*returns\s*\(\s*(stream\s+)?([\w.]+)\s*\)", body)}
    return pkg, msgs, svcs


def _type_name(fd):
    from google.protobuf.descriptor import FieldDescriptor as FD

    if fd.type == FD.TYPE_MESSAGE:
        if fd.message_type.GetOptions().map_entry:
            k, v = fd.message_type.fields_by_name["key"], fd.message_type.fields_by_name["value"]
            return f"map<{_type_name(k)},{_type_name(v)}>"
        return fd.message_type.full_name
    return {FD.TYPE_STRING: "string", FD.TYPE_INT32: "int32", FD.TYPE_INT64: "int64", FD.TYPE_UINT32: "uint32",
            FD.TYPE_UINT64: "uint64", FD.TYPE_BOOL: "bool", FD.TYPE_BYTES: "bytes", FD.TYPE_DOUBLE: "double",
            FD.TYPE_FLOAT: "float"}[fd.type]


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference proto tree not present")
@pytest.mark.parametrize("fname", sorted(f for f in os.listdir(REF) if f.endswith(".proto")) if os.path.isdir(REF) else [])
def test_proto_matches_reference(fname):
    pkg, msgs, svcs = _parse_ref(fname)
    pool = build_pool()
    for mname, fields in msgs.items():
        d = pool.FindMessageTypeByName(f"{pkg}.{mname}")
        ours = {f.name: f for f in d.fields}
        assert set(ours) == set(fields), f"{pkg}.{mname}: {set(ours) ^ set(fields)}"
        for fname_, (rep, typ, num) in fields.items():
            fd = ours[fname_]
            assert fd.number == num, f"{pkg}.{mname}.{fname_} number"
            t = _type_name(fd)
            if typ.startswith("map<"):
                assert t == typ.replace(" ", ""), (mname, fname_, t, typ)
                continue
            assert fd.is_repeated == rep, f"{pkg}.{mname}.{fname_} label"
            if typ in SCALAR:
                assert t == typ, (mname, fname_, t, typ)
            else:
                assert t.split(".")[-1] == typ.split(".")[-1], (mname, fname_, t, typ)
    for sname, methods in svcs.items():
        sd = pool.FindServiceByName(f"{pkg}.{sname}")
        ours = {m.name: m for m in sd.methods}
        assert set(ours) == set(methods), f"{sname}: {set(ours) ^ set(methods)}"
        for mname, (req, stream, resp) in methods.items():
            md = ours[mname]
            assert md.input_type.name == req.split(".")[-1]
            assert md.output_type.name == resp.split(".")[-1]
            assert md.server_streaming == stream


def test_service_inventory():
    n = sum(len(service(s).methods) for s in schema.SERVICES)
    assert n == 63
    assert schema.SERVICES["aios.runtime.AIRuntime"] == 50055
    assert [m.name for m in service("aios.runtime.AIRuntime").methods] == [
        "LoadModel", "UnloadModel", "ListModels", "Infer", "StreamInfer", "HealthCheck"]


def test_message_roundtrip():
    r = pb.runtime.InferRequest(model="m", prompt="p", max_tokens=5, temperature=0.5, intelligence_level="tactical")
    r2 = pb.runtime.InferRequest.FromString(r.SerializeToString())
    assert r2 == r
    h = pb.common.HealthStatus(healthy=True, service="x")
    h.details["a"] = "b"
    assert pb.common.HealthStatus.FromString(h.SerializeToString()).details["a"] == "b"
    assert message("aios.runtime.InferChunk")(text="t", done=True).done


def test_emit_proto_is_parseable_text():
    for fname in schema.ORDER:
        txt = schema.emit_proto(fname)
        assert txt.startswith('syntax = "proto3";')
        assert "package aios." in txt
