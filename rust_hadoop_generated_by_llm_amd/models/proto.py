"""proto3 message classes built at import time from ``proto/dfs.proto``.

There is no ``protoc`` in this environment, so a small parser turns the IDL into a
``FileDescriptorProto`` and ``google.protobuf`` builds real (upb-backed) message classes
from it. The wire encoding is therefore exactly protobuf's, i.e. byte-compatible with the
reference's prost/tonic messages (reference: proto/dfs.proto).

Usage::

    from rust_hadoop_generated_by_llm_amd.models import proto as pb
    req = pb.WriteBlockRequest(block_id="x", data=b"...")
    pb.SERVICES["ChunkServerService"]  # -> [(method, request_cls, response_cls), ...]
"""
from __future__ import annotations

import re
from pathlib import Path

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

PROTO_PATH = Path(__file__).resolve().parents[2] / "proto" / "dfs.proto"

_SCALARS = {
    "double": descriptor_pb2.FieldDescriptorProto.TYPE_DOUBLE,
    "float": descriptor_pb2.FieldDescriptorProto.TYPE_FLOAT,
    "int64": descriptor_pb2.FieldDescriptorProto.TYPE_INT64,
    "uint64": descriptor_pb2.FieldDescriptorProto.TYPE_UINT64,
    "int32": descriptor_pb2.FieldDescriptorProto.TYPE_INT32,
    "uint32": descriptor_pb2.FieldDescriptorProto.TYPE_UINT32,
    "bool": descriptor_pb2.FieldDescriptorProto.TYPE_BOOL,
    "string": descriptor_pb2.FieldDescriptorProto.TYPE_STRING,
    "bytes": descriptor_pb2.FieldDescriptorProto.TYPE_BYTES,
    "sint32": descriptor_pb2.FieldDescriptorProto.TYPE_SINT32,
    "sint64": descriptor_pb2.FieldDescriptorProto.TYPE_SINT64,
    "fixed32": descriptor_pb2.FieldDescriptorProto.TYPE_FIXED32,
    "fixed64": descriptor_pb2.FieldDescriptorProto.TYPE_FIXED64,
}
_TOKEN = re.compile(r'[A-Za-z_][A-Za-z0-9_.]*|\d+|"[^"]*"|[{}()<>;=,\[\]]')
_FDP = descriptor_pb2.FieldDescriptorProto


def _tokens(text: str) -> list[str]:
    text = re.sub(r"//[^\n]*", "", text)
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return _TOKEN.findall(text)


class _Parser:
    def __init__(self, toks: list[str]):
        self.t = toks
        self.i = 0
        self.fd = descriptor_pb2.FileDescriptorProto(name="dfs.proto", syntax="proto3")
        self.pending: list[tuple[_FDP, str, list[str]]] = []  # (field, type name, scope)
        self.known_types: dict[str, str] = {}  # full name -> "message" | "enum"

    def peek(self) -> str:
        return self.t[self.i]

    def take(self, expect: str | None = None) -> str:
        tok = self.t[self.i]
        if expect is not None and tok != expect:
            raise SyntaxError(f"expected {expect!r}, got {tok!r} at token {self.i}")
        self.i += 1
        return tok

    def parse(self) -> descriptor_pb2.FileDescriptorProto:
        while self.i < len(self.t):
            tok = self.take()
            if tok == "syntax":
                self.take("=")
                self.take()
                self.take(";")
            elif tok == "package":
                self.fd.package = self.take()
                self.take(";")
            elif tok == "message":
                self._message(self.fd.message_type.add(), [])
            elif tok == "service":
                self._service()
            elif tok == "enum":
                self._enum(self.fd.enum_type.add(), [])
            else:
                raise SyntaxError(f"unexpected token {tok!r}")
        self._resolve()
        return self.fd

    def _full(self, scope: list[str], name: str) -> str:
        return "." + ".".join([self.fd.package, *scope, name])

    def _enum(self, ed: descriptor_pb2.EnumDescriptorProto, scope: list[str]) -> None:
        ed.name = self.take()
        self.known_types[self._full(scope, ed.name)] = "enum"
        self.take("{")
        while self.peek() != "}":
            name = self.take()
            self.take("=")
            num = int(self.take())
            self.take(";")
            ed.value.add(name=name, number=num)
        self.take("}")

    def _message(self, md: descriptor_pb2.DescriptorProto, scope: list[str]) -> None:
        md.name = self.take()
        inner = [*scope, md.name]
        self.known_types[self._full(scope, md.name)] = "message"
        self.take("{")
        while self.peek() != "}":
            tok = self.peek()
            if tok == "message":
                self.take()
                self._message(md.nested_type.add(), inner)
            elif tok == "enum":
                self.take()
                self._enum(md.enum_type.add(), inner)
            elif tok == "map":
                self.take()
                self.take("<")
                ktype = self.take()
                self.take(",")
                vtype = self.take()
                self.take(">")
                fname = self.take()
                self.take("=")
                num = int(self.take())
                self.take(";")
                entry = md.nested_type.add()
                entry.name = "".join(p.capitalize() for p in fname.split("_")) + "Entry"
                entry.options.map_entry = True
                self.known_types[self._full(inner, entry.name)] = "message"
                k = entry.field.add(name="key", number=1, label=_FDP.LABEL_OPTIONAL, json_name="key")
                v = entry.field.add(name="value", number=2, label=_FDP.LABEL_OPTIONAL, json_name="value")
                self._set_type(k, ktype, [*inner, entry.name])
                self._set_type(v, vtype, [*inner, entry.name])
                f = md.field.add(name=fname, number=num, label=_FDP.LABEL_REPEATED, json_name=fname)
                f.type = _FDP.TYPE_MESSAGE
                f.type_name = self._full(inner, entry.name)
            else:
                label = _FDP.LABEL_OPTIONAL
                if tok == "repeated":
                    self.take()
                    label = _FDP.LABEL_REPEATED
                ftype = self.take()
                fname = self.take()
                self.take("=")
                num = int(self.take())
                self.take(";")
                f = md.field.add(name=fname, number=num, label=label, json_name=fname)
                self._set_type(f, ftype, inner)
        self.take("}")

    def _set_type(self, f: _FDP, ftype: str, scope: list[str]) -> None:
        if ftype in _SCALARS:
            f.type = _SCALARS[ftype]
        else:
            self.pending.append((f, ftype, scope))

    def _resolve(self) -> None:
        for f, name, scope in self.pending:
            for depth in range(len(scope), -1, -1):
                cand = "." + ".".join([self.fd.package, *scope[:depth], name])
                if cand in self.known_types:
                    f.type_name = cand
                    f.type = _FDP.TYPE_ENUM if self.known_types[cand] == "enum" else _FDP.TYPE_MESSAGE
                    break
            else:
                raise SyntaxError(f"unknown type {name}")

    def _service(self) -> None:
        sd = self.fd.service.add()
        sd.name = self.take()
        self.take("{")
        while self.peek() != "}":
            self.take("rpc")
            m = sd.method.add(name=self.take())
            self.take("(")
            m.input_type = "." + self.fd.package + "." + self.take()
            self.take(")")
            self.take("returns")
            self.take("(")
            m.output_type = "." + self.fd.package + "." + self.take()
            self.take(")")
            if self.peek() == "{":
                self.take()
                self.take("}")
            else:
                self.take(";")
        self.take("}")


def _build():
    fdp = _Parser(_tokens(PROTO_PATH.read_text())).parse()
    pool = descriptor_pool.DescriptorPool()
    fd = pool.Add(fdp)
    fdesc = pool.FindFileByName(fdp.name)
    classes = {}
    for name in fdesc.message_types_by_name:
        classes[name] = message_factory.GetMessageClass(fdesc.message_types_by_name[name])
    services = {}
    for sname, sdesc in fdesc.services_by_name.items():
        services[sname] = [
            (m.name, classes[m.input_type.name], classes[m.output_type.name]) for m in sdesc.methods
        ]
    return fdp, fdesc, classes, services


FILE_DESCRIPTOR_PROTO, FILE_DESCRIPTOR, MESSAGES, SERVICES = _build()
PACKAGE = FILE_DESCRIPTOR_PROTO.package
globals().update(MESSAGES)


def method_path(service: str, method: str) -> str:
    return f"/{PACKAGE}.{service}/{method}"
