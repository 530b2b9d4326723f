"""The ``lms.proto`` wire contract, defined as data and compiled at import time.

The reference ships ``lms.proto`` plus ``protoc``-generated ``lms_pb2*.py``
(``lms.proto:1-248``).  This box has no ``protoc``/``grpc_tools``, so the schema is declared
here as a table and turned into a ``FileDescriptorProto`` at runtime.  Package, file name,
message names, field names, numbers, types and labels, and the four services with their
method names and streaming shapes are identical to the reference,
which is what makes the reference's generated client stubs -- and so ``lms_gui_final.py`` --
interoperate unchanged.  ``render_proto()`` emits equivalent ``.proto`` text for users who
want to run ``protoc`` elsewhere.
"""
from __future__ import annotations

from google.protobuf import descriptor_pb2

PACKAGE = "lms"
FILE_NAME = "lms.proto"

# field: (name, number, type, label) with type in {"string","bytes","bool","int32"} or a message
# name, label "" (singular) or "repeated".
MESSAGES: list[tuple[str, list[tuple]]] = [
    ("RegisterRequest", [("username", 1, "string"), ("password", 2, "string"), ("role", 3, "string")]),
    ("RegisterResponse", [("success", 1, "bool"), ("message", 2, "string")]),
    ("LoginRequest", [("username", 1, "string"), ("password", 2, "string")]),
    ("LoginResponse", [("success", 1, "bool"), ("token", 2, "string"), ("role", 3, "string")]),
    ("LogoutRequest", [("token", 1, "string")]),
    ("LogoutResponse", [("success", 1, "bool")]),
    ("PostRequest", [("token", 1, "string"), ("type", 2, "string"), ("file", 3, "bytes"), ("filename", 4, "string"),
                     ("data", 5, "string"), ("studentId", 6, "string")]),
    ("PostResponse", [("success", 1, "bool")]),
    ("GetRequest", [("token", 1, "string"), ("type", 2, "string"), ("studentId", 3, "string")]),
    ("DataEntry", [("id", 1, "string"), ("filename", 2, "string"), ("file", 3, "bytes"), ("data", 4, "string"),
                   ("instructor", 5, "string")]),
    ("GetResponse", [("success", 1, "bool"), ("message", 2, "string"), ("entries", 3, "DataEntry", "repeated")]),
    ("GradeRequest", [("token", 1, "string"), ("studentId", 2, "string"), ("grade", 3, "string")]),
    ("GradeResponse", [("success", 1, "bool"), ("message", 2, "string")]),
    ("GetGradeRequest", [("token", 1, "string")]),
    ("GetGradeResponse", [("success", 1, "bool"), ("grade", 2, "string")]),
    ("QueryRequest", [("token", 1, "string"), ("query", 2, "string")]),
    ("QueryResponse", [("success", 1, "bool"), ("response", 2, "string")]),
    ("FileChunk", [("content", 1, "bytes"), ("destination_path", 2, "string")]),
    ("FileTransferResponse", [("status", 1, "string")]),
    ("ReplicateDataRequest", [("type", 1, "string"), ("username", 2, "string"), ("instructor", 3, "string"),
                              ("filename", 4, "string"), ("file_content", 5, "bytes"), ("text", 6, "string")]),
    ("ReplicateDataResponse", [("success", 1, "bool")]),
    ("TermCandIDPair", [("term", 1, "int32"), ("candidateID", 2, "int32")]),
    ("TermResultPair", [("term", 1, "int32"), ("verdict", 2, "bool")]),
    ("LogEntry", [("term", 1, "int32"), ("command", 2, "string")]),
    ("RequestVoteRequest", [("candidate", 1, "TermCandIDPair"), ("lastLogIndex", 2, "int32"),
                            ("lastLogTerm", 3, "int32")]),
    ("RequestVoteResponse", [("result", 1, "TermResultPair")]),
    ("AppendEntriesRequest", [("leader", 1, "TermLeaderIDPair"), ("prevLogIndex", 2, "int32"),
                              ("prevLogTerm", 3, "int32"), ("entries", 4, "LogEntry", "repeated"),
                              ("leaderCommit", 5, "int32")]),
    ("AppendEntriesResponse", [("result", 1, "TermResultPair"), ("term", 2, "int32"), ("success", 3, "bool")]),
    ("SetValRequest", [("key", 1, "string"), ("value", 2, "string")]),
    ("SetValResponse", [("verdict", 1, "bool")]),
    ("GetValRequest", [("key", 1, "string")]),
    ("GetValResponse", [("verdict", 1, "bool"), ("value", 2, "string")]),
    ("GetLeaderRequest", []),
    ("GetLeaderResponse", [("nodeId", 1, "int32"), ("nodeAddress", 2, "string")]),
    ("LeaderResponse", [("leader_id", 1, "int32")]),
    ("TermLeaderIDPair", [("leaderID", 1, "int32"), ("term", 2, "int32")]),
    ("Empty", []),
]

# (method, request, response, client_streaming)
SERVICES: list[tuple[str, list[tuple]]] = [
    ("LMS", [
        ("Register", "RegisterRequest", "RegisterResponse", False),
        ("Login", "LoginRequest", "LoginResponse", False),
        ("Logout", "LogoutRequest", "LogoutResponse", False),
        ("Post", "PostRequest", "PostResponse", False),
        ("Get", "GetRequest", "GetResponse", False),
        ("GradeAssignment", "GradeRequest", "GradeResponse", False),
        ("GetGrade", "GetGradeRequest", "GetGradeResponse", False),
        ("GetLLMAnswer", "QueryRequest", "QueryResponse", False),
        ("GetUnansweredQueries", "GetRequest", "GetResponse", False),
        ("RespondToQuery", "PostRequest", "PostResponse", False),
        ("GetInstructorResponse", "GetRequest", "GetResponse", False),
        ("WhoIsLeader", "Empty", "LeaderResponse", False),
    ]),
    ("Tutoring", [
        ("GetLLMAnswer", "QueryRequest", "QueryResponse", False),
    ]),
    ("RaftService", [
        ("RequestVote", "RequestVoteRequest", "RequestVoteResponse", False),
        ("AppendEntries", "AppendEntriesRequest", "AppendEntriesResponse", False),
        ("SetVal", "SetValRequest", "SetValResponse", False),
        ("GetVal", "GetValRequest", "GetValResponse", False),
        ("GetLeader", "GetLeaderRequest", "GetLeaderResponse", False),
        ("WhoIsLeader", "Empty", "LeaderResponse", False),
    ]),
    ("FileTransferService", [
        ("SendFile", "FileChunk", "FileTransferResponse", True),
        ("ReplicateData", "ReplicateDataRequest", "ReplicateDataResponse", False),
    ]),
]

_SCALARS = {
    "string": descriptor_pb2.FieldDescriptorProto.TYPE_STRING,
    "bytes": descriptor_pb2.FieldDescriptorProto.TYPE_BYTES,
    "bool": descriptor_pb2.FieldDescriptorProto.TYPE_BOOL,
    "int32": descriptor_pb2.FieldDescriptorProto.TYPE_INT32,
}


def _json_name(name: str) -> str:
    parts = name.split("_")
    return parts[0] + "".join(p[:1].upper() + p[1:] for p in parts[1:])


def build_file_descriptor_proto() -> descriptor_pb2.FileDescriptorProto:
    fdp = descriptor_pb2.FileDescriptorProto(name=FILE_NAME, package=PACKAGE, syntax="proto3")
    for mname, fields in MESSAGES:
        m = fdp.message_type.add(name=mname)
        for spec in fields:
            fname, number, ftype = spec[0], spec[1], spec[2]
            label = spec[3] if len(spec) > 3 else ""
            f = m.field.add(name=fname, number=number, json_name=_json_name(fname))
            f.label = (descriptor_pb2.FieldDescriptorProto.LABEL_REPEATED if label == "repeated"
                       else descriptor_pb2.FieldDescriptorProto.LABEL_OPTIONAL)
            if ftype in _SCALARS:
                f.type = _SCALARS[ftype]
            else:
                f.type = descriptor_pb2.FieldDescriptorProto.TYPE_MESSAGE
                f.type_name = f".{PACKAGE}.{ftype}"
    for sname, methods in SERVICES:
        s = fdp.service.add(name=sname)
        for meth, req, resp, cstream in methods:
            md = s.method.add(name=meth, input_type=f".{PACKAGE}.{req}", output_type=f".{PACKAGE}.{resp}")
            if cstream:
                md.client_streaming = True
    return fdp


def render_proto() -> str:
    """Equivalent ``.proto`` source text (for use with an external ``protoc``)."""
    lines = ['syntax = "proto3";', "", f"package {PACKAGE};", ""]
    for mname, fields in MESSAGES:
        lines.append(f"message {mname} {{")
        for spec in fields:
            rep = "repeated " if len(spec) > 3 and spec[3] == "repeated" else ""
            lines.append(f"  {rep}{spec[2]} {spec[0]} = {spec[1]};")
        lines.append("}")
        lines.append("")
    for sname, methods in SERVICES:
        lines.append(f"service {sname} {{")
        for meth, req, resp, cstream in methods:
            lines.append(f"  rpc {meth}({'stream ' if cstream else ''}{req}) returns ({resp});")
        lines.append("}")
        lines.append("")
    return "\n".join(lines)
