"""The Raft log command format.

Every log entry is ``{"term": int, "command": str}`` and ``command`` is
``json.dumps({"operation": <op>, "args": [...]})`` -- exactly what the reference's live
``create_log_entry`` emits (``lms_server.py:335-340``).  The six reference operations keep their
names and argument orders:

=====================  ==============================================  =======================
operation              args (order)                                    proposed at (reference)
=====================  ==============================================  =======================
Register               [username, password, role]                      lms_server.py:749
PostAssignment         [student, filename, file_path, assignment_text] lms_server.py:921
PostCourseMaterial     [instructor, filename, file_path]               lms_server.py:902
AskQuery               [username, query]                               lms_server.py:932
RespondToQuery         [instructor, student_id, response]              lms_server.py:1017
GradeAssignment        [student, grade]                                lms_server.py:1191
=====================  ==============================================  =======================

Additional operations of this implementation (new ``operation`` values, format unchanged):
``NoOp`` (leader's first entry of a term), ``Login`` [username, token, role] / ``Logout``
[token] (sessions survive leader failover), ``PutBlob`` [filename, sha256, size] (an upload the
leader pre-replicated to a majority over ``FileTransferService.SendFile``: lms/blobs.py), the
legacy ``StoreBlob`` [filename, sha256, base64] (still applied when replaying old logs) and
``SetVal`` [key, value] (the RaftService debug KV API).

An optional top-level ``"rid"`` (client request id) makes a write idempotent: the state machine
applies a given rid once and answers retries with the first result (a client that retries a
write after a leader failover must not post the same assignment twice).  An optional top-level
``"sha256"`` on ``PostAssignment`` / ``PostCourseMaterial`` names the entry's own upload (its
CAS object), so two same-named uploads keep their own bytes; ``args`` stay the reference's.

``decode`` also accepts the reference's shadowed legacy encoder (``lms_server.py:317-333``):
``Op arg1 "multi word arg" ...`` (shlex quoting).
"""
from __future__ import annotations

import json
import shlex

REFERENCE_OPS = {
    "Register": 3,
    "PostAssignment": 4,
    "PostCourseMaterial": 3,
    "AskQuery": 2,
    "RespondToQuery": 3,
    "GradeAssignment": 2,
}
EXTRA_OPS = {"NoOp": 0, "Login": 3, "Logout": 1, "PutBlob": 3, "StoreBlob": 3, "SetVal": 2}
ALL_OPS = {**REFERENCE_OPS, **EXTRA_OPS}


class BadCommand(ValueError):
    pass


META_KEYS = ("sha256",)


def encode(operation: str, args: list, rid: str | None = None, meta: dict | None = None) -> str:
    if operation not in ALL_OPS:
        raise BadCommand(f"unknown operation {operation!r}")
    if len(args) != ALL_OPS[operation]:
        raise BadCommand(f"{operation} takes {ALL_OPS[operation]} args, got {len(args)}")
    obj = {"operation": operation, "args": list(args)}
    if rid:
        obj["rid"] = str(rid)
    for k, v in (meta or {}).items():
        if k not in META_KEYS:
            raise BadCommand(f"unknown command field {k!r}")
        obj[k] = v
    return json.dumps(obj)


def decode_meta(command: str) -> dict:
    """The optional top-level fields (``META_KEYS``) of a JSON command ({} for the legacy form)."""
    s = command.strip()
    if not s.startswith("{"):
        return {}
    try:
        obj = json.loads(s)
    except ValueError:
        return {}
    return {k: obj[k] for k in META_KEYS if k in obj}


def decode(command: str) -> tuple[str, list]:
    op, args, _ = decode_full(command)
    return op, args


def decode_full(command: str) -> tuple[str, list, str | None]:
    """(operation, args, request id or None)."""
    s = command.strip()
    if s.startswith("{"):
        try:
            obj = json.loads(s)
        except ValueError as e:
            raise BadCommand(f"malformed JSON command: {e}") from e
        op, args, rid = obj.get("operation"), obj.get("args", []), obj.get("rid")
        if not isinstance(op, str) or not isinstance(args, list):
            raise BadCommand("command must carry a string 'operation' and a list 'args'")
        return op, args, (str(rid) if rid else None)
    try:
        parts = shlex.split(s)
    except ValueError as e:
        raise BadCommand(f"malformed legacy command: {e}") from e
    if not parts:
        raise BadCommand("empty command")
    return parts[0], parts[1:], None
