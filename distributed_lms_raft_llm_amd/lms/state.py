"""The replicated LMS state machine (C6/C7/C8 of SURVEY.md §2.0).

``LMSState.apply(index, command)`` is called for every committed Raft entry, in log order, on
every node.  The data layout is the reference's ``lms_data.json`` schema (``lms_server.py:44-49``,
SURVEY.md §2.4)::

    users            {username: {"password", "role"}}
    assignments      {student: [{"filename", "filepath": "uploads/<f>", "grade": null|str, "text"}]}
    grades           {}            (created by the reference's defaults, never used)
    course_materials [{"filename", "filepath", "instructor"}]
    queries          {student: [{"query", "answered": bool, "response": null|str}]}

Differences from the reference, all deliberate:

* committed JSON commands are actually applied (the reference's ``_apply_commits`` only parses
  a legacy space-separated form and silently drops every live entry, Appendix A.1);
* sessions are replicated (``Login``/``Logout`` log entries) so tokens survive a leader change;
* upload bytes travel in the log (``StoreBlob``), written atomically and idempotently under
  ``uploads/`` on every replica -- the reference streams them after commit to hard-coded IPs and
  its ``SendFile`` appends, so a retry duplicates bytes (Appendix A.10);
* ``lms_data.json`` is an export of the state written atomically after each applied batch (the
  Raft log + snapshot are the source of truth); it is imported once when a node starts with no
  Raft state, so an existing reference data file migrates.
"""
from __future__ import annotations

import base64
import copy
import hashlib
import json
import os
import threading

from . import commands

DATABASE_FILE = "lms_data.json"
UPLOAD_FOLDER = "uploads"


def default_data() -> dict:
    return {"users": {}, "assignments": {}, "grades": {}, "course_materials": [], "queries": {}}


def safe_filename(name: str) -> str:
    """Strip directories and control characters: upload names come from clients."""
    base = os.path.basename(name.replace("\\", "/")).strip()
    base = "".join(ch for ch in base if ch.isprintable() and ch not in '<>:"|?*')
    if base in ("", ".", ".."):
        base = "unnamed"
    return base[:255]


class BlobStore:
    """``uploads/<filename>`` files.  Writes are atomic (tmp + rename) and idempotent."""

    def __init__(self, root: str):
        self.root = root
        os.makedirs(os.path.join(root, UPLOAD_FOLDER), exist_ok=True)

    def relpath(self, filename: str) -> str:
        return os.path.join(UPLOAD_FOLDER, safe_filename(filename))

    def abspath(self, relpath: str) -> str:
        rel = os.path.normpath(relpath)
        if rel.startswith("..") or os.path.isabs(rel):
            rel = self.relpath(os.path.basename(relpath))
        return os.path.join(self.root, rel)

    def put(self, filename: str, data: bytes) -> str:
        rel = self.relpath(filename)
        path = self.abspath(rel)
        if os.path.exists(path):
            with open(path, "rb") as f:
                if hashlib.sha256(f.read()).digest() == hashlib.sha256(data).digest():
                    return rel
        tmp = f"{path}.tmp{os.getpid()}.{threading.get_ident()}"
        with open(tmp, "wb") as f:
            f.write(data)
        os.replace(tmp, path)
        return rel

    def get(self, relpath: str) -> bytes:
        try:
            with open(self.abspath(relpath), "rb") as f:
                return f.read()
        except FileNotFoundError:
            return b""

    def names(self) -> list[str]:
        d = os.path.join(self.root, UPLOAD_FOLDER)
        return sorted(n for n in os.listdir(d) if ".tmp" not in n)


class LMSState:
    def __init__(self, data_dir: str, export: bool = True):
        self.dir = data_dir
        os.makedirs(data_dir, exist_ok=True)
        self.blobs = BlobStore(data_dir)
        self.data = default_data()
        self.sessions: dict[str, dict] = {}  # token -> {"username", "role"}
        self.kv: dict[str, str] = {}
        self.applied_index = 0
        self.export_enabled = export
        self._dirty = False
        self.lock = threading.RLock()
        self.listeners = []  # callables(op, args) run after each apply (e.g. gate embedding cache)

    # ------------------------------------------------------------------ bootstrap / export
    def import_reference_file(self) -> bool:
        """Load an existing reference ``lms_data.json`` (used only when there is no Raft state)."""
        path = os.path.join(self.dir, DATABASE_FILE)
        if not os.path.exists(path):
            return False
        with open(path, encoding="utf-8") as f:
            loaded = json.load(f)
        base = default_data()
        base.update({k: v for k, v in loaded.items() if k in base})
        self.data = base
        return True

    def export(self, force: bool = False):
        if not self.export_enabled or (not self._dirty and not force):
            return
        path = os.path.join(self.dir, DATABASE_FILE)
        tmp = f"{path}.tmp{os.getpid()}"
        with self.lock:
            text = json.dumps(self.data, indent=2)
        with open(tmp, "w", encoding="utf-8") as f:
            f.write(text)
        os.replace(tmp, path)
        self._dirty = False

    # ------------------------------------------------------------------ snapshots
    def snapshot(self) -> str:
        with self.lock:
            blobs = {n: base64.b64encode(self.blobs.get(os.path.join(UPLOAD_FOLDER, n))).decode()
                     for n in self.blobs.names()}
            return json.dumps({"data": self.data, "sessions": self.sessions, "kv": self.kv,
                               "applied_index": self.applied_index, "blobs": blobs})

    def restore(self, snap: str):
        obj = json.loads(snap) if snap else {}
        with self.lock:
            self.data = obj.get("data", default_data())
            self.sessions = obj.get("sessions", {})
            self.kv = obj.get("kv", {})
            self.applied_index = obj.get("applied_index", 0)
            for name, b64 in obj.get("blobs", {}).items():
                self.blobs.put(name, base64.b64decode(b64))
            self._dirty = True

    # ------------------------------------------------------------------ apply
    def apply(self, index: int, command: str):
        try:
            op, args = commands.decode(command)
        except commands.BadCommand:
            return None
        with self.lock:
            self.applied_index = max(self.applied_index, index)
            fn = getattr(self, "_op_" + op, None)
            if fn is None:
                return None
            try:
                res = fn(*args)
            except TypeError:  # wrong arity from a foreign/legacy writer: ignore the entry
                return None
            if op not in ("NoOp", "SetVal"):
                self._dirty = True
        for cb in self.listeners:
            try:
                cb(op, args)
            except Exception:
                pass
        return res

    # reference operations ----------------------------------------------------------------
    def _op_Register(self, username, password, role):
        users = self.data.setdefault("users", {})
        if username in users:
            return False
        users[username] = {"password": password, "role": role}
        return True

    def _op_PostAssignment(self, student, filename, file_path, assignment_text):
        self.data.setdefault("assignments", {}).setdefault(student, []).append({
            "filename": filename, "filepath": self.blobs.relpath(filename), "grade": None, "text": assignment_text})
        return True

    def _op_PostCourseMaterial(self, instructor, filename, file_path):
        self.data.setdefault("course_materials", []).append({
            "filename": filename, "filepath": self.blobs.relpath(filename), "instructor": instructor})
        return True

    def _op_AskQuery(self, username, query):
        self.data.setdefault("queries", {}).setdefault(username, []).append(
            {"query": query, "answered": False, "response": None})
        return True

    def _op_RespondToQuery(self, instructor, student_id, response):
        for q in self.data.get("queries", {}).get(student_id, []):
            if not q["answered"]:
                q["response"] = response
                q["answered"] = True
                return True
        return False

    def _op_GradeAssignment(self, student, grade):
        items = self.data.get("assignments", {}).get(student)
        if not items:
            return False
        for a in items:
            a["grade"] = grade
        return True

    # extensions -------------------------------------------------------------------------
    def _op_NoOp(self):
        return True

    def _op_Login(self, username, token, role):
        self.sessions[token] = {"username": username, "role": role}
        return True

    def _op_Logout(self, token):
        return self.sessions.pop(token, None) is not None

    def _op_StoreBlob(self, filename, sha256, b64):
        data = base64.b64decode(b64)
        if hashlib.sha256(data).hexdigest() != sha256:
            return False
        self.blobs.put(filename, data)
        return True

    def _op_SetVal(self, key, value):
        self.kv[key] = value
        return True

    # ------------------------------------------------------------------ reads (callers hold no lock)
    def session(self, token: str) -> dict | None:
        with self.lock:
            s = self.sessions.get(token)
            if s is None:
                return None
            user = self.data["users"].get(s["username"])
            if user is None:
                return None
            return {"username": s["username"], "role": user["role"]}

    def read(self, fn):
        """Run ``fn(data)`` under the state lock; ``fn`` must copy out what it returns.  The read
        path of every RPC (no whole-state copies: state grows with every upload)."""
        with self.lock:
            return fn(self.data)

    def view(self) -> dict:
        """Deep copy of the whole state (tests / debugging only)."""
        with self.lock:
            return copy.deepcopy(self.data)
