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
* uploads are content-addressed and pre-replicated to a majority over ``SendFile`` before the
  (tiny) ``PutBlob`` entry commits (lms/blobs.py) -- the reference streams them after commit to
  hard-coded IPs and its ``SendFile`` appends, so a retry duplicates bytes (Appendix A.10); the
  replicated ``blob_index`` maps each ``uploads/<f>`` to its sha256 and a replica that misses an
  object pulls it from a peer;
* writes carrying a client request id (``rid``) apply once; a retry gets the first result;
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
import logging
import threading
from collections import OrderedDict

from . import commands
from .blobs import UPLOAD_FOLDER, BlobStore, safe_filename  # noqa: F401  (re-exported)

log = logging.getLogger("dlms.lms.state")

DATABASE_FILE = "lms_data.json"
DEDUPE_CAP = 20000  # client request ids remembered (oldest evicted first, identically on every replica)


def default_data() -> dict:
    return {"users": {}, "assignments": {}, "grades": {}, "course_materials": [], "queries": {}}


class LMSState:
    def __init__(self, data_dir: str, export: bool = True):
        self.dir = data_dir
        os.makedirs(data_dir, exist_ok=True)
        self.blobs = BlobStore(data_dir)
        self.data = default_data()
        self.sessions: dict[str, dict] = {}  # token -> {"username", "role"}
        self.kv: dict[str, str] = {}
        self.blob_index: dict[str, str] = {}  # "uploads/<f>" -> sha256 of its CAS object
        self.dedupe: OrderedDict[str, object] = OrderedDict()  # client request id -> first result
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
        """The replicated state as JSON -- blob BYTES are not included (``blob_index`` names each
        upload's CAS object; a restoring replica pulls what it lacks from its peers)."""
        with self.lock:
            snap = json.dumps({"data": self.data, "sessions": self.sessions, "kv": self.kv,
                               "applied_index": self.applied_index, "blob_index": self.blob_index,
                               "dedupe": list(self.dedupe.items())})
        # the log prefix this snapshot replaces is the last thing that could name an object the
        # state no longer references: collect those CAS objects now (off the caller's thread)
        refs = self.referenced_blobs()
        threading.Thread(target=self._gc, args=(refs,), daemon=True, name="blob-gc").start()
        return snap

    gc_grace_s = 600.0  # unreferenced objects younger than this survive (uploads in flight)

    def _gc(self, refs: set[str]):
        try:
            n = self.blobs.gc(refs, self.gc_grace_s, live_refs=self.referenced_blobs)
            if n:
                log.info("blob gc: removed %d unreferenced object(s)", n)
        except OSError as e:
            log.warning("blob gc failed: %s", e)

    def restore(self, snap: str):
        obj = json.loads(snap) if snap else {}
        with self.lock:
            self.data = obj.get("data", default_data())
            self.sessions = obj.get("sessions", {})
            self.kv = obj.get("kv", {})
            self.applied_index = obj.get("applied_index", 0)
            self.blob_index = dict(obj.get("blob_index", {}))
            self.dedupe = OrderedDict((k, v) for k, v in obj.get("dedupe", []))
            for name, b64 in obj.get("blobs", {}).items():  # snapshots of the round-1 format
                rel = self.blobs.put(name, base64.b64decode(b64))
                self.blob_index.setdefault(rel, hashlib.sha256(base64.b64decode(b64)).hexdigest())
            index = dict(self.blob_index)
            self._dirty = True
        for rel, sha in index.items():
            self._materialize(rel, sha)

    def _materialize(self, rel: str, sha: str):
        if self.blobs.materialize(rel, sha):
            return
        if self.blobs.fetcher is not None:  # missed the leader's push: pull it in the background
            self.blobs.fetcher.fetch_async(sha, then=lambda: self.blobs.materialize(rel, sha))

    def rid_result(self, rid: str | None):
        """(already applied?, its result) for a client request id."""
        if not rid:
            return False, None
        with self.lock:
            if rid in self.dedupe:
                return True, self.dedupe[rid]
        return False, None

    def blob_sha(self, relpath: str) -> str | None:
        with self.lock:
            return self.blob_index.get(relpath)

    def read_blob(self, relpath: str, sha: str | None = None) -> bytes:
        """An upload's bytes (fetched from a peer first if this replica does not hold them):
        by the entry's own sha when it has one, else the latest upload under that name."""
        if sha:
            return self.blobs.get_sha(sha, relpath)
        return self.blobs.get(relpath, self.blob_sha(relpath))

    def referenced_blobs(self) -> set[str]:
        """Every CAS object the replicated state still points at (snapshot-time GC)."""
        with self.lock:
            refs = set(self.blob_index.values())
            for items in self.data.get("assignments", {}).values():
                refs.update(a["sha256"] for a in items if a.get("sha256"))
            refs.update(m["sha256"] for m in self.data.get("course_materials", []) if m.get("sha256"))
        return refs

    # ------------------------------------------------------------------ apply
    def apply(self, index: int, command: str):
        try:
            op, args, rid = commands.decode_full(command)
        except commands.BadCommand:
            return None
        with self.lock:
            self.applied_index = max(self.applied_index, index)
            if rid is not None and rid in self.dedupe:
                return self.dedupe[rid]  # a retried write: applied once, same answer
            fn = getattr(self, "_op_" + op, None)
            if fn is None:
                return None
            meta = commands.decode_meta(command) if op in ("PostAssignment", "PostCourseMaterial") else {}
            try:
                res = fn(*args, **meta)
            except TypeError:  # wrong arity from a foreign/legacy writer: ignore the entry
                return None
            if rid is not None:
                self.dedupe[rid] = res
                while len(self.dedupe) > DEDUPE_CAP:
                    self.dedupe.popitem(last=False)
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

    # (the reference's argument order; ``sha256`` -- the command's top-level field, lms/commands.py
    # -- keys the entry to ITS upload, so a later same-named upload does not change its download)
    def _op_PostAssignment(self, student, filename, file_path, assignment_text, sha256=None):
        rel = self.blobs.relpath(filename)
        entry = {"filename": filename, "filepath": rel, "grade": None, "text": assignment_text}
        sha = sha256 if isinstance(sha256, str) and len(sha256) == 64 else self.blob_index.get(rel)
        if sha:
            entry["sha256"] = sha
        self.data.setdefault("assignments", {}).setdefault(student, []).append(entry)
        return True

    def _op_PostCourseMaterial(self, instructor, filename, file_path, sha256=None):
        rel = self.blobs.relpath(filename)
        entry = {"filename": filename, "filepath": rel, "instructor": instructor}
        sha = sha256 if isinstance(sha256, str) and len(sha256) == 64 else self.blob_index.get(rel)
        if sha:
            entry["sha256"] = sha
        self.data.setdefault("course_materials", []).append(entry)
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

    def _op_PutBlob(self, filename, sha256, size):
        """An upload pre-replicated to a majority (lms/blobs.py): record it, and link it into
        ``uploads/`` here -- or pull it from a peer if this replica missed the push."""
        if not isinstance(sha256, str) or len(sha256) != 64:
            return False
        rel = self.blobs.relpath(filename)
        self.blob_index[rel] = sha256
        self._materialize(rel, sha256)
        return True

    def _op_StoreBlob(self, filename, sha256, b64):  # round-1 log entries (bytes inside the entry)
        data = base64.b64decode(b64)
        if hashlib.sha256(data).hexdigest() != sha256:
            return False
        self.blob_index[self.blobs.put(filename, data)] = sha256
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
