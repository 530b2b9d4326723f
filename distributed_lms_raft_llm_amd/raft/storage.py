"""Durable Raft state: ``current_term``/``voted_for``, the log and snapshots.

The reference keeps all of it in memory (``lms_server.py:124-140``): a restarted node comes back
with term 0 and an empty log.  Here:

* ``raft_meta.json``     -- ``{"current_term", "voted_for"}``, replaced atomically (write, fsync,
  rename) before any vote or term change is acted on;
* ``raft_log.jsonl``     -- append-only, one ``{"term": int, "command": str, "index": int}`` object
  per line: the reference's ``LogEntry`` / log-entry format (``lms.proto:180-183``,
  ``lms_server.py:335-340``) plus the entry's own log index, so the file is self-describing -- a
  crash between replacing the snapshot and rewriting the log (compaction, InstallSnapshot) leaves
  an OLD log whose entries still carry their true indices; loading drops those at or below the
  snapshot instead of shifting every entry to the wrong index.  A conflicting suffix is cut with
  ``truncate(2)`` at the entry's byte offset;
* ``raft_snapshot.json`` -- ``{"last_index", "last_term", "data"}`` where ``data`` is the state
  machine's JSON snapshot (the ``lms_data.json`` schema); compaction rewrites the log without the
  snapshotted prefix.

``MemoryStorage`` has the same interface for the deterministic tests.
"""
from __future__ import annotations

import json
import os
import threading

from .core import Entry


class MemoryStorage:
    def __init__(self):
        self._term, self._voted = 0, None
        self._log: list[Entry] = []
        self._snap_index, self._snap_term, self._snap_data = 0, 0, ""

    # meta
    def load_meta(self):
        return self._term, self._voted

    def save_meta(self, term: int, voted_for):
        self._term, self._voted = term, voted_for

    # log
    def last_index(self) -> int:
        return self._snap_index + len(self._log)

    def term_at(self, i: int) -> int:
        if i == self._snap_index:
            return self._snap_term
        if i < self._snap_index or i > self.last_index() or i <= 0:
            return 0
        return self._log[i - self._snap_index - 1].term

    def entries(self, lo: int, hi: int, max_bytes: int | None = None) -> list[Entry]:
        lo = max(lo, self._snap_index + 1)
        hi = min(hi, self.last_index() + 1)
        out = self._log[lo - self._snap_index - 1: hi - self._snap_index - 1]
        if max_bytes is not None and out:
            total, cut = 0, 0
            for e in out:
                total += len(e.command) + 16
                if total > max_bytes and cut > 0:
                    break
                cut += 1
            out = out[:cut]
        return list(out)

    def append(self, entries: list[Entry]):
        self._log.extend(Entry(e.term, e.command) for e in entries)

    def truncate_from(self, i: int):
        if i <= self._snap_index:
            raise ValueError("cannot truncate into the snapshot")
        del self._log[i - self._snap_index - 1:]

    # snapshots
    def snapshot_meta(self):
        return self._snap_index, self._snap_term

    def snapshot_data(self) -> str:
        return self._snap_data

    def compact(self, index: int, term: int, data: str):
        if index <= self._snap_index:
            return
        del self._log[: index - self._snap_index]
        self._snap_index, self._snap_term, self._snap_data = index, term, data

    def install_snapshot(self, index: int, term: int, data: str):
        if self.term_at(index) == term and index <= self.last_index():
            del self._log[: index - self._snap_index]  # keep the matching suffix
        else:
            self._log = []
        self._snap_index, self._snap_term, self._snap_data = index, term, data


def _atomic_write(path: str, text: str, fsync: bool):
    tmp = f"{path}.tmp{os.getpid()}.{threading.get_ident()}"
    with open(tmp, "w", encoding="utf-8") as f:
        f.write(text)
        f.flush()
        if fsync:
            os.fsync(f.fileno())
    os.replace(tmp, path)


class FileStorage(MemoryStorage):
    """MemoryStorage mirrored to disk under ``data_dir``."""

    META, LOG, SNAP = "raft_meta.json", "raft_log.jsonl", "raft_snapshot.json"

    def __init__(self, data_dir: str, fsync: bool = True):
        super().__init__()
        self.dir = data_dir
        self.fsync = fsync
        os.makedirs(data_dir, exist_ok=True)
        self._offsets: list[int] = []  # byte offset of each in-memory entry's line
        self._load()
        self._fh = open(self._path(self.LOG), "ab")

    def _path(self, name: str) -> str:
        return os.path.join(self.dir, name)

    def _load(self):
        mp = self._path(self.META)
        if os.path.exists(mp):
            with open(mp, encoding="utf-8") as f:
                m = json.load(f)
            self._term, self._voted = int(m.get("current_term", 0)), m.get("voted_for")
        sp = self._path(self.SNAP)
        if os.path.exists(sp):
            with open(sp, encoding="utf-8") as f:
                s = json.load(f)
            self._snap_index, self._snap_term, self._snap_data = int(s["last_index"]), int(s["last_term"]), s["data"]
        lp = self._path(self.LOG)
        if os.path.exists(lp):
            good, stale = 0, False
            with open(lp, "rb") as f:
                off = 0
                for line in f:
                    try:
                        obj = json.loads(line)
                        e = Entry(int(obj["term"]), str(obj["command"]))
                    except (ValueError, KeyError):
                        break  # torn tail from a crash mid-append: drop it
                    if not line.endswith(b"\n"):
                        break
                    expect = self._snap_index + len(self._log) + 1
                    idx = int(obj.get("index", expect))  # round-1 logs carry no index: sequential
                    if idx <= self._snap_index:
                        stale = True  # already inside the snapshot (crash mid-compaction)
                        off += len(line)
                        continue
                    if idx != expect:
                        break  # a gap cannot be trusted: keep the consistent prefix only
                    self._log.append(e)
                    self._offsets.append(off)
                    off += len(line)
                    good = off
            if stale:
                self._rewrite_log(reopen=False)  # drop the snapshotted prefix from the file too
            elif good != os.path.getsize(lp):
                os.truncate(lp, good)

    def save_meta(self, term: int, voted_for):
        super().save_meta(term, voted_for)
        _atomic_write(self._path(self.META), json.dumps({"current_term": term, "voted_for": voted_for}), self.fsync)

    def append(self, entries: list[Entry]):
        if not entries:
            return
        off = self._fh.tell()
        buf = bytearray()
        first = self.last_index() + 1
        for k, e in enumerate(entries):
            line = (json.dumps({"term": e.term, "command": e.command, "index": first + k}) + "\n").encode("utf-8")
            self._offsets.append(off + len(buf))
            buf += line
        self._fh.write(buf)
        self._fh.flush()
        if self.fsync:
            os.fsync(self._fh.fileno())
        super().append(entries)

    def truncate_from(self, i: int):
        k = i - self._snap_index - 1
        if k < 0:
            raise ValueError("cannot truncate into the snapshot")
        if k < len(self._offsets):
            cut = self._offsets[k]
            self._fh.flush()
            os.truncate(self._path(self.LOG), cut)
            self._fh.seek(0, os.SEEK_END)
            del self._offsets[k:]
        super().truncate_from(i)

    def _rewrite_log(self, reopen: bool = True):
        if reopen:
            self._fh.close()
        lines, self._offsets, off = [], [], 0
        for k, e in enumerate(self._log):
            line = json.dumps({"term": e.term, "command": e.command, "index": self._snap_index + 1 + k}) + "\n"
            self._offsets.append(off)
            off += len(line.encode("utf-8"))
            lines.append(line)
        _atomic_write(self._path(self.LOG), "".join(lines), self.fsync)
        if reopen:
            self._fh = open(self._path(self.LOG), "ab")

    def _save_snapshot(self):
        _atomic_write(self._path(self.SNAP), json.dumps({"last_index": self._snap_index, "last_term": self._snap_term,
                                                         "data": self._snap_data}), self.fsync)

    def compact(self, index: int, term: int, data: str):
        if index <= self._snap_index:
            return
        super().compact(index, term, data)
        self._save_snapshot()
        self._rewrite_log()

    def install_snapshot(self, index: int, term: int, data: str):
        super().install_snapshot(index, term, data)
        self._save_snapshot()
        self._rewrite_log()

    def close(self):
        try:
            self._fh.close()
        except Exception:
            pass
