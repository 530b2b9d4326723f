"""Upload storage and replication (C8 of SURVEY.md §2.0), designed for multi-MB PDFs.

The reference writes the upload on the leader, proposes a log entry, and only after commit streams
the file in 1 MiB ``FileChunk``s to hard-coded follower IPs (``lms_server.py:1462-1492``; the
receiver appends, so a retry duplicates bytes, ``:1496-1521``).  Round 1 of this framework put the
whole base64 file inside one Raft entry instead, which a 40 MiB upload turned into a lost quorum.

Here uploads are **content-addressed and pre-replicated**:

* ``BlobStore``: ``cas/<sha256>`` holds the bytes (written to a temp file chunk by chunk, verified
  against the hash, renamed into place -- idempotent); ``uploads/<filename>`` is the reference's
  path layout, materialised as a hard link (or copy) of the CAS object;
* ``BlobReplicator`` (leader): before proposing, streams the file to every follower over the
  reference's own ``FileTransferService.SendFile`` (1 MiB ``FileChunk``s, ``destination_path =
  "cas/<sha256>"``) and waits until a MAJORITY of the cluster (itself included) holds it; the log
  then carries only ``PutBlob [filename, sha256, size]`` -- a few bytes, never a multi-MB entry;
* ``BlobFetcher`` (any node): a replica that missed the push (down, partitioned, restored from a
  snapshot) pulls the object from a peer over ``lmsinternal.Blob/Fetch`` (server-streaming 1 MiB
  chunks) -- a majority holds every committed blob, so some live peer always has it.

Snapshots therefore carry the ``filename -> sha256`` index, not the bytes.
"""
from __future__ import annotations

import hashlib
import logging
import os
import threading
import time
from concurrent.futures import ThreadPoolExecutor

import grpc

log = logging.getLogger("dlms.blobs")

UPLOAD_FOLDER = "uploads"
CAS_FOLDER = "cas"
CHUNK = 1 << 20  # 1 MiB, the reference's FileChunk size (lms_server.py:1467)
FETCH_METHOD = "/lmsinternal.Blob/Fetch"


def safe_filename(name: str) -> str:
    """Strip directories and control characters: upload names come from clients."""
    base = os.path.basename(name.replace("\\", "/")).strip()
    base = "".join(ch for ch in base if ch.isprintable() and ch not in '<>:"|?*')
    if base in ("", ".", ".."):
        base = "unnamed"
    return base[:255]


def is_sha256(s: str) -> bool:
    return len(s) == 64 and all(c in "0123456789abcdef" for c in s)


class BlobStore:
    """``uploads/<filename>`` (reference layout) backed by ``cas/<sha256>`` objects."""

    def __init__(self, root: str):
        self.root = root
        os.makedirs(os.path.join(root, UPLOAD_FOLDER), exist_ok=True)
        os.makedirs(os.path.join(root, CAS_FOLDER), exist_ok=True)
        self.fetcher = None  # BlobFetcher: pulls objects this replica is missing
        self._gc_lock = threading.Lock()  # _touch vs the GC's last re-check + unlink

    # ---------------------------------------------------------------- uploads/ (reference layout)
    def relpath(self, filename: str) -> str:
        return os.path.join(UPLOAD_FOLDER, safe_filename(filename))

    def abspath(self, relpath: str) -> str:
        rel = os.path.normpath(relpath)
        if rel.startswith("..") or os.path.isabs(rel):
            rel = self.relpath(os.path.basename(relpath))
        return os.path.join(self.root, rel)

    def names(self) -> list[str]:
        d = os.path.join(self.root, UPLOAD_FOLDER)
        return sorted(n for n in os.listdir(d) if ".tmp" not in n)

    def get(self, relpath: str, sha: str | None = None, fetch_timeout: float = 30.0) -> bytes:
        """Bytes of an upload; a replica that does not hold the object yet fetches it first."""
        path = self.abspath(relpath)
        try:
            with open(path, "rb") as f:
                return f.read()
        except FileNotFoundError:
            pass
        if sha and self.fetcher is not None and self.fetcher.fetch(sha, timeout=fetch_timeout):
            self.materialize(relpath, sha)
            try:
                with open(path, "rb") as f:
                    return f.read()
            except FileNotFoundError:
                pass
        return b""

    def put(self, filename: str, data: bytes) -> str:
        """Store ``data`` under ``uploads/<filename>`` (and its CAS object); returns the relpath."""
        sha = self.put_bytes(data)
        rel = self.relpath(filename)
        self.materialize(rel, sha)
        return rel

    def materialize(self, relpath: str, sha: str) -> bool:
        """Point ``uploads/<name>`` at the CAS object (atomic replace; no-op if already identical)."""
        src = self.cas_path(sha)
        if not os.path.exists(src):
            return False
        dst = self.abspath(relpath)
        tmp = f"{dst}.tmp{os.getpid()}.{threading.get_ident()}"
        try:
            if os.path.exists(dst) and os.path.samefile(src, dst):
                return True
        except OSError:
            pass
        try:
            os.link(src, tmp)
        except OSError:
            with open(src, "rb") as fi, open(tmp, "wb") as fo:
                while True:
                    b = fi.read(CHUNK)
                    if not b:
                        break
                    fo.write(b)
        os.replace(tmp, dst)
        return True

    # ---------------------------------------------------------------- cas/ (content addressed)
    def cas_path(self, sha: str) -> str:
        if not is_sha256(sha):
            raise ValueError(f"not a sha256: {sha!r}")
        return os.path.join(self.root, CAS_FOLDER, sha)

    def has(self, sha: str) -> bool:
        return is_sha256(sha) and os.path.exists(self.cas_path(sha))

    def put_bytes(self, data: bytes) -> str:
        sha = hashlib.sha256(data).hexdigest()
        if not self._touch(sha):
            self.put_chunks(sha, [data])
        return sha

    def _touch(self, sha: str) -> bool:
        """Refresh an existing object's mtime (False if absent): an upload of content that is
        already here counts as a fresh upload for the GC's grace period -- otherwise a stale
        unreferenced object re-uploaded just before a GC pass could be deleted under a PutBlob
        that is about to commit a reference to it."""
        with self._gc_lock:  # never between the GC's last mtime check and its unlink
            try:
                os.utime(self.cas_path(sha))
                return True
            except FileNotFoundError:
                return False

    def get_sha(self, sha: str, relpath: str | None = None, fetch_timeout: float = 30.0) -> bytes:
        """Bytes of CAS object ``sha`` (an entry's own upload: two same-named uploads keep their
        own bytes), pulled from a peer if this replica does not hold it; ``relpath`` is the
        fallback for entries recorded before uploads carried their sha."""
        if is_sha256(sha):
            for attempt in range(2):
                try:
                    with open(self.cas_path(sha), "rb") as f:
                        return f.read()
                except FileNotFoundError:
                    if attempt or self.fetcher is None or not self.fetcher.fetch(sha, timeout=fetch_timeout):
                        break
        return self.get(relpath, sha) if relpath else b""

    def gc(self, referenced: set[str], grace_s: float = 600.0, live_refs=None) -> int:
        """Delete CAS objects no replicated entry references any more (snapshot time).  Objects
        younger than ``grace_s`` survive: a pre-replicated upload whose PutBlob has not committed
        yet is unreferenced but live (re-uploads refresh the mtime, ``_touch``).  The scan runs in
        the background while entries keep committing, so the candidates are re-checked against
        ``live_refs()`` (the live state's reference set, built ONCE per pass, not per candidate)
        and each one's mtime is read again right before its unlink -- that re-check and the unlink
        hold ``_gc_lock``, which ``_touch`` holds too, so a re-upload either lands before the
        re-check (the object survives) or after the unlink (``_touch`` sees it absent and the
        upload writes it again).  ``uploads/<name>`` links keep their own inode.
        Returns the number of objects removed."""
        d = os.path.join(self.root, CAS_FOLDER)
        now = time.time()
        cands = []
        for name in os.listdir(d):
            if not is_sha256(name) or name in referenced:
                continue
            try:
                if now - os.path.getmtime(os.path.join(d, name)) >= grace_s:
                    cands.append(name)
            except FileNotFoundError:
                pass
        if not cands:
            return 0
        live = live_refs() if live_refs is not None else set()
        removed = 0
        for name in cands:
            if name in live:
                continue
            path = os.path.join(d, name)
            with self._gc_lock:
                try:
                    if time.time() - os.path.getmtime(path) < grace_s:  # touched meanwhile
                        continue
                    os.unlink(path)
                    removed += 1
                except FileNotFoundError:
                    pass
        return removed

    def _fsync_dir(self, path: str):
        fd = os.open(os.path.dirname(path), os.O_RDONLY)
        try:
            os.fsync(fd)
        finally:
            os.close(fd)

    def put_chunks(self, sha: str, chunks, fsync: bool = True) -> bool:
        """Write an object from an iterable of byte chunks; verified against ``sha`` before it
        becomes visible (a torn or corrupted transfer never lands).  Idempotent.  ``fsync``
        (default): the file AND its directory entry are on disk before this returns -- a
        replica acknowledges a pre-replication push only then, so "a majority holds the blob"
        survives a crash just like the log entry that depends on it."""
        path = self.cas_path(sha)
        if self._touch(sha):
            for _ in chunks:  # drain the stream
                pass
            return True
        tmp = f"{path}.tmp{os.getpid()}.{threading.get_ident()}.{time.monotonic_ns()}"
        h = hashlib.sha256()
        try:
            with open(tmp, "wb") as f:
                for c in chunks:
                    h.update(c)
                    f.write(c)
                if fsync:
                    f.flush()
                    os.fsync(f.fileno())
            if h.hexdigest() != sha:
                raise ValueError(f"blob content does not match {sha[:12]}")
            os.replace(tmp, path)
            if fsync:
                self._fsync_dir(path)
            return True
        finally:
            if os.path.exists(tmp):
                os.unlink(tmp)

    def iter_chunks(self, sha: str, chunk: int = CHUNK):
        with open(self.cas_path(sha), "rb") as f:
            while True:
                b = f.read(chunk)
                if not b:
                    return
                yield b

    def size(self, sha: str) -> int:
        return os.path.getsize(self.cas_path(sha))


class BlobReplicator:
    """Leader side: push a CAS object to the followers over ``FileTransferService.SendFile``
    (1 MiB ``FileChunk``s) and wait for a majority of the cluster to hold it."""

    def __init__(self, store: BlobStore, peers: dict[int, str], timeout: float = 60.0):
        from .. import wire

        self.store = store
        self.timeout = timeout
        self._stubs = {pid: wire.Stub("FileTransferService", wire.channel(a)) for pid, a in peers.items()}
        self._pool = ThreadPoolExecutor(max_workers=max(1, 2 * len(peers)), thread_name_prefix="blob-push")
        self.pushed = 0

    def _push(self, pid: int, sha: str) -> bool:
        from ..wire import pb

        def chunks():
            first = True
            for b in self.store.iter_chunks(sha):
                yield pb.FileChunk(content=b, destination_path=f"{CAS_FOLDER}/{sha}" if first else "")
                first = False
            if first:  # empty object: one empty chunk still names the destination
                yield pb.FileChunk(content=b"", destination_path=f"{CAS_FOLDER}/{sha}")

        try:
            r = self._stubs[pid].SendFile(chunks(), timeout=self.timeout)
            ok = r.status.startswith("File received")
            if not ok:
                log.warning("blob %s push to %s: %s", sha[:12], pid, r.status)
            return ok
        except grpc.RpcError as e:
            log.warning("blob %s push to %s failed: %s", sha[:12], pid, e.code())
            return False

    def replicate(self, sha: str, cluster_size: int, timeout: float | None = None) -> bool:
        """True once ``cluster_size // 2 + 1`` replicas (this one included) hold ``sha``; the
        remaining pushes continue in the background."""
        need = cluster_size // 2 + 1 - 1  # peers besides this node
        if need <= 0:
            return True
        done = threading.Semaphore(0)
        acks = []

        def one(pid):
            ok = self._push(pid, sha)
            acks.append(ok)
            done.release()

        for pid in self._stubs:
            self._pool.submit(one, pid)
        end = time.monotonic() + (timeout or self.timeout)
        while sum(acks) < need:
            if len(acks) == len(self._stubs):
                return False
            if not done.acquire(timeout=max(0.0, end - time.monotonic())):
                return False
        self.pushed += 1
        return True

    def close(self):
        self._pool.shutdown(wait=False, cancel_futures=True)


class BlobFetcher:
    """Any replica: pull CAS objects it is missing from peers (``lmsinternal.Blob/Fetch``)."""

    def __init__(self, store: BlobStore, peers: dict[int, str], leader_id=lambda: None, timeout: float = 60.0):
        from .. import wire

        self.store = store
        self.peers = dict(peers)
        self.leader_id = leader_id
        self.timeout = timeout
        self._calls = {pid: wire.channel(a).unary_stream(FETCH_METHOD) for pid, a in self.peers.items()}
        self._lock = threading.Lock()
        self._inflight: dict[str, threading.Event] = {}
        self._pool = ThreadPoolExecutor(max_workers=2, thread_name_prefix="blob-fetch")
        self.fetched = 0

    def _order(self) -> list[int]:
        lid = self.leader_id()
        rest = [p for p in self.peers if p != lid]
        return ([lid] if lid in self.peers else []) + rest

    def _fetch_once(self, sha: str) -> bool:
        for pid in self._order():
            try:
                stream = self._calls[pid](sha.encode(), timeout=self.timeout)
                if self.store.put_chunks(sha, stream):
                    self.fetched += 1
                    return True
            except (grpc.RpcError, ValueError, OSError) as e:
                log.info("blob %s not fetched from %s: %s", sha[:12], pid, getattr(e, "code", lambda: e)())
        return False

    def fetch(self, sha: str, timeout: float | None = None) -> bool:
        """Block until this replica holds ``sha`` (pulling it if needed) or ``timeout``."""
        if self.store.has(sha):
            return True
        with self._lock:
            ev = self._inflight.get(sha)
            owner = ev is None
            if owner:
                ev = self._inflight[sha] = threading.Event()
        if owner:
            try:
                self._fetch_once(sha)
            finally:
                ev.set()
                with self._lock:
                    self._inflight.pop(sha, None)
        else:
            ev.wait(timeout if timeout is not None else self.timeout)
        return self.store.has(sha)

    def fetch_async(self, sha: str, then=None):
        """Background pull (the apply thread never blocks on a transfer); ``then()`` on success."""

        def run():
            for attempt in range(20):
                if self.fetch(sha):
                    if then is not None:
                        then()
                    return
                time.sleep(min(5.0, 0.2 * 2 ** attempt))
            log.warning("blob %s still missing after retries", sha[:12])

        return self._pool.submit(run)

    def close(self):
        self._pool.shutdown(wait=False, cancel_futures=True)


def fetch_handler(store: BlobStore):
    """Server side of ``lmsinternal.Blob/Fetch``: request body = sha256 hex, response = the
    object as a stream of 1 MiB chunks (NOT_FOUND if this replica does not hold it)."""

    def fetch(body: bytes, context):
        sha = body.decode(errors="replace")
        if not store.has(sha):
            context.abort(grpc.StatusCode.NOT_FOUND, "blob not held here")
        yield from store.iter_chunks(sha)

    return grpc.method_handlers_generic_handler("lmsinternal.Blob", {
        "Fetch": grpc.unary_stream_rpc_method_handler(fetch)})
