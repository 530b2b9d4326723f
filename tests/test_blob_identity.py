"""Upload identity and durability and request-id idempotence of
Login / Logout: same-named uploads keep their own bytes, CAS objects are fsync'd
(file and directory) before a replica acknowledges them, unreferenced objects are collected at
snapshot time, and retried Login / Logout / pdf-capped uploads behave."""
import os
import sys
import types

import pytest

from distributed_lms_raft_llm_amd.lms import blobs as B
from distributed_lms_raft_llm_amd.lms import commands
from distributed_lms_raft_llm_amd.lms.pdf import extract_text
from distributed_lms_raft_llm_amd.lms.state import LMSState
from distributed_lms_raft_llm_amd.wire import pb
from lms_harness import Cluster

pytestmark = pytest.mark.timeout(120)


def _login(stub, user, role, meta=()):
    stub.Register(pb.RegisterRequest(username=user, password="pw", role=role), timeout=10)
    r = stub.Login(pb.LoginRequest(username=user, password="pw"), timeout=10, metadata=meta)
    assert r.success
    return r.token


def test_same_named_uploads_keep_their_own_bytes(tmp_path):
    """Two students upload ``report.pdf``: the instructor downloads each student's own bytes
    (the reference, and round 2, overwrote uploads/<name> and served the last one to both)."""
    c = Cluster(3, tmp_path)
    try:
        lid = c.wait_leader()
        st = c.stub(lid)
        ta, tb = _login(st, "ann", "student"), _login(st, "ben", "student")
        ti = _login(st, "ivy", "instructor")
        assert st.Post(pb.PostRequest(token=ta, type="assignment", file=b"ANN'S REPORT", filename="report.pdf"),
                       timeout=15).success
        assert st.Post(pb.PostRequest(token=tb, type="assignment", file=b"BEN'S REPORT", filename="report.pdf"),
                       timeout=15).success
        g = st.Get(pb.GetRequest(token=ti, type="student_list"), timeout=15)
        got = {(e.id, e.filename): e.file for e in g.entries}
        assert got == {("ann", "report.pdf"): b"ANN'S REPORT", ("ben", "report.pdf"): b"BEN'S REPORT"}
        # the reference layout is still there: uploads/<name> holds the latest upload
        path = os.path.join(str(tmp_path / f"node{lid}"), "uploads", "report.pdf")
        with open(path, "rb") as f:
            assert f.read() == b"BEN'S REPORT"
        # same for course materials
        assert st.Post(pb.PostRequest(token=ti, type="course_material", file=b"v1", filename="notes.pdf"),
                       timeout=15).success
        assert st.Post(pb.PostRequest(token=ti, type="course_material", file=b"v2", filename="notes.pdf"),
                       timeout=15).success
        g = st.Get(pb.GetRequest(token=ta, type="course_material"), timeout=15)
        assert [e.file for e in g.entries] == [b"v1", b"v2"]
    finally:
        c.close()


def test_post_commands_keep_reference_args_and_carry_sha():
    sha = "ab" * 32
    cmd = commands.encode("PostAssignment", ["s", "f.pdf", "uploads/f.pdf", "text"], meta={"sha256": sha})
    assert commands.decode(cmd) == ("PostAssignment", ["s", "f.pdf", "uploads/f.pdf", "text"])
    assert commands.decode_meta(cmd) == {"sha256": sha}
    with pytest.raises(commands.BadCommand):
        commands.encode("PostAssignment", ["s", "f.pdf", "p", "t"], meta={"bogus": 1})


def test_cas_objects_are_fsynced_file_and_directory(tmp_path, monkeypatch):
    """A replica acknowledges a pre-replication push (SendFile) only after the object's bytes AND
    its directory entry are on disk, so "a majority holds the blob" is crash-durable like the log
    entry that depends on it."""
    store = B.BlobStore(str(tmp_path))
    synced = []
    real = os.fsync

    def spy(fd):
        synced.append(os.readlink(f"/proc/self/fd/{fd}"))
        return real(fd)

    monkeypatch.setattr(os, "fsync", spy)
    data = b"x" * 4096
    sha = B.hashlib.sha256(data).hexdigest()
    from distributed_lms_raft_llm_amd.lms.service import FileTransferServicer

    state = types.SimpleNamespace(blobs=store)
    r = FileTransferServicer(state).SendFile(iter([pb.FileChunk(content=data, destination_path=f"cas/{sha}")]), None)
    assert r.status == "File received successfully"
    cas_dir = os.path.join(str(tmp_path), B.CAS_FOLDER)
    assert any(p.startswith(cas_dir + os.sep) and sha[:8] in p for p in synced), synced  # the file
    assert cas_dir in synced  # its directory entry
    assert store.has(sha)


def test_unreferenced_objects_collected_at_snapshot(tmp_path):
    s = LMSState(str(tmp_path))
    s.gc_grace_s = 0.0
    keep = s.blobs.put_bytes(b"referenced")
    stale = s.blobs.put_bytes(b"orphan")
    s.apply(1, commands.encode("PutBlob", ["a.pdf", keep, 10]))
    s.snapshot()
    import time

    for _ in range(100):  # collection runs on a background thread
        if not s.blobs.has(stale):
            break
        time.sleep(0.02)
    assert s.blobs.has(keep) and not s.blobs.has(stale)
    # within the grace period nothing is collected (an upload whose PutBlob is still in flight)
    s.gc_grace_s = 3600.0
    young = s.blobs.put_bytes(b"in flight")
    s.snapshot()
    time.sleep(0.2)
    assert s.blobs.has(young)


def test_gc_spares_reuploaded_and_newly_referenced_objects(tmp_path):
    """a stale unreferenced object that is uploaded again (pre-replication
    acknowledges it from the existing file) must survive the next GC pass, and an object whose
    PutBlob commits while a pass runs is re-checked against the live state before its unlink."""
    import time

    store = B.BlobStore(str(tmp_path))
    old = store.put_bytes(b"old content")
    path = store.cas_path(old)
    os.utime(path, (time.time() - 7200, time.time() - 7200))
    store.put_bytes(b"old content")  # re-upload of identical bytes: refreshes the mtime
    assert time.time() - os.path.getmtime(path) < 60
    assert store.gc(set(), grace_s=3600.0) == 0 and store.has(old)
    # the streamed pre-replication path too
    os.utime(path, (time.time() - 7200, time.time() - 7200))
    assert store.put_chunks(old, [b"old content"])
    assert store.gc(set(), grace_s=3600.0) == 0 and store.has(old)
    # snapshot-time set says unreferenced, the live state now references it: kept
    os.utime(path, (time.time() - 7200, time.time() - 7200))
    calls = []
    assert store.gc(set(), grace_s=3600.0, live_refs=lambda: calls.append(1) or {old}) == 0 and store.has(old)
    assert store.gc(set(), grace_s=3600.0, live_refs=lambda: calls.append(1) or set()) == 1 and not store.has(old)
    assert len(calls) == 2  # the live set is built once per pass, not once per candidate
    # a re-upload racing the unlink: _touch waits for the GC's re-check + unlink, then sees the
    # object absent and the upload writes it again
    old = store.put_bytes(b"racing content")
    os.utime(store.cas_path(old), (time.time() - 7200, time.time() - 7200))
    import threading

    store._gc_lock.acquire()
    t = threading.Thread(target=lambda: store.put_bytes(b"racing content"))
    t.start()
    time.sleep(0.05)
    assert t.is_alive()  # the touch is parked behind the GC's lock
    os.unlink(store.cas_path(old))  # what the GC does while holding it
    store._gc_lock.release()
    t.join(5)
    assert store.has(old) and store.get_sha(old) == b"racing content"


def test_login_and_logout_retries_are_idempotent(tmp_path):
    c = Cluster(3, tmp_path)
    try:
        lid = c.wait_leader()
        st = c.stub(lid)
        st.Register(pb.RegisterRequest(username="amy", password="pw", role="student"), timeout=10)
        meta = (("x-dlms-request-id", "login-1"),)
        r1 = st.Login(pb.LoginRequest(username="amy", password="pw"), timeout=10, metadata=meta)
        r2 = st.Login(pb.LoginRequest(username="amy", password="pw"), timeout=10, metadata=meta)
        assert r1.success and r2.success and r1.token == r2.token  # one session, not two
        server = c.servers[lid]
        assert sum(1 for v in server.state.sessions.values() if v["username"] == "amy") == 1
        lm = (("x-dlms-request-id", "logout-1"),)
        assert st.Logout(pb.LogoutRequest(token=r1.token), timeout=10, metadata=lm).success
        # the reply was "lost": the retry reports the committed result instead of failing
        assert st.Logout(pb.LogoutRequest(token=r1.token), timeout=10, metadata=lm).success
        # a fresh Logout of the dead session (no retry id) still fails
        assert not st.Logout(pb.LogoutRequest(token=r1.token), timeout=10).success
    finally:
        c.close()


def test_pypdf_branch_honours_the_text_cap(monkeypatch):
    """With pypdf importable, extraction stops once the cap is reached."""
    pages_read = []

    class Page:
        def __init__(self, i):
            self.i = i

        def extract_text(self):
            pages_read.append(self.i)
            return "x" * 1000

    class Reader:
        def __init__(self, f):
            self.pages = [Page(i) for i in range(100)]

    monkeypatch.setitem(sys.modules, "pypdf", types.SimpleNamespace(PdfReader=Reader))
    out = extract_text(b"%PDF-1.4 fake", limit=2500)
    assert len(out) == 2500 and len(pages_read) == 3
