"""Upload durability across a leader crash: a ``PutBlob`` is proposed only
after its content-addressed object is durable (fsync'd file + directory) on a majority, so a
leader that dies between the push acknowledgements and the commit leaves at worst an orphan
object -- never a committed entry whose bytes a majority cannot serve."""
import hashlib
import os
import threading

import pytest

from distributed_lms_raft_llm_amd.lms import blobs as B
from distributed_lms_raft_llm_amd.lms import commands
from distributed_lms_raft_llm_amd.wire import pb
from lms_harness import Cluster

pytestmark = pytest.mark.timeout(180)


def _holders(c, tmp_path, sha):
    """Nodes whose data directory holds the object (running or stopped)."""
    return {i for i in c.addrs if B.BlobStore(str(tmp_path / f"node{i}")).has(sha)}


def _login(st, user, role="student"):
    st.Register(pb.RegisterRequest(username=user, password="pw", role=role), timeout=10)
    r = st.Login(pb.LoginRequest(username=user, password="pw"), timeout=10)
    assert r.success
    return r.token


def _committed_shas(server):
    return server.state.read(lambda d: [a.get("sha256") for items in d["assignments"].values() for a in items])


def test_leader_crash_between_push_ack_and_commit(tmp_path):
    c = Cluster(3, tmp_path, fsync=True)
    try:
        lid = c.wait_leader()
        st = c.stub(lid)
        tok = _login(st, "amy")
        data = os.urandom(200_000)
        sha = hashlib.sha256(data).hexdigest()
        pushed = threading.Event()
        leader = c.servers[lid]
        real = leader.lms._write_many

        def crash_before_propose(items, rid=None):
            # the majority push has been acknowledged (``_store_upload`` returned): die here,
            # before anything is proposed
            if any(it[0] == "PutBlob" for it in items):
                pushed.set()
                raise RuntimeError("leader crashed")
            return real(items, rid)

        leader.lms._write_many = crash_before_propose
        r = st.Post(pb.PostRequest(token=tok, type="assignment", file=data, filename="hw.pdf"), timeout=30)
        assert pushed.is_set() and not r.success
        c.stop(lid)  # the crash: its disk stays, its process is gone
        # the pushed object is durable on a majority (the dead leader's disk included) ...
        assert len(_holders(c, tmp_path, sha)) >= 2
        # ... and the survivors elect a leader that never committed the upload
        new = c.wait_leader(timeout=15)
        assert new != lid
        assert sha not in _committed_shas(c.servers[new])
        # the dead node comes back, the student retries: committed, and a majority holds the bytes
        c.start(lid)
        new = c.wait_leader(timeout=15)
        st2 = c.stub(new)
        assert st2.Post(pb.PostRequest(token=tok, type="assignment", file=data, filename="hw.pdf"),
                        timeout=30).success
        assert sha in _committed_shas(c.servers[new])
        assert len(_holders(c, tmp_path, sha)) >= 2
        ti = _login(st2, "ivy", role="instructor")
        g = st2.Get(pb.GetRequest(token=ti, type="student_list"), timeout=30)
        assert [e.file for e in g.entries] == [data]
    finally:
        c.close()


def test_putblob_is_proposed_only_after_a_durable_majority(tmp_path, monkeypatch):
    """At the moment the leader proposes a PutBlob, the object's file AND directory entry have been
    fsync'd on a majority of the nodes (one process here, so one fsync spy sees every replica)."""
    synced: list[str] = []
    real_fsync = os.fsync

    def spy(fd):
        try:
            synced.append(os.readlink(f"/proc/self/fd/{fd}"))
        except OSError:
            pass
        return real_fsync(fd)

    monkeypatch.setattr(os, "fsync", spy)
    c = Cluster(3, tmp_path)
    try:
        lid = c.wait_leader()
        st = c.stub(lid)
        tok = _login(st, "ben")
        data = os.urandom(50_000)
        sha = hashlib.sha256(data).hexdigest()
        node = c.servers[lid].node
        real_submit = node.submit
        seen = []

        def checked_submit(cmd, *a, **k):
            op, args = commands.decode(cmd)
            if op == "PutBlob" and args[1] == sha:
                durable = set()
                for i in c.addrs:
                    cas = str(tmp_path / f"node{i}" / B.CAS_FOLDER)
                    if any(p.startswith(cas + os.sep) and sha[:16] in p for p in synced) and cas in synced:
                        durable.add(i)
                seen.append(durable)
            return real_submit(cmd, *a, **k)

        node.submit = checked_submit
        assert st.Post(pb.PostRequest(token=tok, type="assignment", file=data, filename="a.pdf"), timeout=30).success
        assert seen and len(seen[0]) >= 2, seen
    finally:
        c.close()
