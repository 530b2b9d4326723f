"""LMS state machine unit tests (SURVEY.md §4.3 "Unit: log format" / "Unit: state machine"):
golden log strings for the six reference ops (§2.3), legacy space/shlex decoding, each commit
hook's semantics, the lms_data.json schema (§2.4), snapshot/restore with blobs, PDF text."""
import base64
import hashlib
import json
import os

import pytest

from distributed_lms_raft_llm_amd.lms import commands
from distributed_lms_raft_llm_amd.lms.pdf import extract_text, make_pdf
from distributed_lms_raft_llm_amd.lms.state import LMSState


def test_golden_log_strings_match_reference_format():
    # the reference's live create_log_entry: json.dumps({"operation": op, "args": args})
    assert commands.encode("Register", ["bob", "pw", "student"]) == \
        '{"operation": "Register", "args": ["bob", "pw", "student"]}'
    assert commands.encode("PostAssignment", ["s", "a.pdf", "uploads/a.pdf", "text"]) == \
        '{"operation": "PostAssignment", "args": ["s", "a.pdf", "uploads/a.pdf", "text"]}'
    assert commands.encode("GradeAssignment", ["s", "A"]) == '{"operation": "GradeAssignment", "args": ["s", "A"]}'
    for op, n in (("PostCourseMaterial", 3), ("AskQuery", 2), ("RespondToQuery", 3)):
        s = commands.encode(op, [f"x{i}" for i in range(n)])
        assert json.loads(s) == {"operation": op, "args": [f"x{i}" for i in range(n)]}
    with pytest.raises(commands.BadCommand):
        commands.encode("Register", ["only-one"])
    with pytest.raises(commands.BadCommand):
        commands.encode("DropTable", [])


def test_decode_json_and_legacy_forms():
    assert commands.decode('{"operation": "AskQuery", "args": ["s", "what is raft"]}') == \
        ("AskQuery", ["s", "what is raft"])
    # legacy (the reference's shadowed v1 writer): space separated, shlex quoting
    assert commands.decode("Register bob pw student") == ("Register", ["bob", "pw", "student"])
    assert commands.decode("AskQuery s 'what is raft'") == ("AskQuery", ["s", "what is raft"])


def test_commit_hooks_semantics(tmp_path):
    st = LMSState(str(tmp_path))
    enc = commands.encode
    assert st.apply(1, enc("Register", ["s", "pw", "student"])) is True
    assert st.apply(2, enc("Register", ["s", "other", "instructor"])) is False  # first writer wins
    assert st.apply(3, enc("Register", ["t", "pw", "instructor"])) is True
    st.apply(4, enc("PostAssignment", ["s", "a.pdf", "uploads/a.pdf", "essay one"]))
    st.apply(5, enc("PostAssignment", ["s", "b.pdf", "uploads/b.pdf", "essay two"]))
    st.apply(6, enc("GradeAssignment", ["s", "B+"]))  # grades EVERY assignment of the student
    assert st.apply(7, enc("GradeAssignment", ["nobody", "A"])) is False
    st.apply(8, enc("AskQuery", ["s", "q1"]))
    st.apply(9, enc("AskQuery", ["s", "q2"]))
    st.apply(10, enc("RespondToQuery", ["t", "s", "r1"]))  # answers the FIRST unanswered query
    st.apply(11, enc("PostCourseMaterial", ["t", "m.pdf", "uploads/m.pdf"]))
    assert st.apply(12, "not a command") is None and st.apply(13, '{"operation": "Register", "args": [1]}') is None
    d = st.view()
    assert d["users"]["s"] == {"password": "pw", "role": "student"}
    assert [a["grade"] for a in d["assignments"]["s"]] == ["B+", "B+"]
    assert d["assignments"]["s"][0] == {"filename": "a.pdf", "filepath": os.path.join("uploads", "a.pdf"),
                                        "grade": "B+", "text": "essay one"}
    assert d["queries"]["s"] == [{"query": "q1", "answered": True, "response": "r1"},
                                 {"query": "q2", "answered": False, "response": None}]
    assert d["course_materials"] == [{"filename": "m.pdf", "filepath": os.path.join("uploads", "m.pdf"),
                                      "instructor": "t"}]
    assert st.applied_index == 13
    # export: the reference's lms_data.json schema, atomically written
    st.export()
    on_disk = json.load(open(tmp_path / "lms_data.json"))
    assert set(on_disk) >= {"users", "assignments", "course_materials", "queries"}
    assert on_disk["users"] == d["users"]


def test_sessions_blobs_snapshot_restore(tmp_path):
    st = LMSState(str(tmp_path / "a"))
    enc = commands.encode
    st.apply(1, enc("Register", ["s", "pw", "student"]))
    st.apply(2, enc("Login", ["s", "tok", "student"]))
    data = b"%PDF-1.4 fake bytes"
    assert st.apply(3, enc("StoreBlob", ["a.pdf", hashlib.sha256(data).hexdigest(),
                                         base64.b64encode(data).decode()])) is True
    assert st.apply(4, enc("StoreBlob", ["b.pdf", "0" * 64, base64.b64encode(data).decode()])) is False
    assert st.session("tok") == {"username": "s", "role": "student"}
    snap = st.snapshot()
    assert base64.b64encode(data).decode() not in snap  # snapshots carry the blob index, not bytes
    st2 = LMSState(str(tmp_path / "b"))
    st2.blobs.fetcher = _PeerFetcher(st2.blobs, st.blobs)  # the restoring replica pulls from a peer
    st2.restore(snap)
    assert st2.session("tok") == {"username": "s", "role": "student"}
    assert st2.read_blob(os.path.join("uploads", "a.pdf")) == data
    assert st2.view() == st.view()
    st2.apply(5, enc("Logout", ["tok"]))
    assert st2.session("tok") is None


class _PeerFetcher:
    """BlobFetcher stand-in: copies CAS objects from another replica's store."""

    def __init__(self, mine, peer):
        self.mine, self.peer = mine, peer

    def fetch(self, sha, timeout=None):
        if not self.mine.has(sha) and self.peer.has(sha):
            self.mine.put_chunks(sha, self.peer.iter_chunks(sha))
        return self.mine.has(sha)

    def fetch_async(self, sha, then=None):
        if self.fetch(sha) and then is not None:
            then()


def test_put_blob_materialises_or_fetches(tmp_path):
    """PutBlob (pre-replicated upload): linked into uploads/ when the CAS object is here, pulled
    from a peer otherwise; a wrong-size hash is refused."""
    leader = LMSState(str(tmp_path / "l"))
    data = os.urandom(3 << 20)  # several 1 MiB chunks
    sha = leader.blobs.put_bytes(data)
    cmd = commands.encode("PutBlob", ["hw.pdf", sha, len(data)])
    assert leader.apply(1, cmd) is True
    assert leader.read_blob("uploads/hw.pdf") == data
    follower = LMSState(str(tmp_path / "f"))
    follower.blobs.fetcher = _PeerFetcher(follower.blobs, leader.blobs)
    assert follower.apply(1, cmd) is True
    assert follower.read_blob("uploads/hw.pdf") == data and follower.blobs.has(sha)
    assert follower.apply(2, commands.encode("PutBlob", ["x.pdf", "abc", 3])) is False


def test_request_id_applies_once(tmp_path):
    st = LMSState(str(tmp_path))
    st.apply(1, commands.encode("Register", ["s", "pw", "student"]))
    st.apply(2, commands.encode("AskQuery", ["s", "q1"]))
    st.apply(3, commands.encode("AskQuery", ["s", "q2"]))
    r = commands.encode("RespondToQuery", ["t", "s", "answer"], rid="abc")
    assert st.apply(4, r) is True
    assert st.apply(5, r) is True  # the retry: same answer, NOT applied to q2
    qs = st.view()["queries"]["s"]
    assert qs[0]["answered"] and not qs[1]["answered"]
    assert st.rid_result("abc") == (True, True) and st.rid_result("zzz") == (False, None)
    st2 = LMSState(str(tmp_path / "b"))
    st2.restore(st.snapshot())
    assert st2.apply(6, r) is True and not st2.view()["queries"]["s"][1]["answered"]
    assert commands.decode(r) == ("RespondToQuery", ["t", "s", "answer"])


def test_pdf_text_roundtrip_and_plain_bytes():
    text = "Assignment 3\nExplain (briefly) Raft's log matching property."
    assert extract_text(make_pdf(text)).split() == text.split()
    assert extract_text(b"plain text upload") == "plain text upload"
