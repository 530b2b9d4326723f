"""LMSClient: the GUI workflows end to end, including a leader crash in the middle of a session."""
import time

import pytest

from distributed_lms_raft_llm_amd.client import LMSClient
from lms_harness import Cluster, KeywordGate, start_tutor

pytestmark = pytest.mark.timeout(120)


def test_client_workflows_and_transparent_failover(tmp_path):
    tsrv, tport, _ = start_tutor()
    c = Cluster(3, tmp_path, tutor_address=f"127.0.0.1:{tport}", gate=KeywordGate())
    try:
        c.wait_leader()
        addrs = [c.addrs[i] for i in sorted(c.addrs)]
        prof, stud = LMSClient(addrs), LMSClient(addrs)
        assert prof.register("prof", "pw", "instructor").success
        assert stud.register("stud", "pw", "student").success
        assert prof.login("prof", "pw") and prof.role == "instructor"
        assert stud.login("stud", "pw") and stud.role == "student"
        assert prof.post_course_material(data=b"lecture 1", filename="l1.pdf")
        assert [e.filename for e in stud.course_materials().entries] == ["l1.pdf"]
        assert stud.post_assignment(data=b"raft paper summary", filename="hw.txt")
        assert stud.grade() == "Grade not yet assigned"
        # kill the leader between two calls: both clients keep working, same tokens
        lid = c.wait_leader()
        c.stop(lid)
        t0 = time.time()
        assert prof.grade_assignment("stud", "B+").success
        assert time.time() - t0 < 5
        assert stud.grade() == "Your grade: B+"
        assert stud.ask_instructor("when is the midterm?")
        assert prof.unanswered_queries() == [("stud", "when is the midterm?")]
        assert prof.respond("stud", "next week")
        assert stud.instructor_responses() == ["Your Query: when is the midterm?\nInstructor Response: next week"]
        assert "raft" in stud.ask_llm("summarize the raft paper")
        assert stud.logout() and prof.logout()
        prof.close()
        stud.close()
    finally:
        c.close()
        tsrv.stop(0)
