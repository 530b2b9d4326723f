"""The framework's own Tk client (``distributed_lms_raft_llm_amd/gui``) driven headless on the fake
tkinter against a live 3-node cluster: every student and instructor workflow through the
widgets, then the leader is killed and the next click still succeeds (failover in LMSClient)."""
import os
import sys

import pytest

from lms_harness import Cluster, KeywordGate, start_tutor

HERE = os.path.dirname(os.path.abspath(__file__))

pytestmark = pytest.mark.timeout(120)


@pytest.fixture
def fake_tk():
    saved = {k: v for k, v in sys.modules.items() if k == "tkinter" or k.startswith("tkinter.")}
    sys.path.insert(0, os.path.join(HERE, "fake_tk"))
    for k in saved:
        del sys.modules[k]
    import tkinter
    from tkinter import filedialog, messagebox

    messagebox.LOG.clear()
    yield tkinter, messagebox, filedialog
    sys.path.remove(os.path.join(HERE, "fake_tk"))
    for k in [k for k in sys.modules if k == "tkinter" or k.startswith("tkinter.")]:
        del sys.modules[k]
    sys.modules.update(saved)


def test_own_gui_workflows_and_failover(tmp_path, fake_tk):
    tk, mb, fd = fake_tk
    from distributed_lms_raft_llm_amd.gui import LMSGui
    from distributed_lms_raft_llm_amd.lms.pdf import make_pdf

    def click(text):
        bs = tk.find_buttons(text)
        assert bs, f"no button {text!r}"
        bs[-1].invoke()

    def last():
        return mb.LOG[-1]

    tsrv, tport, tutor = start_tutor()
    c = Cluster(3, tmp_path, tutor_address=f"127.0.0.1:{tport}", gate=KeywordGate())
    try:
        c.wait_leader()
        app = LMSGui(tk.Tk(), [c.addrs[i] for i in sorted(c.addrs)], sync=True)
        assert app.screen == "login"

        def login(user):
            app.w["username"].insert(0, user)
            app.w["password"].insert(0, "pw")
            click("Login")

        for user, role in (("stud", "student"), ("prof", "instructor")):
            click("Register")
            assert app.screen == "register"
            app.w["username"].insert(0, user)
            app.w["password"].insert(0, "pw")
            app.w["role"].set(role)
            click("Create Account")
            assert last()[:2] == ("info", "Registration Success"), last()
            assert app.screen == "login"

        # instructor posts course material
        material = tmp_path / "raft_notes.pdf"
        material.write_bytes(make_pdf("raft consensus: leader election and log replication"))
        login("prof")
        assert app.screen == "instructor"
        fd.OPEN_PATHS.append(str(material))
        click("Post Course Material")
        assert last() == ("info", "Success", "Course material posted successfully."), last()
        click("Logout")
        assert last() == ("info", "Logout", "Logged out successfully.") and app.screen == "login"

        # student: material download, assignment, grade, LLM tutor, instructor query
        login("stud")
        assert app.screen == "student"
        click("View Course Material")
        assert app.screen == "course_material"
        saved = tmp_path / "downloaded.pdf"
        fd.SAVE_PATHS.append(str(saved))
        click("Download")
        assert saved.read_bytes() == material.read_bytes()
        click("Back")
        assignment = tmp_path / "hw1.pdf"
        assignment.write_bytes(make_pdf("how does raft leader election work with terms and votes"))
        fd.OPEN_PATHS.append(str(assignment))
        click("Post Assignment")
        assert last() == ("info", "Success", "Assignment posted successfully."), last()
        click("View Grades")
        assert last() == ("info", "Grades", "Grade not yet assigned"), last()
        click("Ask LLM Tutor")
        app.w["query"].insert(0, "how does raft leader election work")
        click("Ask Tutor")
        kind, title, text = last()
        assert (kind, title) == ("info", "LLM Response") and "how does raft leader election work" in text
        assert app.w["answer"].cget("text") == text
        assert tutor.calls == ["how does raft leader election work"]
        click("Back")
        click("Ask Instructor")
        app.w["query"].insert(0, "is the midterm open book?")
        click("Send Query")
        assert last() == ("info", "Query", "Query sent to the instructor."), last()
        click("Back")
        click("Logout")

        # instructor grades and answers
        login("prof")
        click("View and Grade Assignments")
        assert app.screen == "assignments" and "grade:0" in app.w
        app.w["grade:0"].insert(0, "A")
        click("Submit Grade")
        assert last()[:2] == ("info", "Grade"), last()
        click("Back")
        click("Respond to Queries")
        assert app.screen == "queries" and "reply:0" in app.w
        app.w["reply:0"].insert(0, "Yes, one sheet of notes.")
        click("Respond")
        assert last() == ("info", "Respond", "Response sent."), last()
        assert app.screen == "queries" and "empty" in app.w  # refreshed: nothing left unanswered
        click("Back")
        click("Logout")

        # student sees both; then the leader dies and the next click fails over
        login("stud")
        click("View Grades")
        assert last() == ("info", "Grades", "Your grade: A"), last()
        click("View Instructor Responses")
        assert app.screen == "responses"
        click("Back")
        c.stop(c.wait_leader())
        click("View Grades")
        assert last() == ("info", "Grades", "Your grade: A"), last()
        click("Logout")
        assert last() == ("info", "Logout", "Logged out successfully.")
        app.close()
    finally:
        c.close()
        tsrv.stop(0)


def test_rpc_results_come_back_on_the_tk_thread(fake_tk):
    """Non-sync mode: the RPC runs on a pool thread, ``done`` runs from ``root.after`` (the Tk
    thread), never from the worker -- the reference GUI touches Tk from its workers."""
    import threading
    import time

    from distributed_lms_raft_llm_amd.gui import LMSGui

    class Root:
        def __init__(self):
            self.q = []

        def title(self, *_):
            pass

        def winfo_children(self):
            return []

        def after(self, ms, fn):
            self.q.append(fn)

    class Client:
        def close(self):
            pass

    root = Root()
    app = LMSGui.__new__(LMSGui)
    app.root, app.sync, app.client = root, False, Client()
    from concurrent.futures import ThreadPoolExecutor

    app.pool = ThreadPoolExecutor(1)
    seen = []
    app.run(lambda: threading.current_thread().name, lambda r, e: seen.append((r, e, threading.current_thread())))
    end = time.time() + 5
    while not seen and time.time() < end:
        while root.q:
            root.q.pop(0)()
        time.sleep(0.01)
    worker, err, caller = seen[0]
    assert err is None and worker != threading.current_thread().name and caller is threading.current_thread()
    app.run(lambda: 1 / 0, lambda r, e: seen.append((r, e)))
    end = time.time() + 5
    while len(seen) < 2 and time.time() < end:
        while root.q:
            root.q.pop(0)()
        time.sleep(0.01)
    assert isinstance(seen[1][1], ZeroDivisionError)
    app.close()
