"""The reference client ``lms_gui_final.py`` connects UNCHANGED to a 5-node cluster of this
framework (north star).  tkinter is absent here, so the GUI runs on a headless fake tkinter in a
subprocess; its hard-coded server list is rewritten to the local cluster by a channel shim."""
import json
import os
import subprocess
import sys

import pytest

from lms_harness import Cluster, start_tutor

REF = "/root/reference/GUI_RAFT_LLM_SourceCode"
GUI_ADDRS = ["172.18.18.37:50051", "172.18.18.28:50052", "172.18.18.43:50053", "172.18.18.30:50054",
             "172.18.18.48:50055"]

pytestmark = [pytest.mark.timeout(180),
              pytest.mark.skipif(not os.path.exists(os.path.join(REF, "lms_gui_final.py")),
                                 reason="reference GUI not mounted")]


@pytest.mark.parametrize("stubs", ["reference", "ours"])
def test_reference_gui_runs_unchanged_against_cluster(tmp_path, stubs):
    """``stubs="ours"``: the GUI imports this framework's lms_pb2 / lms_pb2_grpc (runtime-built
    drop-ins), so a user needs nothing from the reference but the GUI file itself."""
    tsrv, tport, tutor = start_tutor()
    from lms_harness import KeywordGate

    c = Cluster(5, tmp_path, tutor_address=f"127.0.0.1:{tport}", gate=KeywordGate())
    try:
        c.wait_leader()
        amap = {g: c.addrs[i + 1] for i, g in enumerate(GUI_ADDRS)}
        env = dict(os.environ)
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        env["PYTHONPATH"] = root + os.pathsep + env.get("PYTHONPATH", "")
        env["GUI_OWN_STUBS"] = "1" if stubs == "ours" else "0"
        p = subprocess.run([sys.executable, os.path.join(os.path.dirname(__file__), "gui_driver.py"), REF,
                            json.dumps(amap), str(tmp_path)], capture_output=True, text=True, timeout=150, env=env)
        line = [ln for ln in p.stdout.splitlines() if ln.startswith("GUI_RESULT ")]
        assert line, p.stdout[-3000:] + p.stderr[-3000:]
        res = json.loads(line[0][len("GUI_RESULT "):])
    finally:
        c.close()
        tsrv.stop(0)
    own = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    assert res["stubs"].startswith(own if stubs == "ours" else REF), res["stubs"]
    steps = {s[0] + (("/" + s[1]) if s[0] in ("register", "login") else ""): s for s in res["steps"]}
    assert steps["register/stud"][2] == ["info", "Registration Success",
                                         "Registration request is being processed. Please wait."]
    assert steps["login/stud"][2] == "student"
    assert steps["post_assignment"][1] == ["info", "Success", "Assignment posted successfully."]
    assert steps["view_grades"][1] == ["info", "Grades", "Grade not yet assigned"]
    kind, title, text = steps["ask_llm"][1]
    assert (kind, title) == ("info", "LLM Response") and "how does raft leader election work" in text
    assert steps["ask_instructor"][1][0] == "info"
    assert steps["login/prof"][2] == "instructor"
    assert steps["instructor_menu"][1] is True
    assert res["steps"][-1][1] == ["info", "Logout", "Logged out successfully."]
    assert tutor.calls == ["how does raft leader election work"]
    # instructor flows and the student's download / response views, all through the unchanged GUI
    assert steps["post_material"][1] == ["info", "Success", "Course material posted successfully."]
    kind, title, text = steps["download_assignment"][1]
    assert (kind, title) == ("info", "Success") and text.startswith("Assignment saved to ")
    assert steps["download_assignment"][2] is True  # the saved bytes are the student's upload
    assert steps["grade"][1] == ["info", "Success", "Grade A submitted for Student ID: stud"]
    assert steps["query_choices"][1] == ["stud: office hours?"] and steps["query_choices"][2] == "stud: office hours?"
    assert steps["respond"][1] == ["info", "Success", "Response sent successfully."]
    assert steps["view_grades_after"][1] == "Your grade: A"
    assert steps["materials"][1] == "Instructor: prof, File: lecture1.pdf"
    kind, title, text = steps["download_material"][1]
    assert (kind, title) == ("info", "Success") and text.startswith("Course material saved to ")
    assert steps["download_material"][2] is True
    assert steps["instructor_responses"][1] == ["Your Query: office hours?\nInstructor Response: Tuesdays at 3pm"]
