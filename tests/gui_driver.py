"""Runs the reference ``lms_gui_final.py`` UNCHANGED (fake headless tkinter, address-rewrite shim
for its hard-coded 172.18.18.x server list) against a live cluster and scripts a session the way
its button lambdas do.  Prints the dialog log and observations as one JSON line.

usage: python gui_driver.py <reference_dir> <addr_map_json> <workdir>
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    ref_dir, addr_map, workdir = sys.argv[1], json.loads(sys.argv[2]), sys.argv[3]
    sys.path.insert(0, os.path.join(HERE, "fake_tk"))
    sys.path.insert(0, ref_dir)
    if os.environ.get("GUI_OWN_STUBS") == "1":  # this framework's lms_pb2 / lms_pb2_grpc, not protoc's
        sys.path.insert(0, os.path.dirname(HERE))
    import grpc

    real = grpc.insecure_channel

    def shim(target, *a, **k):
        return real(addr_map.get(target, target), *a, **k)

    grpc.insecure_channel = shim
    import tkinter as tk
    from tkinter import filedialog, messagebox

    import lms_gui_final as gui
    import lms_pb2

    out_stub_origin = lms_pb2.__file__

    out = {"steps": [], "stubs": out_stub_origin}

    def click(text, idx=-1):
        bs = tk.find_buttons(text)
        assert bs, f"no button {text!r}"
        bs[idx].invoke()

    def dialogs_after(n, timeout=60):
        log = messagebox.wait_for(n + 1, timeout)
        return log[n] if len(log) > n else None

    root = tk.Tk()
    app = gui.LMSApp(root)
    out["leader_address"] = app.leader_address

    def register(user, role):
        n = len(messagebox.LOG)
        click("Register")  # login screen -> register screen
        app.reg_username.insert(0, user)
        app.reg_password.insert(0, "pw")
        app.reg_role.set(role)
        click("Register")  # submit on the register screen
        out["steps"].append(["register", user, dialogs_after(n)])

    def login(user):
        app.username.insert(0, user)
        app.password.insert(0, "pw")
        click("Login")
        end = time.time() + 30
        while app.token is None and time.time() < end:
            time.sleep(0.02)
        out["steps"].append(["login", user, app.role])

    def logout():
        n = len(messagebox.LOG)
        click("Logout")
        out["steps"].append(["logout", dialogs_after(n)])

    register("stud", "student")
    register("prof", "instructor")
    login("stud")
    # post assignment through the file-path entry
    path = os.path.join(workdir, "homework.pdf")
    from distributed_lms_raft_llm_amd.lms.pdf import make_pdf

    with open(path, "wb") as f:
        f.write(make_pdf("Raft consensus: leader election and log replication"))
    n = len(messagebox.LOG)
    click("Post Assignment")
    app.file_path.insert(0, path)
    click("Submit")
    out["steps"].append(["post_assignment", dialogs_after(n)])
    n = len(messagebox.LOG)
    click("Go Back")
    click("View Grades")
    out["steps"].append(["view_grades", dialogs_after(n)])
    # LLM query (radio default "llm")
    n = len(messagebox.LOG)
    click("Ask Query")
    app.query_text.insert(0, "how does raft leader election work")
    click("Submit Query")
    out["steps"].append(["ask_llm", dialogs_after(n)])
    # instructor question
    n = len(messagebox.LOG)
    click("Go Back")
    click("Ask Query")
    app.query_text.insert(0, "office hours?")
    app.query_option.set("instructor")
    click("Submit Query")
    out["steps"].append(["ask_instructor", dialogs_after(n)])
    click("Go Back")
    logout()
    login("prof")
    out["steps"].append(["instructor_menu", bool(tk.find_buttons("View and Grade Assignments"))])

    def wait_buttons(text, timeout=30, exclude=()):
        end = time.time() + timeout
        while time.time() < end:
            bs = [b for b in tk.find_buttons(text) if b not in exclude]
            if bs:
                return bs
            time.sleep(0.02)
        raise AssertionError(f"button {text!r} never appeared")

    def wait_label(pred, timeout=30):
        end = time.time() + timeout
        while time.time() < end:
            with tk._lock:
                hits = [w.kw.get("text") for w in tk.REGISTRY
                        if isinstance(w, tk.Label) and not w.destroyed and pred(str(w.kw.get("text", "")))]
            if hits:
                return hits
            time.sleep(0.02)
        raise AssertionError("label never appeared")

    def sha(path):
        import hashlib

        with open(path, "rb") as f:
            return hashlib.sha256(f.read()).hexdigest()

    # instructor: post course material (lms_gui_final.py:1034-1109)
    mat = os.path.join(workdir, "lecture1.pdf")
    with open(mat, "wb") as f:
        f.write(make_pdf("Lecture 1: replicated state machines and Raft"))
    n = len(messagebox.LOG)
    click("Post Course Material")
    app.file_path.insert(0, mat)
    click("Submit")
    out["steps"].append(["post_material", dialogs_after(n)])
    click("Go Back")
    # view & grade: download the assignment, then grade it (:1112-1248)
    n = len(messagebox.LOG)
    click("View and Grade Assignments")
    wait_buttons("Submit Grade")
    saved_hw = os.path.join(workdir, "downloaded_homework.pdf")
    filedialog.SAVE_PATHS.append(saved_hw)
    click("Download", 0)
    out["steps"].append(["download_assignment", dialogs_after(n), sha(saved_hw) == sha(path)])
    n = len(messagebox.LOG)
    old_btn = wait_buttons("Submit Grade")[0]
    old_btn.kw["command"].__defaults__[1].insert(0, "A")  # the row's grade Entry (lambda default g=)
    old_btn.invoke()
    out["steps"].append(["grade", dialogs_after(n)])
    wait_buttons("Submit Grade", exclude=(old_btn,))  # the list refreshes after grading (:1244)
    click("Go Back")
    # respond to the student's query through the "{id}: {data}" dropdown (:1255-1361)
    n = len(messagebox.LOG)
    click("Respond to Query")
    wait_buttons("Submit Response")
    out["steps"].append(["query_choices", sorted(app.student_queries), app.selected_query.get()])
    app.query_response.insert(0, "Tuesdays at 3pm")
    click("Submit Response")
    out["steps"].append(["respond", dialogs_after(n)])
    logout()
    # student: grade, course material download, instructor responses (:474-593, :730-838, :946-1013)
    login("stud")
    click("View Grades")
    out["steps"].append(["view_grades_after", wait_label(lambda t: t.startswith("Your grade"))[0]])
    click("Go Back")
    n = len(messagebox.LOG)
    click("View Course Material")
    out["steps"].append(["materials", wait_label(lambda t: t.startswith("Instructor: "))[0]])
    saved_mat = os.path.join(workdir, "downloaded_lecture1.pdf")
    filedialog.SAVE_PATHS.append(saved_mat)
    click("Download", 0)
    out["steps"].append(["download_material", dialogs_after(n), sha(saved_mat) == sha(mat)])
    click("Go Back")
    click("View Instructor Responses")
    out["steps"].append(["instructor_responses", wait_label(lambda t: "Instructor Response:" in t)])
    click("Go Back")
    logout()
    print("GUI_RESULT " + json.dumps(out), flush=True)
    os._exit(0)  # the GUI's executor threads are non-daemon


if __name__ == "__main__":
    main()
