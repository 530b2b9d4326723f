"""Desktop GUI for the LMS cluster (tkinter), built on ``LMSClient``.

The reference ships a Tk client, ``lms_gui_final.py`` (components C15-C19:
connection/leader discovery, login/register, student and instructor workflows, logout); it keeps
working unchanged against this framework (``tests/test_gui_compat.py``).  This is the framework's
own front end for the same workflows, designed around two defects of that client:

* every RPC runs on a worker thread and its result is handed back to the Tk thread with
  ``root.after`` -- the reference calls Tk from its worker threads, which Tk does
  not allow;
* leader discovery, retries and failover live in ``LMSClient`` (cached leader, re-discovery only
  after an UNAVAILABLE/DEADLINE error) instead of a 5 x N x 3 s WhoIsLeader sweep before every
  click (``lms_gui_final.py:64-185``).

Screens: login / register -> student menu (course material + download, post assignment, grade,
ask the LLM tutor, ask the instructor, instructor responses) or instructor menu (post course
material, view + download + grade assignments, answer unanswered queries) -> logout.  The user
visible strings come from the servers (they are the reference's, §2.5).

``python -m distributed_lms_raft_llm_amd.gui --servers h1:50051,h2:50052,...`` (or ``lms_gui.py``).
``sync=True`` runs RPCs inline (headless tests drive the widgets directly).
"""
from __future__ import annotations

import os
from concurrent.futures import ThreadPoolExecutor

from ..client import LMSClient


class LMSGui:
    def __init__(self, root, servers: list[str], sync: bool = False, client: LMSClient | None = None):
        import tkinter as tk
        from tkinter import filedialog, messagebox

        self.tk, self.mb, self.fd = tk, messagebox, filedialog
        self.root = root
        self.client = client or LMSClient(servers)
        self.sync = sync
        self.pool = None if sync else ThreadPoolExecutor(max_workers=2, thread_name_prefix="lms-gui-rpc")
        self.screen = None
        self.w: dict[str, object] = {}  # named widgets of the current screen (tests fill these in)
        root.title("Distributed LMS")
        self.show_login()

    # ------------------------------------------------------------------ plumbing
    def run(self, fn, done):
        """``fn()`` off the Tk thread; ``done(result, error)`` back on it."""
        if self.sync:
            try:
                res, err = fn(), None
            except Exception as e:  # noqa: BLE001 -- every failure becomes an error dialog
                res, err = None, e
            done(res, err)
            return
        fut = self.pool.submit(fn)

        def poll():
            if not fut.done():
                self.root.after(40, poll)
                return
            err = fut.exception()
            done(None if err else fut.result(), err)

        self.root.after(40, poll)

    def error(self, err, title="Error"):
        self.mb.showerror(title, f"{type(err).__name__}: {err}" if isinstance(err, Exception) else str(err))

    def clear(self, name: str):
        for c in list(self.root.winfo_children()):
            c.destroy()
        self.screen, self.w = name, {}
        frame = self.tk.Frame(self.root, padx=20, pady=20)
        frame.pack(fill=self.tk.BOTH, expand=True)
        return frame

    def _entry(self, frame, name: str, label: str, row: int, show: str | None = None):
        self.tk.Label(frame, text=label).grid(row=row, column=0, sticky=self.tk.W, pady=4)
        e = self.tk.Entry(frame, width=40, **({"show": show} if show else {}))
        e.grid(row=row, column=1, pady=4)
        self.w[name] = e
        return e

    def _button(self, frame, text: str, cmd, row: int, col: int = 0, span: int = 2):
        b = self.tk.Button(frame, text=text, command=cmd, width=28)
        b.grid(row=row, column=col, columnspan=span, pady=3)
        return b

    def _label(self, frame, text: str, row: int, name: str | None = None, **kw):
        lab = self.tk.Label(frame, text=text, justify=self.tk.LEFT, wraplength=560, **kw)
        lab.grid(row=row, column=0, columnspan=2, sticky=self.tk.W, pady=3)
        if name:
            self.w[name] = lab
        return lab

    # ------------------------------------------------------------------ auth
    def show_login(self):
        f = self.clear("login")
        self._label(f, "Distributed LMS -- sign in", 0, font=("Helvetica", 16, "bold"))
        self._entry(f, "username", "Username", 1)
        self._entry(f, "password", "Password", 2, show="*")
        self._button(f, "Login", self.login, 3)
        self._button(f, "Register", self.show_register, 4)

    def show_register(self):
        f = self.clear("register")
        self._label(f, "Create an account", 0, font=("Helvetica", 16, "bold"))
        self._entry(f, "username", "Username", 1)
        self._entry(f, "password", "Password", 2, show="*")
        role = self.tk.StringVar(self.root, value="student")
        self.tk.Label(f, text="Role").grid(row=3, column=0, sticky=self.tk.W)
        self.tk.OptionMenu(f, role, "student", "instructor").grid(row=3, column=1, sticky=self.tk.W)
        self.w["role"] = role
        self._button(f, "Create Account", self.register, 4)
        self._button(f, "Back to Login", self.show_login, 5)

    def register(self):
        user, pw, role = self.w["username"].get().strip(), self.w["password"].get(), self.w["role"].get()
        if not user or not pw:
            self.mb.showwarning("Register", "Username and password are required.")
            return

        def done(r, err):
            if err:
                return self.error(err, "Registration Failed")
            (self.mb.showinfo if r.success else self.mb.showerror)(
                "Registration Success" if r.success else "Registration Failed", r.message)
            if r.success:
                self.show_login()

        self.run(lambda: self.client.register(user, pw, role), done)

    def login(self):
        user, pw = self.w["username"].get().strip(), self.w["password"].get()

        def done(ok, err):
            if err:
                return self.error(err, "Login Failed")
            if not ok:
                return self.mb.showerror("Login Failed", "Invalid username or password.")
            self.user = user
            (self.show_instructor_menu if self.client.role == "instructor" else self.show_student_menu)()

        self.run(lambda: self.client.login(user, pw), done)

    def logout(self):
        def done(ok, err):
            if err:
                return self.error(err, "Logout")
            self.mb.showinfo("Logout", "Logged out successfully." if ok else "Session already ended.")
            self.show_login()

        self.run(self.client.logout, done)

    # ------------------------------------------------------------------ student
    def show_student_menu(self):
        f = self.clear("student")
        self._label(f, f"Student: {self.user}   (leader {self.client.leader_address})", 0)
        for i, (text, cmd) in enumerate((("View Course Material", self.view_course_material),
                                         ("Post Assignment", self.post_assignment),
                                         ("View Grades", self.view_grades),
                                         ("Ask LLM Tutor", self.show_ask_llm),
                                         ("Ask Instructor", self.show_ask_instructor),
                                         ("View Instructor Responses", self.view_responses),
                                         ("Logout", self.logout))):
            self._button(f, text, cmd, i + 1)

    def _back(self, f, row: int):
        back = self.show_instructor_menu if self.client.role == "instructor" else self.show_student_menu
        self._button(f, "Back", back, row)

    def view_course_material(self):
        def done(r, err):
            if err:
                return self.error(err)
            f = self.clear("course_material")
            self._label(f, "Course material", 0, font=("Helvetica", 14, "bold"))
            if not r.entries:
                self._label(f, r.message or "No course material available.", 1, name="empty")
            for i, e in enumerate(r.entries):
                self._label(f, f"{e.filename}  (by {e.instructor or e.id})", 2 * i + 1)
                self._button(f, "Download", lambda e=e: self.save_file(e.filename, e.file), 2 * i + 2)
            self._back(f, 2 * len(r.entries) + 3)

        self.run(self.client.course_materials, done)

    def save_file(self, filename: str, data: bytes):
        path = self.fd.asksaveasfilename(initialfile=filename, defaultextension=os.path.splitext(filename)[1])
        if not path:
            return
        with open(path, "wb") as fh:
            fh.write(data)
        self.mb.showinfo("Download", f"Saved {filename} to {path}")

    def post_assignment(self):
        path = self.fd.askopenfilename(filetypes=[("PDF files", "*.pdf"), ("All files", "*")])
        if not path:
            return

        def done(ok, err):
            if err:
                return self.error(err)
            (self.mb.showinfo if ok else self.mb.showerror)(
                "Success" if ok else "Error", "Assignment posted successfully." if ok else "Failed to post assignment.")

        self.run(lambda: self.client.post_assignment(path), done)

    def view_grades(self):
        def done(grade, err):
            if err:
                return self.error(err)
            self.mb.showinfo("Grades", grade)

        self.run(self.client.grade, done)

    def _ask_screen(self, title: str, button: str, action):
        f = self.clear(title)
        self._label(f, title, 0, font=("Helvetica", 14, "bold"))
        self._entry(f, "query", "Your question", 1)
        self._button(f, button, action, 2)
        self._label(f, "", 3, name="answer")
        self._back(f, 4)

    def show_ask_llm(self):
        self._ask_screen("Ask the LLM tutor", "Ask Tutor", self.ask_llm)

    def ask_llm(self):
        q = self.w["query"].get().strip()
        if not q:
            return self.mb.showwarning("Ask", "Type a question first.")
        self.w["answer"].config(text="Thinking ...")

        def done(ans, err):
            if err:
                return self.error(err, "LLM Tutor")
            if "answer" in self.w:
                self.w["answer"].config(text=ans)
            self.mb.showinfo("LLM Response", ans)

        self.run(lambda: self.client.ask_llm(q), done)

    def show_ask_instructor(self):
        self._ask_screen("Ask the instructor", "Send Query", self.ask_instructor)

    def ask_instructor(self):
        q = self.w["query"].get().strip()
        if not q:
            return self.mb.showwarning("Ask", "Type a question first.")

        def done(ok, err):
            if err:
                return self.error(err)
            (self.mb.showinfo if ok else self.mb.showerror)(
                "Query", "Query sent to the instructor." if ok else "Failed to send the query.")

        self.run(lambda: self.client.ask_instructor(q), done)

    def view_responses(self):
        def done(rs, err):
            if err:
                return self.error(err)
            f = self.clear("responses")
            self._label(f, "Instructor responses", 0, font=("Helvetica", 14, "bold"))
            for i, text in enumerate(rs or ["No responses yet."]):
                self._label(f, text, i + 1)
            self._back(f, len(rs or [0]) + 2)

        self.run(self.client.instructor_responses, done)

    # ------------------------------------------------------------------ instructor
    def show_instructor_menu(self):
        f = self.clear("instructor")
        self._label(f, f"Instructor: {self.user}   (leader {self.client.leader_address})", 0)
        for i, (text, cmd) in enumerate((("Post Course Material", self.post_course_material),
                                         ("View and Grade Assignments", self.view_assignments),
                                         ("Respond to Queries", self.view_queries),
                                         ("Logout", self.logout))):
            self._button(f, text, cmd, i + 1)

    def post_course_material(self):
        path = self.fd.askopenfilename(filetypes=[("PDF files", "*.pdf"), ("All files", "*")])
        if not path:
            return

        def done(ok, err):
            if err:
                return self.error(err)
            (self.mb.showinfo if ok else self.mb.showerror)(
                "Success" if ok else "Error",
                "Course material posted successfully." if ok else "Failed to post course material.")

        self.run(lambda: self.client.post_course_material(path), done)

    def view_assignments(self):
        def done(r, err):
            if err:
                return self.error(err)
            f = self.clear("assignments")
            self._label(f, "Submitted assignments", 0, font=("Helvetica", 14, "bold"))
            row = 1
            if not r.entries:
                self._label(f, r.message or "No assignments submitted.", row, name="empty")
                row += 1
            for i, e in enumerate(r.entries):
                self._label(f, f"{e.id}: {e.filename}", row)
                self._button(f, "Download", lambda e=e: self.save_file(e.filename, e.file), row + 1)
                self._entry(f, f"grade:{i}", "Grade", row + 2)
                self._button(f, "Submit Grade", lambda i=i, s=e.id: self.grade(i, s), row + 3)
                row += 4
            self._back(f, row)

        self.run(self.client.assignments, done)

    def grade(self, i: int, student: str):
        g = self.w[f"grade:{i}"].get().strip()
        if not g:
            return self.mb.showwarning("Grade", "Enter a grade first.")

        def done(r, err):
            if err:
                return self.error(err)
            (self.mb.showinfo if r.success else self.mb.showerror)("Grade", r.message)

        self.run(lambda: self.client.grade_assignment(student, g), done)

    def view_queries(self):
        def done(qs, err):
            if err:
                return self.error(err)
            f = self.clear("queries")
            self._label(f, "Unanswered queries", 0, font=("Helvetica", 14, "bold"))
            row = 1
            if not qs:
                self._label(f, "No unanswered queries.", row, name="empty")
                row += 1
            for i, (student, text) in enumerate(qs):
                self._label(f, f"{student}: {text}", row)
                self._entry(f, f"reply:{i}", "Response", row + 1)
                self._button(f, "Respond", lambda i=i, s=student: self.respond(i, s), row + 2)
                row += 3
            self._back(f, row)

        self.run(self.client.unanswered_queries, done)

    def respond(self, i: int, student: str):
        text = self.w[f"reply:{i}"].get().strip()
        if not text:
            return self.mb.showwarning("Respond", "Type a response first.")

        def done(ok, err):
            if err:
                return self.error(err)
            (self.mb.showinfo if ok else self.mb.showerror)(
                "Respond", "Response sent." if ok else "Failed to send the response.")
            if ok:
                self.view_queries()

        self.run(lambda: self.client.respond(student, text), done)

    def close(self):
        if self.pool is not None:
            self.pool.shutdown(wait=False)
        self.client.close()


def main(argv=None):
    import argparse

    ap = argparse.ArgumentParser(description="Distributed LMS desktop client (tkinter)")
    ap.add_argument("--servers", default="127.0.0.1:50051,127.0.0.1:50052,127.0.0.1:50053",
                    help="comma-separated LMS server addresses, in server-id order")
    ap.add_argument("--config", help="cluster YAML/JSON with a 'servers' map (as lms_server.py --config)")
    args = ap.parse_args(argv)
    servers = [s for s in args.servers.split(",") if s]
    if args.config:
        from ..utils.config import load_config

        m = load_config(args.config).get("servers") or {}
        servers = [m[k] for k in sorted(m, key=int)]
    import tkinter as tk

    root = tk.Tk()
    app = LMSGui(root, servers)
    try:
        root.mainloop()
    finally:
        app.close()
