"""Command-line LMS client (the GUI's workflows, scriptable).

    python -m distributed_lms_raft_llm_amd.client --servers h1:50051,h2:50052,... <command> [args]

Commands: leader | register USER PASS ROLE | login USER PASS | logout | post-assignment FILE |
post-material FILE | materials [--save DIR] | grade | ask-llm QUERY | ask-instructor QUERY |
responses | assignments [--save DIR] | grade-assignment STUDENT GRADE | unanswered |
respond STUDENT TEXT.   The session token is kept in ~/.dlms_session (or --session FILE).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

from . import LMSClient


def main(argv=None):
    ap = argparse.ArgumentParser(prog="dlms-client")
    ap.add_argument("--servers", default=os.environ.get("DLMS_SERVERS", "localhost:50051"))
    ap.add_argument("--session", default=os.path.expanduser("~/.dlms_session"))
    ap.add_argument("command")
    ap.add_argument("args", nargs="*")
    ap.add_argument("--save", default=None)
    a = ap.parse_args(argv)
    c = LMSClient(a.servers.split(","))
    if os.path.exists(a.session):
        with open(a.session) as f:
            s = json.load(f)
        c.token, c.role = s.get("token"), s.get("role")

    def save():
        with open(a.session, "w") as f:
            json.dump({"token": c.token, "role": c.role}, f)

    cmd, args = a.command, a.args
    out = None
    if cmd == "leader":
        out = c.discover()
    elif cmd == "register":
        r = c.register(*args)
        out = {"success": r.success, "message": r.message}
    elif cmd == "login":
        out = {"success": c.login(*args), "role": c.role}
        save()
    elif cmd == "logout":
        out = c.logout()
        save()
    elif cmd == "post-assignment":
        out = c.post_assignment(args[0])
    elif cmd == "post-material":
        out = c.post_course_material(args[0])
    elif cmd in ("materials", "assignments"):
        r = c.course_materials() if cmd == "materials" else c.assignments()
        out = {"success": r.success, "message": r.message,
               "entries": [{"id": e.id, "filename": e.filename, "bytes": len(e.file), "instructor": e.instructor}
                           for e in r.entries]}
        if a.save:
            os.makedirs(a.save, exist_ok=True)
            for e in r.entries:
                with open(os.path.join(a.save, os.path.basename(e.filename)), "wb") as f:
                    f.write(e.file)
    elif cmd == "grade":
        out = c.grade()
    elif cmd == "ask-llm":
        out = c.ask_llm(" ".join(args))
    elif cmd == "ask-instructor":
        out = c.ask_instructor(" ".join(args))
    elif cmd == "responses":
        out = c.instructor_responses()
    elif cmd == "grade-assignment":
        r = c.grade_assignment(args[0], args[1])
        out = {"success": r.success, "message": r.message}
    elif cmd == "unanswered":
        out = c.unanswered_queries()
    elif cmd == "respond":
        out = c.respond(args[0], " ".join(args[1:]))
    else:
        ap.error(f"unknown command {cmd}")
    print(out if isinstance(out, str) else json.dumps(out, indent=2))
    c.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
