"""``lms.LMS`` gRPC service: authentication, course workflows and the LLM tutoring path.

Behaviour and every user-visible string follow the reference handlers
(``lms_server.py:740-1274``) because ``lms_gui_final.py`` branches on them
(e.g. ``"Grade not yet assigned"`` at ``lms_gui_final.py:790``).  What changes:

* writes are proposed through Raft and the RPC returns after the entry is committed AND applied
  (the reference acknowledges before replication); the reply strings stay the same;
* a follower forwards any call to the current leader (the reference's follower writes crashed
  with ``KeyError``, Appendix A.7) -- the GUI always asks ``WhoIsLeader`` first, so this only
  matters during failover;
* reads are served after a leader read-barrier, so an acknowledged write is always visible;
* ``LMS.WhoIsLeader`` is implemented (the reference left it UNIMPLEMENTED, Appendix A.8);
* ``GetLLMAnswer`` runs the BERT relevance gate with cached assignment embeddings and calls the
  tutoring service with a deadline.
"""
from __future__ import annotations

import logging
import threading
import time
import uuid

import grpc

from .. import wire
from ..raft.core import NotLeader
from ..utils.metrics import METRICS
from ..utils.trace import TRACER
from ..wire import pb
from . import commands
from .pdf import extract_text

log = logging.getLogger("dlms.lms")

FORWARD_HEADER = "x-dlms-forwarded"
REQUEST_ID_HEADER = "x-dlms-request-id"  # client request id: writes carrying one apply once
# assignment text kept in the replicated state (the relevance gate reads <= 512 tokens of it);
# a multi-MB upload must not become a multi-MB Raft entry
TEXT_CAP = 256 * 1024

MSG_REGISTER_OK = "Registration request is being processed. Please wait."
MSG_USER_EXISTS = "Username already exists."
MSG_GRADE_OK = "Grading request is being processed. Please wait."
MSG_BAD_TOKEN = "Invalid session token"
MSG_ONLY_INSTRUCTORS_GRADE = "Only instructors can grade assignments"
MSG_NO_STUDENT_ASSIGNMENT = "Student assignment not found"
MSG_NO_MATERIALS = "No course materials available."
MSG_BAD_GET = "Invalid request type or unauthorized access"
MSG_INVALID_SESSION = "Invalid session"
MSG_ONLY_STUDENTS_GRADES = "Only students can view grades"
MSG_GRADE_NOT_ASSIGNED = "Grade not yet assigned"
MSG_NO_GRADE = "No grade assigned yet."
MSG_NO_ASSIGNMENTS = "No assignments found for this student."
MSG_LLM_INVALID_SESSION = "Invalid session."
MSG_LLM_ONLY_STUDENTS = "Only students can ask queries."
MSG_LLM_NO_ASSIGNMENT = "No assignment found for this student."
MSG_LLM_IRRELEVANT = ("Your query does not relate to your assignment. "
                      "Please ask a question related to your assignment.")
MSG_UNAVAILABLE = "The LMS cluster is unavailable (no leader). Please retry."
MSG_TUTOR_UNAVAILABLE = "The tutoring service is unavailable. Please retry later."
MSG_TUTOR_BUSY = "The tutoring service is busy. Please retry in a moment."


class TutoringClient:
    """Client of the tutoring tier.  ``address`` may list several tutoring replicas (one per GPU or
    TP group, comma-separated): a query goes to the replica with the fewest queries in flight and
    fails over to the next one when a replica is unreachable (UNAVAILABLE / connection errors
    mark it down for ``down_s``), so a dead tutoring process costs one retry, not an outage.
    The reference has one module-level channel to a hard-coded address (``lms_server.py:39-40``)."""

    RETRY_CODES = (grpc.StatusCode.UNAVAILABLE, grpc.StatusCode.CANCELLED)
    # an overloaded replica refuses at once (its admission queue is full): try the others, but it
    # is healthy -- not marked down
    BUSY_CODES = (grpc.StatusCode.RESOURCE_EXHAUSTED,)

    def __init__(self, address, timeout: float = 120.0, down_s: float = 2.0, aio_connections: int = 4):
        addrs = address.split(",") if isinstance(address, str) else list(address)
        self.addresses = [a.strip() for a in addrs if a.strip()]
        if not self.addresses:
            raise ValueError("no tutoring address")
        self.address = self.addresses[0]
        self.timeout = timeout
        self.down_s = down_s
        self._channels = [wire.channel(a) for a in self.addresses]
        self._stubs = [wire.Stub("Tutoring", c) for c in self._channels]
        self._inflight = [0] * len(self.addresses)
        self._down_until = [0.0] * len(self.addresses)
        self._lock = threading.Lock()
        self._aio_channels = self._aio_stubs = None
        self.aio_connections = max(1, aio_connections)

    def _order(self) -> list[int]:
        now = time.monotonic()
        with self._lock:
            up = [i for i in range(len(self.addresses)) if self._down_until[i] <= now]
            down = [i for i in range(len(self.addresses)) if self._down_until[i] > now]
            up.sort(key=lambda i: self._inflight[i])
        return up + down  # down replicas last: still tried if nothing else answers

    def ask(self, token: str, query: str) -> pb.QueryResponse:
        last = None
        for i in self._order():
            with self._lock:
                self._inflight[i] += 1
            try:
                return self._stubs[i].GetLLMAnswer(pb.QueryRequest(token=token, query=query), timeout=self.timeout)
            except grpc.RpcError as e:
                last = e
                if e.code() in self.BUSY_CODES:
                    METRICS.inc("tutor_busy_total")
                    continue
                if e.code() not in self.RETRY_CODES:
                    raise
                METRICS.inc("tutor_failover_total")
                log.warning("tutoring replica %s unavailable, failing over", self.addresses[i])
                with self._lock:
                    self._down_until[i] = time.monotonic() + self.down_s
            finally:
                with self._lock:
                    self._inflight[i] -= 1
        raise last

    async def ask_async(self, token: str, query: str) -> pb.QueryResponse:
        """``ask`` on ``grpc.aio`` channels (created on first use, on the calling event loop)."""
        if self._aio_stubs is None:
            # ``aio_connections`` connections per replica (own subchannel pools): a replica's
            # front-end processes share its port through SO_REUSEPORT, which balances connections
            opts = list(wire.CHANNEL_OPTIONS) + [("grpc.use_local_subchannel_pool", 1)]
            self._aio_channels = [[grpc.aio.insecure_channel(a, options=opts) for _ in range(self.aio_connections)]
                                  for a in self.addresses]
            self._aio_stubs = [[wire.Stub("Tutoring", c) for c in cs] for cs in self._aio_channels]
            self._rr = 0
        last = None
        for i in self._order():
            with self._lock:
                self._inflight[i] += 1
            try:
                self._rr += 1
                stub = self._aio_stubs[i][self._rr % self.aio_connections]
                return await stub.GetLLMAnswer(pb.QueryRequest(token=token, query=query), timeout=self.timeout)
            except grpc.RpcError as e:
                last = e
                if e.code() in self.BUSY_CODES:
                    METRICS.inc("tutor_busy_total")
                    continue
                if e.code() not in self.RETRY_CODES:
                    raise
                METRICS.inc("tutor_failover_total")
                log.warning("tutoring replica %s unavailable, failing over", self.addresses[i])
                with self._lock:
                    self._down_until[i] = time.monotonic() + self.down_s
            finally:
                with self._lock:
                    self._inflight[i] -= 1
        raise last

    async def aclose(self):
        for cs in self._aio_channels or ():
            for c in cs:
                await c.close()
        self._aio_channels = self._aio_stubs = None

    def close(self):
        for c in self._channels:
            c.close()


_SLOW = object()  # _llm_prelude_fast: "run the full prelude on the worker pool"


def _tutor_error_message(e: grpc.RpcError) -> str:
    """What the student sees when the tutoring tier fails: every replica refusing for load is
    "busy" (retry soon), anything else "unavailable"."""
    code = e.code() if hasattr(e, "code") else None
    if code == grpc.StatusCode.RESOURCE_EXHAUSTED:
        METRICS.inc("llm_answer_busy_total")
        return MSG_TUTOR_BUSY
    return MSG_TUTOR_UNAVAILABLE


class LMSServicer:
    def __init__(self, node, state, addresses: dict[int, str], tutor: TutoringClient | None = None, gate=None,
                 write_timeout: float = 5.0, forward_timeout: float = 130.0, replicator=None):
        self.node = node
        self.state = state
        self.replicator = replicator  # lms.blobs.BlobReplicator (None: single node / tests)
        self.addresses = addresses
        self.tutor = tutor
        self.gate = gate
        self.write_timeout = write_timeout
        self.forward_timeout = forward_timeout
        self._leader_stubs: dict[int, wire.Stub] = {}

    # ------------------------------------------------------------------ plumbing
    def _forward(self, method: str, request, context):
        """If this node is not the leader, relay the call to the leader.  Returns the leader's
        response, or None when the call should be served here."""
        if self.node.is_leader:
            return None
        md = dict(context.invocation_metadata() or ())
        if md.get(FORWARD_HEADER):
            return None
        lid = self.node.leader_id
        if lid is None or lid not in self.addresses:
            return None
        stub = self._leader_stubs.get(lid)
        if stub is None:
            stub = wire.Stub("LMS", wire.channel(self.addresses[lid]))
            self._leader_stubs[lid] = stub
        meta = [(FORWARD_HEADER, "1")]
        if md.get(REQUEST_ID_HEADER):
            meta.append((REQUEST_ID_HEADER, md[REQUEST_ID_HEADER]))
        try:
            METRICS.inc("lms_forwarded_total")
            return getattr(stub, method)(request, timeout=self.forward_timeout, metadata=tuple(meta))
        except grpc.RpcError as e:
            log.warning("forward %s to leader %s failed: %s", method, lid, e.code())
            return None

    @staticmethod
    def _rid(context, suffix: str = "") -> str | None:
        md = dict(context.invocation_metadata() or ()) if context is not None else {}
        rid = md.get(REQUEST_ID_HEADER)
        return f"{rid}{suffix}" if rid else None

    def _write(self, op: str, args: list, rid: str | None = None):
        return self.node.propose(commands.encode(op, args, rid), timeout=self.write_timeout)

    def _write_many(self, items: list[tuple], rid: str | None = None):
        """(operation, args[, meta]) items proposed back to back."""
        futs = [self.node.submit(commands.encode(it[0], it[1], f"{rid}.{k}" if rid else None,
                                                 it[2] if len(it) > 2 else None))
                for k, it in enumerate(items)]
        return [f.result(timeout=self.write_timeout) for f in futs]

    def _read_fence(self):
        if self.node.is_leader:
            self.node.read_barrier(self.write_timeout)

    def _session(self, token: str):
        # fenced: a leader elected a moment ago may not have applied the Login entry its
        # predecessor committed -- the token must still be valid right after a failover
        self._read_fence()
        return self.state.session(token)

    def _store_upload(self, filename: str, blob: bytes):
        """Pre-replicate an upload (content-addressed) to a majority, then return the small
        ``PutBlob`` log item that makes it part of the replicated state."""
        sha = self.state.blobs.put_bytes(blob)
        if self.replicator is not None and not self.replicator.replicate(sha, len(self.addresses)):
            raise TimeoutError(f"upload {filename!r} did not reach a majority")
        return ("PutBlob", [filename, sha, len(blob)])

    # ------------------------------------------------------------------ auth
    def Register(self, request, context):
        fwd = self._forward("Register", request, context)
        if fwd is not None:
            return fwd
        self._read_fence()
        rid = self._rid(context)
        done, first = self.state.rid_result(rid)
        if not done and self.state.read(lambda d: request.username in d["users"]):
            return pb.RegisterResponse(success=False, message=MSG_USER_EXISTS)
        try:
            ok = first if done else self._write("Register", [request.username, request.password, request.role], rid)
        except (NotLeader, TimeoutError, Exception):
            return pb.RegisterResponse(success=False, message=MSG_UNAVAILABLE)
        if not ok:
            return pb.RegisterResponse(success=False, message=MSG_USER_EXISTS)
        return pb.RegisterResponse(success=True, message=MSG_REGISTER_OK)

    def Login(self, request, context):
        fwd = self._forward("Login", request, context)
        if fwd is not None:
            return fwd
        self._read_fence()
        user = self.state.read(lambda d: dict(d["users"][request.username]) if request.username in d["users"] else None)
        if user is None or user["password"] != request.password:
            return pb.LoginResponse(success=False)
        # with a client request id the token is derived from it, so a retried Login (reply lost)
        # is deduplicated by the state machine and returns the SAME session instead of minting a
        # second one
        rid = self._rid(context)
        token = str(uuid.uuid5(uuid.NAMESPACE_URL, f"dlms-login/{request.username}/{rid}")) if rid else str(uuid.uuid4())
        try:
            self._write("Login", [request.username, token, user["role"]], rid)
        except Exception:
            return pb.LoginResponse(success=False)
        return pb.LoginResponse(success=True, token=token, role=user["role"])

    def Logout(self, request, context):
        fwd = self._forward("Logout", request, context)
        if fwd is not None:
            return fwd
        rid = self._rid(context)
        self._read_fence()
        done, first = self.state.rid_result(rid)
        if done:  # a retry of a Logout that already committed: the same answer
            return pb.LogoutResponse(success=bool(first))
        if self._session(request.token) is None:
            return pb.LogoutResponse(success=False)
        try:
            ok = self._write("Logout", [request.token], rid)
        except Exception:
            return pb.LogoutResponse(success=False)
        return pb.LogoutResponse(success=bool(ok))

    # ------------------------------------------------------------------ course workflows
    def Post(self, request, context):
        fwd = self._forward("Post", request, context)
        if fwd is not None:
            return fwd
        s = self._session(request.token)
        if s is None:
            return pb.PostResponse(success=False)
        user, role = s["username"], s["role"]
        rid = self._rid(context)
        try:
            # (the entry carries its upload's sha as a command field: a later same-named upload
            # replaces uploads/<name> but not what this entry downloads)
            if role == "instructor" and request.type == "course_material":
                path = self.state.blobs.relpath(request.filename)
                put = self._store_upload(request.filename, bytes(request.file))
                self._write_many([put, ("PostCourseMaterial", [user, request.filename, path],
                                        {"sha256": put[1][1]})], rid)
                return pb.PostResponse(success=True)
            if role == "student" and request.type == "assignment":
                blob = bytes(request.file)
                text = extract_text(blob, TEXT_CAP)
                path = self.state.blobs.relpath(request.filename)
                put = self._store_upload(request.filename, blob)
                self._write_many([put, ("PostAssignment", [user, request.filename, path, text],
                                        {"sha256": put[1][1]})], rid)
                return pb.PostResponse(success=True)
            if role == "student" and request.type == "query":
                self._write("AskQuery", [user, request.data], rid)
                return pb.PostResponse(success=True)
        except Exception as e:
            log.warning("Post failed: %s", e)
        return pb.PostResponse(success=False)

    def Get(self, request, context):
        fwd = self._forward("Get", request, context)
        if fwd is not None:
            return fwd
        s = self._session(request.token)
        if s is None:
            return pb.GetResponse(success=False)
        self._read_fence()
        if request.type == "course_material" and s["role"] == "student":
            mats = self.state.read(lambda d: [(m["filename"], m["filepath"], m.get("instructor", "Unknown"),
                                               m.get("sha256")) for m in d["course_materials"]])
            if not mats:
                return pb.GetResponse(success=True, message=MSG_NO_MATERIALS)
            return pb.GetResponse(success=True, entries=[
                pb.DataEntry(id="1", filename=f, file=self.state.read_blob(p, sha), instructor=ins)
                for f, p, ins, sha in mats])
        if s["role"] == "instructor" and request.type == "student_list":
            rows = self.state.read(lambda d: [(st, a["filename"], a["filepath"], a.get("sha256"))
                                              for st, items in d["assignments"].items() for a in items])
            return pb.GetResponse(success=True, entries=[
                pb.DataEntry(id=st, filename=f, file=self.state.read_blob(p, sha)) for st, f, p, sha in rows])
        return pb.GetResponse(success=False, message=MSG_BAD_GET)

    def GradeAssignment(self, request, context):
        fwd = self._forward("GradeAssignment", request, context)
        if fwd is not None:
            return fwd
        s = self._session(request.token)
        if s is None:
            return pb.GradeResponse(success=False, message=MSG_BAD_TOKEN)
        if s["role"] != "instructor":
            return pb.GradeResponse(success=False, message=MSG_ONLY_INSTRUCTORS_GRADE)
        self._read_fence()
        if not self.state.read(lambda d: request.studentId in d["assignments"]):
            return pb.GradeResponse(success=False, message=MSG_NO_STUDENT_ASSIGNMENT)
        try:
            self._write("GradeAssignment", [request.studentId, request.grade], self._rid(context))
        except Exception:
            return pb.GradeResponse(success=False, message=MSG_UNAVAILABLE)
        return pb.GradeResponse(success=True, message=MSG_GRADE_OK)

    def GetGrade(self, request, context):
        fwd = self._forward("GetGrade", request, context)
        if fwd is not None:
            return fwd
        s = self._session(request.token)
        if s is None:
            return pb.GetGradeResponse(success=False, grade=MSG_INVALID_SESSION)
        if s["role"] != "student":
            return pb.GetGradeResponse(success=False, grade=MSG_ONLY_STUDENTS_GRADES)
        self._read_fence()
        user = s["username"]
        items = self.state.read(lambda d: [dict(a) for a in d["assignments"][user]] if user in d["assignments"] else None)
        if items is None:
            return pb.GetGradeResponse(success=True, grade=MSG_NO_ASSIGNMENTS)
        for a in items:
            if "grade" in a:
                if a["grade"] is None:
                    return pb.GetGradeResponse(success=True, grade=MSG_GRADE_NOT_ASSIGNED)
                return pb.GetGradeResponse(success=True, grade=f"Your grade: {a['grade']}")
        return pb.GetGradeResponse(success=True, grade=MSG_NO_GRADE)

    # ------------------------------------------------------------------ queries
    def GetUnansweredQueries(self, request, context):
        fwd = self._forward("GetUnansweredQueries", request, context)
        if fwd is not None:
            return fwd
        s = self._session(request.token)
        if s is None or s["role"] != "instructor":
            return pb.GetResponse(success=False)
        self._read_fence()
        rows = self.state.read(lambda d: [(st, q["query"]) for st, qs in d.get("queries", {}).items() for q in qs
                                          if "query" in q and "response" in q and not q["answered"]])
        return pb.GetResponse(success=True, entries=[pb.DataEntry(id=st, data=q) for st, q in rows])

    def RespondToQuery(self, request, context):
        fwd = self._forward("RespondToQuery", request, context)
        if fwd is not None:
            return fwd
        s = self._session(request.token)
        if s is None or s["role"] != "instructor":
            return pb.PostResponse(success=False)
        try:
            self._write("RespondToQuery", [s["username"], request.studentId, request.data], self._rid(context))
        except Exception:
            return pb.PostResponse(success=False)
        return pb.PostResponse(success=True)

    def GetInstructorResponse(self, request, context):
        fwd = self._forward("GetInstructorResponse", request, context)
        if fwd is not None:
            return fwd
        s = self._session(request.token)
        if s is None or s["role"] != "student":
            return pb.GetResponse(success=False)
        self._read_fence()
        user = s["username"]
        texts = self.state.read(lambda d: [f"Your Query: {q['query']}\nInstructor Response: {q['response']}"
                                           for q in d.get("queries", {}).get(user, []) if q.get("answered", False)])
        return pb.GetResponse(success=True, entries=[pb.DataEntry(id=user, data=t) for t in texts])

    # ------------------------------------------------------------------ LLM tutoring
    def _llm_prelude(self, request, context):
        """Everything of GetLLMAnswer before the tutoring call (session, assignment, relevance
        gate): a final ``QueryResponse``, or ``None`` when the query goes to the tutoring tier."""
        s = self._session(request.token)
        if s is None:
            # sessions replicate through the log; a brand-new token may not have reached this node yet
            fwd = self._forward("GetLLMAnswer", request, context)
            if fwd is not None:
                return fwd
            return pb.QueryResponse(success=True, response=MSG_LLM_INVALID_SESSION)
        if s["role"] != "student":
            return pb.QueryResponse(success=True, response=MSG_LLM_ONLY_STUDENTS)
        user = s["username"]
        assignment_text = self.state.read(
            lambda d: d["assignments"][user][0]["text"] if d["assignments"].get(user) else None)
        if assignment_text is None:
            # a follower may not have applied an assignment its leader just committed: ask the
            # leader (which fences its reads) before answering "no assignment"
            if not self.node.is_leader:
                fwd = self._forward("GetLLMAnswer", request, context)
                if fwd is not None:
                    return fwd
            return pb.QueryResponse(success=True, response=MSG_LLM_NO_ASSIGNMENT)
        if self.gate is not None:
            tg = time.perf_counter()
            relevant, sim = self.gate.check(request.query, assignment_text)
            METRICS.observe("gate_ms", (time.perf_counter() - tg) * 1e3)
            TRACER.complete("lms.gate", tg, cat="lms", similarity=round(float(sim), 4), relevant=bool(relevant))
            METRICS.observe("gate_similarity", sim)
            if not relevant:
                METRICS.inc("gate_rejected_total")
                return pb.QueryResponse(success=True, response=MSG_LLM_IRRELEVANT)
        if self.tutor is None:
            return pb.QueryResponse(success=True, response=MSG_TUTOR_UNAVAILABLE)
        return None

    def _llm_prelude_fast(self, request):
        """The common case of ``_llm_prelude`` without blocking the event loop: a student session
        present on this node (a leader only once its read fence is already satisfied) with an
        assignment.  Returns ``_SLOW`` when the full prelude must run on the pool (unknown token
        or no assignment here -- possibly a forward to the leader --, an unfenced leader, a gate
        without ``check_async``), the assignment text when the gate is to decide, else the final
        response or None (no gate: straight to the tutoring tier)."""
        if self.gate is not None and not hasattr(self.gate, "check_async"):
            return _SLOW
        if self.node.is_leader and not self.node.read_ready():
            return _SLOW
        s = self.state.session(request.token)
        if s is None:
            return _SLOW
        if s["role"] != "student":
            return pb.QueryResponse(success=True, response=MSG_LLM_ONLY_STUDENTS)
        user = s["username"]
        text = self.state.read(lambda d: d["assignments"][user][0]["text"] if d["assignments"].get(user) else None)
        if text is None:
            return _SLOW
        if self.gate is not None:
            return text
        return None if self.tutor is not None else pb.QueryResponse(success=True, response=MSG_TUTOR_UNAVAILABLE)

    async def _gate_async(self, request, assignment_text: str):
        tg = time.perf_counter()
        relevant, sim = await self.gate.check_async(request.query, assignment_text)
        METRICS.observe("gate_ms", (time.perf_counter() - tg) * 1e3)
        TRACER.complete("lms.gate", tg, cat="lms", similarity=round(float(sim), 4), relevant=bool(relevant))
        METRICS.observe("gate_similarity", sim)
        if not relevant:
            METRICS.inc("gate_rejected_total")
            return pb.QueryResponse(success=True, response=MSG_LLM_IRRELEVANT)
        if self.tutor is None:
            return pb.QueryResponse(success=True, response=MSG_TUTOR_UNAVAILABLE)
        return None

    def _llm_done(self, t0: float, tt: float):
        TRACER.complete("lms.tutor_call", tt, cat="lms")
        TRACER.complete("lms.GetLLMAnswer", t0, cat="lms")
        METRICS.observe("llm_answer_ms", (time.perf_counter() - t0) * 1e3)

    def GetLLMAnswer(self, request, context):
        t0 = time.perf_counter()
        early = self._llm_prelude(request, context)
        if early is not None:
            return early
        tt = time.perf_counter()
        try:
            resp = self.tutor.ask(request.token, request.query)
        except grpc.RpcError as e:
            log.warning("tutoring call failed: %s", e.code())
            return pb.QueryResponse(success=True, response=_tutor_error_message(e))
        self._llm_done(t0, tt)
        return resp

    async def GetLLMAnswerAsync(self, request, context):
        """GetLLMAnswer for the ``grpc.aio`` front end (LMSServer ``frontend="aio"``): the session
        and assignment reads run on the event loop (a lock-protected dict lookup each), the
        batched relevance gate and the long tutoring call are awaited -- a query in flight holds
        no thread at all, so one LMS node carries thousands of concurrent tutoring queries and the
        worker pool stays free for the Raft RPCs.  Only the rare slow cases (a follower's forward
        to the leader, a fenced read that has to wait) go to the pool, through ``_llm_prelude``."""
        import asyncio

        t0 = time.perf_counter()
        fast = self._llm_prelude_fast(request)
        if fast is _SLOW:
            early = await asyncio.get_running_loop().run_in_executor(None, self._llm_prelude, request, context)
        elif isinstance(fast, str):  # the assignment text: the gate decides
            early = await self._gate_async(request, fast)
        else:
            early = fast
        if early is not None:
            return early
        tt = time.perf_counter()
        try:
            resp = await self.tutor.ask_async(request.token, request.query)
        except grpc.RpcError as e:
            log.warning("tutoring call failed: %s", e.code())
            return pb.QueryResponse(success=True, response=_tutor_error_message(e))
        self._llm_done(t0, tt)
        return resp

    def WhoIsLeader(self, request, context):
        lid = self.node.leader_id
        return pb.LeaderResponse(leader_id=lid if lid is not None else -1)


class FileTransferServicer:
    """``lms.FileTransferService.SendFile``: a reference server can still stream an upload to us.
    Writes land under ``uploads/`` only (the client-supplied path is reduced to its basename),
    atomically and idempotently -- the reference appended (``'ab'``), duplicating bytes on retry."""

    def __init__(self, state):
        self.state = state

    def SendFile(self, request_iterator, context):
        """``destination_path = "cas/<sha256>"``: a leader's pre-replication push (lms/blobs.py),
        streamed to disk chunk by chunk and verified against the hash; any other path: the
        reference's upload to ``uploads/<basename>``."""
        it = iter(request_iterator)
        try:
            first = next(it, None)
            if first is None:
                return pb.FileTransferResponse(status="Error receiving file: empty stream")
            name = first.destination_path

            def chunks():
                yield first.content
                for c in it:
                    yield c.content

            blobs = self.state.blobs
            if name.startswith("cas/"):
                blobs.put_chunks(name[4:], chunks())
            else:
                blobs.put(name, b"".join(chunks()))
            return pb.FileTransferResponse(status="File received successfully")
        except Exception as e:  # mirror the reference's error reporting
            return pb.FileTransferResponse(status=f"Error receiving file: {e}")
