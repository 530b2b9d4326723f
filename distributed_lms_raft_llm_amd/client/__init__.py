"""Programmatic LMS client: every workflow of the reference GUI (``lms_gui_final.py``, SURVEY.md
§2.6) without Tk, with leader discovery and transparent failover.

The GUI discovers the leader by polling ``RaftService.WhoIsLeader`` (5 rounds x N servers, 3 s
apart, no deadlines) before EVERY action (``lms_gui_final.py:64-185``).  ``LMSClient`` caches the
leader, re-discovers it only when a call fails with UNAVAILABLE / DEADLINE_EXCEEDED, and retries
the call, so a leader crash costs one election (~0.2-0.3 s here) instead of minutes.

Writes (Register, Post, GradeAssignment, RespondToQuery, Logout) carry a client request id
(``x-dlms-request-id`` metadata) that is the same on every retry of one logical call; the state
machine applies an id once (``lms/commands.py``), so retrying a write whose first attempt committed
before its reply was lost can never post twice or answer the student's NEXT query.
"""
from __future__ import annotations

import os
import time
import uuid

import grpc

from .. import wire
from ..wire import pb

RETRYABLE = {grpc.StatusCode.UNAVAILABLE, grpc.StatusCode.DEADLINE_EXCEEDED, grpc.StatusCode.CANCELLED,
             grpc.StatusCode.UNKNOWN}


class NoLeader(RuntimeError):
    pass


class LMSClient:
    def __init__(self, addresses: list[str], timeout: float = 10.0, llm_timeout: float = 300.0,
                 discover_timeout: float = 10.0):
        self.addresses = list(addresses)
        self.timeout = timeout
        self.llm_timeout = llm_timeout
        self.discover_timeout = discover_timeout
        self._channels: dict[str, grpc.Channel] = {}
        self.leader_address: str | None = None
        self.token: str | None = None
        self.role: str | None = None

    # ------------------------------------------------------------------ plumbing
    def _ch(self, addr: str) -> grpc.Channel:
        ch = self._channels.get(addr)
        if ch is None:
            ch = self._channels[addr] = wire.channel(addr)
        return ch

    def discover(self, avoid: str | None = None) -> str:
        """Ask the servers who leads; ignore answers naming ``avoid`` (a leader whose call just
        failed: followers keep naming it until their election timeout fires)."""
        end = time.time() + self.discover_timeout
        while time.time() < end:
            for addr in self.addresses:
                try:
                    lid = wire.Stub("RaftService", self._ch(addr)).WhoIsLeader(pb.Empty(), timeout=0.5).leader_id
                except grpc.RpcError:
                    continue
                if 1 <= lid <= len(self.addresses) and self.addresses[lid - 1] != avoid:
                    self.leader_address = self.addresses[lid - 1]
                    return self.leader_address
            time.sleep(0.05)
        raise NoLeader(f"no leader among {self.addresses}")

    WRITES = {"Register", "Post", "GradeAssignment", "RespondToQuery", "Logout"}

    def call(self, method: str, request, timeout: float | None = None, service: str = "LMS"):
        end = time.time() + self.discover_timeout
        avoid = None
        md = (("x-dlms-request-id", uuid.uuid4().hex),) if method in self.WRITES else None
        while True:
            addr = self.leader_address or self.discover(avoid)
            try:
                return getattr(wire.Stub(service, self._ch(addr)), method)(request, timeout=timeout or self.timeout,
                                                                           metadata=md)
            except grpc.RpcError as e:
                if e.code() not in RETRYABLE or time.time() >= end:
                    raise
                avoid, self.leader_address = addr, None
                time.sleep(0.02)

    def close(self):
        for ch in self._channels.values():
            ch.close()
        self._channels.clear()

    # ------------------------------------------------------------------ auth
    def register(self, username: str, password: str, role: str = "student"):
        return self.call("Register", pb.RegisterRequest(username=username, password=password, role=role))

    def login(self, username: str, password: str) -> bool:
        r = self.call("Login", pb.LoginRequest(username=username, password=password))
        if r.success:
            self.token, self.role = r.token, r.role
        return r.success

    def logout(self) -> bool:
        r = self.call("Logout", pb.LogoutRequest(token=self.token or ""))
        if r.success:
            self.token = self.role = None
        return r.success

    # ------------------------------------------------------------------ student
    def post_assignment(self, path: str | None = None, data: bytes | None = None, filename: str | None = None) -> bool:
        if data is None:
            with open(path, "rb") as f:
                data = f.read()
        name = filename or os.path.basename(path or "assignment.pdf")
        return self.call("Post", pb.PostRequest(token=self.token, type="assignment", file=data, filename=name)).success

    def course_materials(self):
        return self.call("Get", pb.GetRequest(token=self.token, type="course_material"))

    def grade(self) -> str:
        return self.call("GetGrade", pb.GetGradeRequest(token=self.token)).grade

    def ask_llm(self, query: str) -> str:
        return self.call("GetLLMAnswer", pb.QueryRequest(token=self.token, query=query),
                         timeout=self.llm_timeout).response

    def ask_instructor(self, query: str) -> bool:
        return self.call("Post", pb.PostRequest(token=self.token, type="query", data=query)).success

    def instructor_responses(self) -> list[str]:
        return [e.data for e in self.call("GetInstructorResponse", pb.GetRequest(token=self.token)).entries]

    # ------------------------------------------------------------------ instructor
    def post_course_material(self, path: str | None = None, data: bytes | None = None,
                             filename: str | None = None) -> bool:
        if data is None:
            with open(path, "rb") as f:
                data = f.read()
        name = filename or os.path.basename(path or "material.pdf")
        return self.call("Post", pb.PostRequest(token=self.token, type="course_material", file=data,
                                                filename=name)).success

    def assignments(self):
        return self.call("Get", pb.GetRequest(token=self.token, type="student_list"))

    def grade_assignment(self, student: str, grade: str):
        return self.call("GradeAssignment", pb.GradeRequest(token=self.token, studentId=student, grade=grade))

    def unanswered_queries(self) -> list[tuple[str, str]]:
        return [(e.id, e.data) for e in self.call("GetUnansweredQueries", pb.GetRequest(token=self.token)).entries]

    def respond(self, student: str, text: str) -> bool:
        return self.call("RespondToQuery", pb.PostRequest(token=self.token, studentId=student, data=text)).success
