"""Runtime-compiled ``lms`` protobuf messages and gRPC plumbing (no protoc needed).

``pb``      -- a namespace exposing one message class per ``lms.proto`` message (``pb.LoginRequest``...),
               drop-in for the generated ``lms_pb2`` module.
``Stub``    -- client stubs per service (``Stub("LMS", channel).Login(req, timeout=...)``).
``register``-- attach a servicer object to a ``grpc.Server`` via generic handlers.

Method paths are ``/lms.<Service>/<Method>``, identical to the reference's generated stubs
(``lms_pb2_grpc.py``), so either side can be swapped for the reference implementation.
"""
from __future__ import annotations

import types

import grpc
from google.protobuf import descriptor_pool, message_factory

from .schema import MESSAGES, PACKAGE, SERVICES, build_file_descriptor_proto

_POOL = descriptor_pool.DescriptorPool()
FILE_DESCRIPTOR = _POOL.Add(build_file_descriptor_proto())

pb = types.SimpleNamespace()
for _name, _ in MESSAGES:
    setattr(pb, _name, message_factory.GetMessageClass(_POOL.FindMessageTypeByName(f"{PACKAGE}.{_name}")))

METHODS: dict[str, dict[str, tuple]] = {
    s: {m: (getattr(pb, req), getattr(pb, resp), cs) for m, req, resp, cs in methods} for s, methods in SERVICES
}

DEFAULT_MAX_MESSAGE = 50 * 1024 * 1024  # the reference's 50 MiB limits (lms_server.py:1577-1578)
CHANNEL_OPTIONS = [
    ("grpc.max_send_message_length", DEFAULT_MAX_MESSAGE),
    ("grpc.max_receive_message_length", DEFAULT_MAX_MESSAGE),
]


def method_path(service: str, method: str) -> str:
    return f"/{PACKAGE}.{service}/{method}"


class Stub:
    """Client stub for one ``lms`` service on a channel."""

    def __init__(self, service: str, channel: grpc.Channel):
        if service not in METHODS:
            raise ValueError(f"unknown service {service}")
        self._service = service
        for meth, (req, resp, cstream) in METHODS[service].items():
            factory = channel.stream_unary if cstream else channel.unary_unary
            setattr(self, meth, factory(method_path(service, meth), request_serializer=req.SerializeToString,
                                        response_deserializer=resp.FromString))


def register(server: grpc.Server, service: str, servicer) -> None:
    """Register every method ``servicer`` implements (others answer UNIMPLEMENTED, like the
    generated base servicers do)."""
    handlers = {}
    for meth, (req, resp, cstream) in METHODS[service].items():
        fn = getattr(servicer, meth, None)
        if fn is None:
            continue
        make = grpc.stream_unary_rpc_method_handler if cstream else grpc.unary_unary_rpc_method_handler
        handlers[meth] = make(fn, request_deserializer=req.FromString, response_serializer=resp.SerializeToString)
    server.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(f"{PACKAGE}.{service}", handlers),))


def channel(address: str, max_message: int = DEFAULT_MAX_MESSAGE,
            reconnect_ms: tuple[int, int] | None = None) -> grpc.Channel:
    opts = [("grpc.max_send_message_length", max_message), ("grpc.max_receive_message_length", max_message)]
    if reconnect_ms is not None:
        opts += [("grpc.initial_reconnect_backoff_ms", reconnect_ms[0]),
                 ("grpc.min_reconnect_backoff_ms", reconnect_ms[0]),
                 ("grpc.max_reconnect_backoff_ms", reconnect_ms[1])]
    return grpc.insecure_channel(address, options=opts)
