"""Drop-in replacement for the grpc-generated ``lms_pb2_grpc`` module (reference
``lms_pb2_grpc.py``): for every service S of ``lms.proto`` -- ``SStub(channel)``, the
``SServicer`` base class (every method answers UNIMPLEMENTED until overridden),
``add_SServicer_to_server(servicer, server)`` and the experimental static-call class ``S`` (the
reference tutoring server subclasses ``lms_pb2_grpc.Tutoring``).  Method paths and serializers
are the generated module's, so stubs and servers interoperate with either implementation."""
import grpc

from . import METHODS, method_path
from .schema import PACKAGE


def _make(service: str):
    methods = METHODS[service]

    def stub_init(self, channel):
        for meth, (req, resp, cstream) in methods.items():
            factory = channel.stream_unary if cstream else channel.unary_unary
            setattr(self, meth, factory(method_path(service, meth), request_serializer=req.SerializeToString,
                                        response_deserializer=resp.FromString))

    stub = type(f"{service}Stub", (object,), {"__init__": stub_init, "__doc__": f"Client stub of lms.{service}."})

    def unimplemented(self, request, context):
        context.set_code(grpc.StatusCode.UNIMPLEMENTED)
        context.set_details("Method not implemented!")
        raise NotImplementedError("Method not implemented!")

    servicer = type(f"{service}Servicer", (object,), {m: unimplemented for m in methods})

    def add_to_server(svc, server):
        handlers = {}
        for meth, (req, resp, cstream) in methods.items():
            make = grpc.stream_unary_rpc_method_handler if cstream else grpc.unary_unary_rpc_method_handler
            handlers[meth] = make(getattr(svc, meth), request_deserializer=req.FromString,
                                  response_serializer=resp.SerializeToString)
        server.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(f"{PACKAGE}.{service}", handlers),))

    def static_call(meth, req, resp, cstream):
        def call(request, target, options=(), channel_credentials=None, call_credentials=None, insecure=False,
                 compression=None, wait_for_ready=None, timeout=None, metadata=None):
            with grpc.insecure_channel(target, options=list(options)) as ch:
                factory = ch.stream_unary if cstream else ch.unary_unary
                fn = factory(method_path(service, meth), request_serializer=req.SerializeToString,
                             response_deserializer=resp.FromString)
                return fn(request, timeout=timeout, metadata=metadata, compression=compression,
                          wait_for_ready=wait_for_ready)

        return staticmethod(call)

    experimental = type(service, (object,), {m: static_call(m, *spec) for m, spec in methods.items()})
    return stub, servicer, add_to_server, experimental


for _service in METHODS:
    _stub, _servicer, _add, _exp = _make(_service)
    globals()[f"{_service}Stub"] = _stub
    globals()[f"{_service}Servicer"] = _servicer
    globals()[f"add_{_service}Servicer_to_server"] = _add
    globals()[_service] = _exp
