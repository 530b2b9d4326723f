"""Drop-in replacement for the protoc-generated ``lms_pb2`` module (reference ``lms_pb2.py``):
``DESCRIPTOR`` plus one message class per ``lms.proto`` message, built at runtime from
``wire/schema.py`` (no protoc on the box).  Clients written against the generated module -- the
reference GUI ``lms_gui_final.py`` -- import this one unchanged (top-level ``lms_pb2.py`` shim)."""
from . import FILE_DESCRIPTOR as DESCRIPTOR
from . import pb as _pb
from .schema import MESSAGES as _MESSAGES

for _name, _ in _MESSAGES:
    globals()[_name] = getattr(_pb, _name)

__all__ = ["DESCRIPTOR"] + [n for n, _ in _MESSAGES]
