"""``import lms_pb2`` for clients of the reference (e.g. ``lms_gui_final.py``): the runtime-built
messages of this framework (``distributed_lms_raft_llm_amd/wire/lms_pb2.py``)."""
from distributed_lms_raft_llm_amd.wire.lms_pb2 import *  # noqa: F401,F403
from distributed_lms_raft_llm_amd.wire.lms_pb2 import DESCRIPTOR  # noqa: F401
