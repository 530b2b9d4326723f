"""``import lms_pb2_grpc`` for clients of the reference (e.g. ``lms_gui_final.py``): stubs,
servicer bases and ``add_*_to_server`` of this framework (``wire/lms_pb2_grpc.py``)."""
from distributed_lms_raft_llm_amd.wire.lms_pb2_grpc import *  # noqa: F401,F403
