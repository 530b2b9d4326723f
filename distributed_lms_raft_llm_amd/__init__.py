"""MI355X-native distributed LMS with Raft replication and GPT-2 tutoring (see README.md)."""
import os as _os

# Cross-process GPU memory sharing (RCCL's peer buffers, the xGMI one-shot collectives' IPC-mapped
# slabs, parallel/xgmi.py) goes through dmabuf IPC: the legacy IPC mode is not supported by this
# platform's driver (hipIpcGetMemHandle fails with "invalid argument").  HIP reads the variable at
# runtime initialisation, so it is set here -- on import, before any GPU call of the tutor, the
# bench or the tests -- unless the operator set it explicitly.
_os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
