#!/usr/bin/env python3
"""CLI-compatible entry point: ``python lms_server.py <id> <port> <peer_address>...``
(see ``distributed_lms_raft_llm_amd/lms/server.py`` for the optional flags)."""
from distributed_lms_raft_llm_amd.lms.server import main

if __name__ == "__main__":
    main()
