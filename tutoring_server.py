#!/usr/bin/env python3
"""CLI-compatible entry point: ``python tutoring_server.py`` serves lms.Tutoring on [::]:50054
with the MI355X GPT-2 engine (``--device cpu`` for the CPU reference engine)."""
from distributed_lms_raft_llm_amd.tutor.server import main

if __name__ == "__main__":
    main()
