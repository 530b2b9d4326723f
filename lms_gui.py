#!/usr/bin/env python3
"""Desktop client for the LMS cluster: ``python lms_gui.py --servers h1:50051,h2:50052,h3:50053``.
(The reference's ``lms_gui_final.py`` also connects unchanged; see distributed_lms_raft_llm_amd/gui.)"""
from distributed_lms_raft_llm_amd.gui import main

if __name__ == "__main__":
    main()
