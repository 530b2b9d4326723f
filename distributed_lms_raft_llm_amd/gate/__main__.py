"""``python -m distributed_lms_raft_llm_amd.gate``: the GPU tier's relevance gate server."""
from .service import main

main()
