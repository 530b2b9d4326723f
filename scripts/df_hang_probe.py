#!/usr/bin/env python3
"""Where a dataflow-decode launch stalls: run a few steps with the stamp buffer on and report,
per CU, the last (layer, event) its comm wave stamped, plus the error word (ops/dataflow.py).
Variants over the grid size localise co-residency / partition-dependent hand-off bugs."""
import argparse
import collections
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2-medium")
    ap.add_argument("--grids", default="256,192,128")
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    os.environ["DLMS_DATAFLOW"] = "1"
    os.environ["DLMS_DATAFLOW_ROWS"] = "2"
    from distributed_lms_raft_llm_amd.engine.gpt2_engine import HipGPT2Engine
    from distributed_lms_raft_llm_amd.models.config import gpt2_config
    from distributed_lms_raft_llm_amd.models.gpt2 import init_gpt2_weights
    from distributed_lms_raft_llm_amd.ops.dataflow import ERRORS, DataflowDecoder

    cfg = gpt2_config(args.model)
    eng = HipGPT2Engine(cfg, init_gpt2_weights(cfg, seed=0), max_batch=2, max_length=80)
    g = torch.Generator().manual_seed(1)
    prompts = torch.randint(0, cfg.vocab_size - 1, (args.batch, 24), generator=g).tolist()
    L = cfg.n_layer
    lines = []
    for G in [int(x) for x in args.grids.split(",")]:
        df = DataflowDecoder(eng, grid=G)
        eng._prefill(prompts, args.batch, 1.2)
        tr = df.trace_buffer()
        torch.cuda.synchronize()
        df.run(args.batch, args.steps, 1.2, trace=tr)
        torch.cuda.synchronize()
        e = df.err[:4].cpu().tolist()
        t = tr.cpu().numpy()
        last = []
        for b in range(G):
            best = (-1, -1, -1)
            for s in range(min(args.steps, t.shape[1])):
                for l in range(L + 1):
                    nz = np.nonzero(t[b, s, l, :12])[0]
                    if len(nz):
                        best = max(best, (s, l, int(nz.max())))
            last.append(best)
        hist = collections.Counter(last)
        cu = df.cus[e[1]] if e[0] else None
        line = {"model": args.model, "grid": G, "gs": df.GS, "ring_bytes": df.ring_bytes(args.batch),
                "max_nq": df.max_nq, "ko": df.ko, "kf": df.kf,
                "error": ERRORS.get(e[0], e[0]) if e[0] else None, "err_block": e[1], "err_step": e[2],
                "err_site": e[3],
                "err_cu": None if cu is None else {"nq": cu.nq, "nf": cu.nf, "nv": cu.nv, "ah": cu.ah, "nk": cu.nk},
                "err_block_last": list(last[e[1]]) if e[0] else None,
                "last_stamp_hist": {f"s{k[0]}l{k[1]}e{k[2]}": v for k, v in sorted(hist.items())}}
        print(json.dumps(line), flush=True)
        lines.append(line)
    if args.out:
        with open(args.out, "w") as f:
            for line in lines:
                f.write(json.dumps(line) + "\n")


if __name__ == "__main__":
    main()
