#!/usr/bin/env python3
"""Per-phase timing of the persistent dataflow decode from its in-kernel wall-clock stamps
(ops/dataflow.py trace buffer): where each layer's time goes on the critical path."""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

EV = {0: "layer_start", 1: "e1_ok", 2: "ln1_ready", 3: "qkv_done", 4: "qkv_published", 5: "gran_ok",
      6: "attn_done", 7: "attn_published", 8: "e3_ok", 9: "ln2_ready", 10: "mlp_done", 11: "mlp_published",
      12: "ring_wait_ticks"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2")
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--step", type=int, default=2)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    from distributed_lms_raft_llm_amd.engine.gpt2_engine import HipGPT2Engine
    from distributed_lms_raft_llm_amd.models.config import gpt2_config
    from distributed_lms_raft_llm_amd.models.gpt2 import init_gpt2_weights

    cfg = gpt2_config(args.model)
    os.environ["DLMS_DATAFLOW"] = "1"
    os.environ["DLMS_DATAFLOW_ROWS"] = "2"
    eng = HipGPT2Engine(cfg, init_gpt2_weights(cfg, seed=0), max_batch=2, max_length=150)
    g = torch.Generator().manual_seed(1)
    prompts = torch.randint(0, cfg.vocab_size - 1, (args.batch, 32), generator=g).tolist()
    eng.generate(prompts)
    df = eng._df
    tr = df.trace_buffer()
    B = args.batch
    eng._prefill(prompts, B, 1.2)
    torch.cuda.synchronize()
    import time
    t0 = time.perf_counter()
    df.run(B, 8, 1.2, trace=tr)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) * 1e3
    df.check()
    t = tr.cpu().numpy().astype(np.float64) / 100.0  # -> microseconds
    s = args.step
    L = cfg.n_layer
    att = np.array([cu.ah >= 0 for cu in df.cus])
    rows = []
    for l in range(L):
        x = t[:, s, l, :]
        med = lambda e, m=None: float(np.median(x[m if m is not None else slice(None), e]))  # noqa: E731
        prev_pub = float(np.max(t[:, s, l - 1, 11])) if l > 0 else float("nan")
        r = {"layer": l,
             "e1_edge_us": round(med(1) - prev_pub, 2) if l > 0 else None,
             "e1_spread_us": round(float(np.max(x[:, 1]) - np.min(x[:, 1])), 2),
             "ln1_us": round(float(np.median(x[:, 2] - x[:, 1])), 2),
             "qkv_us": round(float(np.median(x[:, 3] - x[:, 2])), 2),
             "qkv_pub_us": round(float(np.median(x[:, 4] - x[:, 3])), 2),
             "gran_edge_us": round(float(np.median(x[att, 5]) - np.max(x[:, 4])), 2),
             "attn_us": round(float(np.median(x[att, 6] - x[att, 5])), 2),
             "attn_pub_us": round(float(np.median(x[att, 7] - x[att, 6])), 2),
             "e3_edge_us": round(med(8) - float(np.max(x[att, 7])), 2),
             "ln2_us": round(float(np.median(x[:, 9] - x[:, 8])), 2),
             "mlp_us": round(float(np.median(x[:, 10] - x[:, 9])), 2),
             "mlp_max_us": round(float(np.max(x[:, 10] - x[:, 9])), 2),
             "mlp_pub_us": round(float(np.median(x[:, 11] - x[:, 10])), 2),
             "mlp_pub_max_us": round(float(np.max(x[:, 11] - x[:, 10])), 2),
             "ring_wait_us": round(float(np.median(x[:, 12])) / 1.0, 2),
             "ld_resid3_us": round(float(np.median(x[:, 25] - x[:, 8])), 2),
             "cw_qkv_seen_us": round(float(np.median(x[:, 16] - x[:, 2])), 2),
             "cw_qkv_rows_us": round(float(np.median(x[:, 17] - x[:, 16])), 2),
             "cw_attn_seen_us": round(float(np.median(x[att, 18] - x[att, 5])), 2),
             "cw_attn_core_us": round(float(np.median(x[att, 19] - x[att, 18])), 2),
             "cw_merge_us": round(float(np.median(x[att, 20] - x[att, 19])), 2),
             "cw_wo_us": round(float(np.median(x[att, 21] - x[att, 20])), 2),
             "cw_mlp_seen_us": round(float(np.median(x[:, 22] - x[:, 9])), 2),
             "cw_mlp_rows_us": round(float(np.median(x[:, 23] - x[:, 22])), 2),
             "layer_us": round(float(np.median(t[:, s, l + 1, 0] if l + 1 < L else t[:, s, L, 0]) - med(0)), 2)}
        rows.append(r)
    lm = t[:, s, L, :]
    lmr = {"lm_ln_ready_us": round(float(np.median(lm[:, 1] - lm[:, 0])), 2),
           "lm_compute_us": round(float(np.median(lm[:, 2] - lm[:, 1])), 2),
           "lm_compute_max_us": round(float(np.max(lm[:, 2] - lm[:, 1])), 2),
           "lm_pub_us": round(float(np.median(lm[:, 3] - lm[:, 2])), 2),
           "lm_edge_us": round(float(np.median(lm[:, 4]) - np.max(lm[:, 3])), 2),
           "lm_ring_wait_us": round(float(np.median(lm[:, 12])), 2),
           "step_us": round(float(np.median(t[:, s + 1, 0, 0] - t[:, s, 0, 0])), 2) if s + 1 < 4 else None,
           "wall_ms_8_steps": round(wall, 3),
           "shader_mhz": round(float(np.median((t[:, s, L, 26] - t[:, s, 0, 26]) / (t[:, s, L, 27] - t[:, s, 0, 27]) * 100.0)), 1),
           "lm_cw0_wait_cycles": float(np.median(t[:, s, L, 28] * 100)),
           "lm_cw0_body_cycles": float(np.median(t[:, s, L, 29] * 100)),
           "lm_cw0_total_cycles": float(np.median(t[:, s, L, 30] * 100))}
    out = {"model": args.model, "batch": B, "step": s, "layers": rows, "lm": lmr}
    for r in rows:
        print(json.dumps(r))
    print(json.dumps(lmr))
    if args.out:
        np.save(args.out.replace(".json", ".npy"), tr.cpu().numpy())
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
