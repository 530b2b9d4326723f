"""BERT relevance-gate encoder on MI355X (K13-K17): packed variable-length batches, no padding.

Per layer (post-LN BERT):
    QKV GEMM (one [3H, H] weight; q out, k/v scattered per sequence) -> bidirectional attention
    -> out-proj (fp32 partials) -> fused residual-add + LayerNorm (eps 1e-12, f32 + bf16 outputs)
    -> intermediate GEMM with fused bias + exact-erf GELU -> output GEMM (partials)
    -> fused residual-add + LayerNorm
then the mean-pool kernel over each sequence's rows and the batched cosine kernel.
Embedding gather + LayerNorm is one fused kernel.
"""
from __future__ import annotations

import os

import torch

from .. import ops
from ..models.config import BertConfig


class HipBertEncoder:
    def __init__(self, cfg: BertConfig, weights: dict[str, torch.Tensor], device=None, use_graph: bool | None = None,
                 graph_max_rows: int | None = None, graph_max_seqs: int | None = None):
        """``graph_max_rows`` / ``graph_max_seqs``: the largest pass replayed from a hipGraph (bigger
        ones run eagerly); the tutor-served gate uses 8192 / 256 for its cross-node passes."""
        if not torch.cuda.is_available():
            raise RuntimeError("HipBertEncoder needs a GPU")
        ops.lib()
        self.cfg = cfg
        self.graph_max_rows = int(graph_max_rows or self.GRAPH_MAX_ROWS)
        self.graph_max_seqs = int(graph_max_seqs or self.GRAPH_MAX_SEQS)
        if use_graph is None:
            use_graph = os.environ.get("DLMS_GATE_GRAPH", "1") != "0"
        self.use_graph = use_graph
        self._gstate: dict[tuple[int, int], dict] = {}
        self._gbuf = None
        self.device = torch.device(device or f"cuda:{torch.cuda.current_device()}")
        dev, f32, bf = self.device, torch.float32, torch.bfloat16

        def t(name, dt=f32):
            return weights[name].to(device=dev, dtype=dt).contiguous()

        self.word = t("embeddings.word_embeddings.weight")
        self.pos = t("embeddings.position_embeddings.weight")
        self.type0 = t("embeddings.token_type_embeddings.weight")[0].contiguous()
        self.emb_g, self.emb_b = t("embeddings.LayerNorm.weight"), t("embeddings.LayerNorm.bias")
        self.layers = []
        for i in range(cfg.n_layer):
            p = f"encoder.layer.{i}."
            wqkv = torch.cat([weights[p + f"attention.self.{n}.weight"] for n in ("query", "key", "value")], 0)
            bqkv = torch.cat([weights[p + f"attention.self.{n}.bias"] for n in ("query", "key", "value")], 0)
            self.layers.append(dict(
                w_qkv=wqkv.to(dev, bf).contiguous(), b_qkv=bqkv.to(dev, f32).contiguous(),
                w_o=t(p + "attention.output.dense.weight", bf), b_o=t(p + "attention.output.dense.bias"),
                ln1_g=t(p + "attention.output.LayerNorm.weight"), ln1_b=t(p + "attention.output.LayerNorm.bias"),
                w_i=t(p + "intermediate.dense.weight", bf), b_i=t(p + "intermediate.dense.bias"),
                w_out=t(p + "output.dense.weight", bf), b_out=t(p + "output.dense.bias"),
                ln2_g=t(p + "output.LayerNorm.weight"), ln2_b=t(p + "output.LayerNorm.bias"),
            ))

    def _buffers(self, R: int, n: int, S: int):
        """Activation buffers, grown on demand and reused (no per-call allocator traffic)."""
        cfg, dev, bf = self.cfg, self.device, torch.bfloat16
        H, nh = cfg.hidden, cfg.n_head
        cap = getattr(self, "_cap", (0, 0, 0))
        if R > cap[0] or n > cap[1] or S > cap[2]:
            R2, n2, S2 = max(R, cap[0], 256), max(n, cap[1], 8), max(S, cap[2], 64)
            self._q = torch.empty(R2, H, dtype=bf, device=dev)
            self._att = torch.empty(R2, H, dtype=bf, device=dev)
            self._ff = torch.empty(R2, cfg.intermediate, dtype=bf, device=dev)
            self._kv = torch.empty(2, n2, nh, S2, 64, dtype=bf, device=dev)
            self._parts = torch.empty(1, R2, H, dtype=torch.float32, device=dev)
            self._cap = (R2, n2, S2)
        kc, vc = (self._kv[i].view(-1)[: n * nh * S * 64].view(n, nh, S, 64) for i in (0, 1))  # contiguous
        return self._q[:R], self._att[:R], self._ff[:R], kc, vc, self._parts[:, :R]

    # hipGraph-replayed passes: packed rows padded to a power-of-two bucket (>= 64) by dummy
    # sequences, sequence slots to a power of two; larger passes run eagerly
    GRAPH_MAX_ROWS = 4096
    GRAPH_MAX_SEQS = 128

    @torch.no_grad()
    def embed(self, batch: list[list[int]]) -> torch.Tensor:
        """Mean-pooled last hidden state per sequence: f32 [len(batch), H].  ``batch`` is packed
        (varlen rows, no padding): the gate encodes every concurrent query in ONE pass, replayed
        from a per-(rows, sequences)-bucket hipGraph when it fits."""
        import numpy as np

        cfg = self.cfg
        lens_np = np.asarray([max(1, min(len(ids), cfg.max_position)) for ids in batch], dtype=np.int64)
        if self.use_graph:
            R, n = int(lens_np.sum()), len(batch)
            Rb = max(64, 1 << (R - 1).bit_length())
            n_dummy = -(-(Rb - R) // cfg.max_position)
            # one bucket dimension only (rows): every pass has GRAPH_MAX_SEQS sequence slots
            if Rb <= self.graph_max_rows and n + n_dummy <= self.graph_max_seqs:
                return self._embed_graphed(batch, lens_np, Rb, self.graph_max_seqs)
        return self._embed_eager(batch, lens_np)

    def warm_graphs(self, max_rows: int | None = None) -> int:
        """Capture every row bucket up to ``max_rows`` now (a first query then never pays a
        capture); returns the number of graphs."""
        if not self.use_graph:
            return 0
        Rb = 64
        while Rb <= min(max_rows or self.graph_max_rows, self.graph_max_rows):
            L = self.cfg.max_position
            rows = Rb // 2 + 1  # lands in bucket Rb
            self.embed([[101] * min(L, rows - i * L) for i in range(-(-rows // L))])
            Rb *= 2
        return len(self._gstate)

    @staticmethod
    def _tile_table(lens):
        """AttnTiles' (row0, nq) table for packed ``lens`` (numpy)."""
        import numpy as np

        nt = (lens + 15) // 16
        starts = np.cumsum(lens) - lens
        seq = np.repeat(np.arange(lens.size), nt)
        k = np.arange(int(nt.sum())) - np.repeat(np.cumsum(nt) - nt, nt)
        return np.stack([starts[seq] + 16 * k, np.minimum(16, lens[seq] - 16 * k)], axis=1)

    def _graph_state(self, Rb: int, nb: int):
        """Static per-bucket inputs (one pinned staging buffer, one device buffer) + the graph."""
        st = self._gstate.get((Rb, nb))
        if st is not None:
            return st
        cfg, dev = self.cfg, self.device
        H, nh, S = cfg.hidden, cfg.n_head, cfg.max_position
        if self._gbuf is None:  # activations shared by every bucket, sized for the largest
            Rm, nm = self.graph_max_rows, self.graph_max_seqs
            bf = torch.bfloat16
            self._gbuf = dict(q=torch.empty(Rm, H, dtype=bf, device=dev), att=torch.empty(Rm, H, dtype=bf, device=dev),
                              ff=torch.empty(Rm, cfg.intermediate, dtype=bf, device=dev),
                              kv=torch.empty(2, nm, nh, S, 64, dtype=bf, device=dev),
                              parts=torch.empty(1, Rm, H, dtype=torch.float32, device=dev),
                              x=torch.empty(Rm, H, dtype=torch.float32, device=dev),
                              h=torch.empty(Rm, H, dtype=bf, device=dev),
                              pooled=torch.empty(nm, H, dtype=torch.float32, device=dev))
        TB = Rb // 16 + min(nb, Rb)  # >= any tile count of Rb rows in <= nb sequences (padding
        # tiles repeat the last one; they run beside the real ones, on otherwise idle CUs)
        words = 4 * Rb + 2 * nb + 2 * TB
        st = dict(host=torch.empty(words, dtype=torch.int32).pin_memory(),
                  dev=torch.empty(words, dtype=torch.int32, device=dev), TB=TB, graph=None,
                  copied=torch.cuda.Event())
        self._gstate[(Rb, nb)] = st
        return st

    def _run_layers(self, ids, pos, seq, kvlen, starts, lens_d, tiles, q, att, ff, kc, vc, parts, x, h, pooled):
        cfg = self.cfg
        eps = cfg.layer_norm_eps
        x, h = ops.bert_embed_ln(ids, pos, self.word, self.pos, self.type0, self.emb_g, self.emb_b, eps, out_f32=x,
                                 out_bf16=h)
        for lw in self.layers:
            ops.gemm(h, lw["w_qkv"], ops.EPI_QKV, bias=lw["b_qkv"], q_out=q, k_cache=kc, v_cache=vc, row_slot=seq,
                     row_pos=pos)
            ops.tile_attention(q, kc, vc, seq, kvlen, tiles, out=att)
            ops.gemm(att, lw["w_o"], ops.EPI_PARTIAL, out=parts, split_k=1)
            ops.add_layernorm(x, lw["ln1_g"], lw["ln1_b"], eps, parts=parts, nsplit=1, bias=lw["b_o"], out_bf16=h,
                              store_normed=True)
            ops.gemm(h, lw["w_i"], ops.EPI_GELU_ERF, bias=lw["b_i"], out=ff)
            ops.gemm(ff, lw["w_out"], ops.EPI_PARTIAL, out=parts, split_k=1)
            ops.add_layernorm(x, lw["ln2_g"], lw["ln2_b"], eps, parts=parts, nsplit=1, bias=lw["b_out"], out_bf16=h,
                              store_normed=True)
        return ops.mean_pool(x, starts, lens_d, out=pooled)

    def _embed_graphed(self, batch, lens_np, Rb: int, nb: int) -> torch.Tensor:
        import numpy as np

        cfg = self.cfg
        n, R, maxp = len(batch), int(lens_np.sum()), cfg.max_position
        pad = Rb - R
        dummy = [maxp] * (pad // maxp) + ([pad % maxp] if pad % maxp else [])
        lens_all = np.concatenate([lens_np, np.asarray(dummy, dtype=np.int64)])
        st = self._graph_state(Rb, nb)
        TB = st["TB"]
        st["copied"].synchronize()  # the previous pass's upload has left the staging buffer
        host = st["host"].numpy()
        ends = np.cumsum(lens_all)
        starts_np = ends - lens_all
        host[:Rb] = 0  # dummy rows: token 0
        host[:R] = np.fromiter((i for b, L in zip(batch, lens_np.tolist()) for i in (b[:L] if b else [0])),
                               dtype=np.int64, count=R)
        host[Rb:2 * Rb] = np.arange(Rb) - np.repeat(starts_np, lens_all)
        host[2 * Rb:3 * Rb] = np.repeat(np.arange(lens_all.size), lens_all)
        host[3 * Rb:4 * Rb] = np.repeat(lens_all, lens_all)
        o = 4 * Rb
        host[o:o + nb] = 0
        host[o:o + lens_all.size] = starts_np
        host[o + nb:o + 2 * nb] = 1  # unused sequence slots: one (ignored) row, never a zero divide
        host[o + nb:o + nb + lens_all.size] = lens_all
        tiles = self._tile_table(lens_all)
        tt = np.empty((TB, 2), dtype=np.int64)
        tt[:len(tiles)] = tiles
        tt[len(tiles):] = tiles[-1]  # padding tiles repeat the last one: identical rows, identical values
        host[o + 2 * nb:] = tt.reshape(-1)
        d = st["dev"]
        d.copy_(st["host"], non_blocking=True)
        st["copied"].record()
        if st["graph"] is None:
            st["graph"] = self._capture(st, Rb, nb)
        st["graph"].replay()
        return self._gbuf["pooled"][:n].clone()

    def _capture(self, st, Rb: int, nb: int):
        cfg = self.cfg
        H, nh, S = cfg.hidden, cfg.n_head, cfg.max_position
        d, TB, g = st["dev"], st["TB"], self._gbuf
        ids, pos, seq, kvlen = d[:Rb], d[Rb:2 * Rb], d[2 * Rb:3 * Rb], d[3 * Rb:4 * Rb]
        o = 4 * Rb
        starts, lens_d = d[o:o + nb], d[o + nb:o + 2 * nb]
        tiles = ops.AttnTiles.__new__(ops.AttnTiles)
        tiles.rows, tiles.n, tiles.t = Rb, TB, d[o + 2 * nb:].view(TB, 2)
        kc, vc = (g["kv"][i].view(-1)[: nb * nh * S * 64].view(nb, nh, S, 64) for i in (0, 1))
        args = (ids, pos, seq, kvlen, starts, lens_d, tiles, g["q"][:Rb], g["att"][:Rb], g["ff"][:Rb], kc, vc,
                g["parts"][:, :Rb], g["x"][:Rb], g["h"][:Rb], g["pooled"][:nb])
        side = torch.cuda.Stream(device=self.device)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):  # warm-up (code objects, allocator) outside the capture
            self._run_layers(*args)
        torch.cuda.current_stream().wait_stream(side)
        from .gpt2_engine import capture_guard

        graph = torch.cuda.CUDAGraph()
        with capture_guard(), torch.cuda.graph(graph):
            self._run_layers(*args)
        return graph

    def _embed_eager(self, batch, lens_np) -> torch.Tensor:
        import numpy as np

        cfg, dev = self.cfg, self.device
        lens = lens_np.tolist()
        R, n, S = int(lens_np.sum()), len(batch), int(lens_np.max())
        # every index array in ONE pinned host buffer -> one H2D copy (was six torch.tensor() uploads)
        ends = np.cumsum(lens_np)
        starts_np = ends - lens_np
        host = np.empty(4 * R + 2 * n, dtype=np.int32)
        host[:R] = np.fromiter((i for b, L in zip(batch, lens) for i in (b[:L] if b else [0])), dtype=np.int64, count=R)
        host[R:2 * R] = np.arange(R) - np.repeat(starts_np, lens_np)       # positions
        host[2 * R:3 * R] = np.repeat(np.arange(n), lens_np)              # sequence (cache slot)
        host[3 * R:4 * R] = np.repeat(lens_np, lens_np)                   # keys seen (bidirectional)
        host[4 * R:4 * R + n] = starts_np
        host[4 * R + n:] = lens_np
        d = torch.from_numpy(host).pin_memory().to(dev, non_blocking=True)
        ids, pos, seq, kvlen = d[:R], d[R:2 * R], d[2 * R:3 * R], d[3 * R:4 * R]
        starts, lens_d = d[4 * R:4 * R + n], d[4 * R + n:]
        q, att, ff, kc, vc, parts = self._buffers(R, n, S)
        tiles = ops.AttnTiles(lens, dev)  # bidirectional: every row of a sequence sees all its keys
        return self._run_layers(ids, pos, seq, kvlen, starts, lens_d, tiles, q, att, ff, kc, vc, parts, None, None,
                                None)

    def cosine(self, a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
        return ops.cosine(a.contiguous(), b.contiguous())
