"""KV-cached greedy decode: the agent's inference call on MI355X (BASELINE.json configs[4]).

Mirrors DrivingModel.forward with predict_language=True (simlingo_training/models/driving.py:104-187):
per sample, LLM.greedy_sample (language_model/llm.py:178-250) decodes up to max_new_tokens=100 tokens
with argmax sampling (temperature 0, sample_categorical :145-160), stopping after the EOS token; then
the driving queries are appended to prompt + generated tokens and one more forward gives the features
the route / speed heads read (driving.py:156-165).

The reference re-runs the whole prefix for every token. Here:
  * the prompt runs once through the batched MFMA kernels (the training forward's GEMMs and flash
    attention), leaving each layer's rotated q|k|v rows in a cache [S_max, (Hq+2Hkv)*64];
  * every further token is ONE replay of a hipGraph holding slx_dec_begin + 24 x {QKV GEMV with the
    RMSNorm fused, slx_dec_attn with RoPE fused, O GEMV + residual, gate/up GEMV with RMSNorm + SwiGLU
    fused, down GEMV + residual} + the LM-head GEMV with the argmax folded in (no logits tensor).
    Position / count / EOS live in device memory, so no host sync per token (the host checks the
    done flag every `check_every` tokens; steps after EOS early-exit in every kernel);
  * LoRA is merged into the frozen weights once (W + (alpha/r) B A, dropout is identity in eval),
    which is what peft computes in eval up to rounding;
  * the final driving forward runs the batched kernels over prompt + generated + queries, exactly the
    sequence the reference feeds (driving.py:156-158).
Left-padded prompts (B > 1) are decoded on their valid tokens only: RoPE scores depend on relative
positions, and the padded keys are masked in the reference's greedy loop, so the tokens are the same;
the reference's final forward passes no attention mask and would attend the pad embeddings — that
quirk (it only arises for padded batches, never in the bs=1 agent) is not reproduced.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

from . import kernels as K

BF16, F32 = torch.bfloat16, torch.float32
# the attention split over keys (Hkv x 8 workgroups) with its partials merged by the O GEMV's prologue
# (slx_dec_attn_o_split) instead of one MFMA workgroup per kv head + the O GEMV: 0.71 vs 0.80 ms per token in
# alternating bench_infer runs (tools/ab/r4_dec_ab.sh, profiles/round4_knobs_ab.txt); SLX_DEC_SPLIT_O=0 restores the old pair
SPLIT_O = os.environ.get("SLX_DEC_SPLIT_O", "1") == "1"
DEC_STORE_ROW, DEC_RESID, DEC_SWIGLU, DEC_ARGMAX = 0, 1, 2, 3


class DecGemvDesc(ctypes.Structure):
    _fields_ = [
        ("mode", K.c_int), ("W", K.c_vp), ("ldw", K.c_i64), ("N", K.c_int), ("K", K.c_int),
        ("X", K.c_vp), ("gamma", K.c_vp), ("eps", K.c_float), ("xb", K.c_vp), ("bias", K.c_vp),
        ("out", K.c_vp), ("out_ld", K.c_i64), ("resid", K.c_vp), ("keys", K.c_vp), ("state", K.c_vp),
    ]


K.register("slx_dec_key_shards", [])
K.register("slx_dec_begin", [K.c_vp, K.c_vp, K.c_vp, K.c_int, K.c_vp, K.c_vp, K.c_vp])
K.register("slx_dec_gemv", [ctypes.POINTER(DecGemvDesc), K.c_vp])
K.register("slx_dec_attn_nsplit", [K.c_int])
K.register("slx_dec_attn_ws_floats", [K.c_int, K.c_int, K.c_int])
K.register("slx_dec_attn", [K.c_vp, K.c_i64, K.c_int, K.c_int, K.c_vp, K.c_vp, K.c_int, K.c_vp, K.c_vp, K.c_vp, K.c_vp])
K.register("slx_dec_attn_o_split_ok", [K.c_int])
K.register("slx_dec_attn_o_split", [K.c_vp, K.c_i64, K.c_int, K.c_int, K.c_vp, K.c_vp, K.c_int, K.c_vp, K.c_vp, K.c_vp,
                                    K.c_vp, K.c_i64, K.c_int, K.c_int, K.c_vp, K.c_vp])


def _gemv_desc(mode, W, N, Kd, *, X=None, gamma=None, eps=0.0, xb=None, bias=None, out=None, out_ld=0, resid=None,
               keys=None, state=None):
    d = DecGemvDesc()
    d._keep = (W, X, gamma, xb, bias, out, resid, keys, state)
    d.mode, d.W, d.ldw, d.N, d.K = mode, W.data_ptr(), W.stride(0), int(N), int(Kd)
    d.X, d.gamma, d.eps = K.P(X).value or 0, K.P(gamma).value or 0, float(eps)
    d.xb, d.bias = K.P(xb).value or 0, K.P(bias).value or 0
    d.out, d.out_ld, d.resid = K.P(out).value or 0, int(out_ld), K.P(resid).value or 0
    d.keys, d.state = K.P(keys).value or 0, K.P(state).value or 0
    return d


class GreedyDecoder:
    """Greedy text decode + driving prediction for one sample at a time, bound to a VLAEngine."""

    def __init__(self, engine, max_len: int = 2048, max_new_tokens: int = 100, eos_id: int | None = None,
                 use_graph: bool = True, check_every: int = 8):
        cfg = engine.cfg
        self.eng, self.cfg = engine, cfg
        self.dev = engine.device
        self.max_len, self.max_new = int(max_len), int(max_new_tokens)
        self.eos = int(cfg.eos_id if eos_id is None else eos_id)
        self.check_every = max(1, int(check_every))
        d, F = cfg.llm_dim, cfg.llm_ffn
        self.qn, self.kn = cfg.llm_heads * 64, cfg.llm_kv_heads * 64
        self.nqkv = self.qn + 2 * self.kn
        dev = self.dev
        self._merge_weights()
        self.cache = [torch.zeros(self.max_len, self.nqkv, dtype=BF16, device=dev) for _ in range(cfg.llm_layers)]
        self.cos, self.sin = K.rope_tables(self.max_len, cfg.rope_theta, dev)
        self.state = torch.zeros(8, dtype=torch.int32, device=dev)       # slx_dec_state
        self.keys = torch.zeros(K.lib().slx_dec_key_shards(), dtype=torch.int64, device=dev)
        self.X = torch.zeros(d, dtype=F32, device=dev)
        self.obuf = torch.zeros(self.qn, dtype=BF16, device=dev)
        self.act = torch.zeros(F, dtype=BF16, device=dev)
        self.tokens = torch.zeros(max(self.max_new, 1), dtype=torch.int32, device=dev)
        self.ones_d = torch.ones(d, dtype=F32, device=dev)
        nws = K.lib().slx_dec_attn_ws_floats(cfg.llm_heads, cfg.llm_kv_heads, self.max_len)
        self.attn_ws = torch.zeros(max(nws, 1), dtype=F32, device=dev)
        # the split path's cache-length limit depends on SLX_DEC_SPLIT_NS (C side); past it, attention + O GEMV
        self.split_ok = bool(K.lib().slx_dec_attn_o_split_ok(self.max_len))
        self._build_step_descs()
        self.graph = None
        if use_graph:
            self._capture()

    # ---- weights --------------------------------------------------------------------------------
    def _merge_weights(self):
        """W_merged = W + (alpha/r) B A for q|k|v, o, gate|up, down (peft eval, llm.py:106-119), via the
        bf16 MFMA GEMM accumulating into an f32 copy of W."""
        eng, cfg = self.eng, self.cfg
        s = float(cfg.lora_scale)
        self.Wm = []
        groups = (("qkv_w", ("q", "k", "v")), ("o_w", ("o",)), ("gate_up_w", ("gate", "up")), ("down_w", ("down",)))
        for i in range(cfg.llm_layers):
            p = f"llm.{i}."
            layer = {}
            for name, sites in groups:
                base = eng.W[p + name]
                if not cfg.lora:
                    layer[name] = base
                    continue
                wf = base.float()
                row = 0
                for site in sites:
                    b = eng.W[p + f"lora.{site}.b"]   # [out, r] bf16
                    a = eng.W[p + f"lora.{site}.a"]   # [r, in] bf16
                    out = b.shape[0]
                    K.gemm(b, a, wf[row:row + out], out, a.shape[1], a.shape[0], K.GEMM_NN, b.stride(0), a.stride(0),
                           wf.stride(0), alpha=s, accumulate=True)
                    row += out
                layer[name] = wf.to(BF16)
                del wf
            self.Wm.append(layer)

    # ---- the decode step ------------------------------------------------------------------------
    def _build_step_descs(self):
        eng, cfg = self.eng, self.cfg
        d, F = cfg.llm_dim, cfg.llm_ffn
        st = self.state
        self._steps = []
        for i in range(cfg.llm_layers):
            p = f"llm.{i}."
            W = self.Wm[i]
            self._steps.append((
                _gemv_desc(DEC_STORE_ROW, W["qkv_w"], self.nqkv, d, X=self.X, gamma=eng.P[p + "ln1"], eps=cfg.rms_eps,
                           bias=eng.P[p + "qkv_b"], out=self.cache[i], out_ld=self.nqkv, state=st),
                self.cache[i],
                _gemv_desc(DEC_RESID, W["o_w"], d, self.qn, xb=self.obuf, resid=self.X, state=st),
                _gemv_desc(DEC_SWIGLU, W["gate_up_w"], F, d, X=self.X, gamma=eng.P[p + "ln2"], eps=cfg.rms_eps,
                           out=self.act, state=st),
                _gemv_desc(DEC_RESID, W["down_w"], d, F, xb=self.act, resid=self.X, state=st),
            ))
        self._head = _gemv_desc(DEC_ARGMAX, eng.W["llm.lm_head"], cfg.vocab, d, X=self.X, gamma=eng.P["llm.norm"],
                                eps=cfg.rms_eps, keys=self.keys, state=st)

    def _begin(self):
        K.call("slx_dec_begin", K.P(self.state), K.P(self.keys), K.P(self.eng.W["llm.embed"]), self.cfg.llm_dim,
               K.P(self.X), K.P(self.tokens), K.stream_ptr())

    def _step(self):
        """One generated token: record the previous argmax, run it through the 24 layers, argmax the next."""
        cfg = self.cfg
        self._begin()
        s = K.stream_ptr()
        lib = K.lib()
        for i, (qkv, cache, o, gu, down) in enumerate(self._steps):
            K.check(lib.slx_dec_gemv(ctypes.byref(qkv), s), "slx_dec_gemv")
            if SPLIT_O and self.split_ok:  # split attention, merged by the O GEMV (+ residual)
                wo = self.Wm[i]["o_w"]
                K.check(lib.slx_dec_attn_o_split(K.P(cache), cache.stride(0), cfg.llm_heads, cfg.llm_kv_heads,
                                                 K.P(self.cos), K.P(self.sin), self.max_len, K.P(self.attn_ws), None,
                                                 K.P(self.state), K.P(wo), wo.stride(0), cfg.llm_dim, self.qn,
                                                 K.P(self.X), s), "slx_dec_attn_o_split")
            else:
                K.check(lib.slx_dec_attn(K.P(cache), cache.stride(0), cfg.llm_heads, cfg.llm_kv_heads, K.P(self.cos),
                                         K.P(self.sin), self.max_len, K.P(self.attn_ws), K.P(self.obuf),
                                         K.P(self.state), s), "slx_dec_attn")
                K.check(lib.slx_dec_gemv(ctypes.byref(o), s), "slx_dec_gemv")
            K.check(lib.slx_dec_gemv(ctypes.byref(gu), s), "slx_dec_gemv")
            K.check(lib.slx_dec_gemv(ctypes.byref(down), s), "slx_dec_gemv")
        K.check(lib.slx_dec_gemv(ctypes.byref(self._head), s), "slx_dec_gemv")

    def _capture(self):
        """Capture one decode step in a hipGraph. Run once first with done=1 (every kernel early-exits; the
        begin kernel only clears the argmax keys) so one-time function attributes are set outside capture."""
        self.state.zero_()
        self.state[2] = 1
        self._step()
        torch.cuda.synchronize(self.dev)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._step()
        torch.cuda.synchronize(self.dev)
        self.graph = g

    # ---- batched LLM forward (prompt prefill and the final driving forward) ---------------------
    def _llm_batched(self, X: torch.Tensor, caches=None) -> torch.Tensor:
        """Qwen2 over the rows of one sequence X [S, d] f32 (causal) with the merged weights; returns the last
        residual stream. With `caches`, layer i writes its rotated q|k|v rows into caches[i][:S]."""
        eng, cfg = self.eng, self.cfg
        S, d = X.shape
        Hq, Hk, F = cfg.llm_heads, cfg.llm_kv_heads, cfg.llm_ffn
        qn, kn = self.qn, self.kn
        seql = torch.full((1,), S, dtype=torch.int32, device=self.dev)
        for i in range(cfg.llm_layers):
            p = f"llm.{i}."
            W = self.Wm[i]
            h, _ = eng._norm(X, eng.P[p + "ln1"], None, S, d, cfg.rms_eps, rms=True)
            qkv = caches[i][:S] if caches is not None else eng._e(S, self.nqkv)
            K.mm(h, W["qkv_w"], qkv, bias=eng.P[p + "qkv_b"])
            K.rope(qkv, S, S, Hq + Hk, self.cos, self.sin)
            o = eng._e(S, qn)
            lse = eng._e(Hq * S, dtype=F32)
            K.attn_fwd(qkv[:, :qn], qkv[:, qn:qn + kn], qkv[:, qn + kn:], o, lse, B=1, S=S, Hq=Hq, Hkv=Hk,
                       causal=True, seqlens=seql)
            Xm = eng._e(S, d, dtype=F32)
            K.mm(o, W["o_w"], Xm, epi=K.EPI_RESID_LS, resid=X, ldr=d, ls=self.ones_d)
            h2, _ = eng._norm(Xm, eng.P[p + "ln2"], None, S, d, cfg.rms_eps, rms=True)
            gu = eng._e(S, 2 * F)
            K.mm(h2, W["gate_up_w"], gu)
            act = eng._e(S, F)
            K.call("slx_swiglu_fwd", K.P(gu), gu.stride(0), K.P(act), act.stride(0), S, F, K.stream_ptr())
            Xo = eng._e(S, d, dtype=F32)
            K.mm(act, W["down_w"], Xo, epi=K.EPI_RESID_LS, resid=Xm, ldr=d, ls=self.ones_d)
            X = Xo
        return X

    # ---- public ---------------------------------------------------------------------------------
    def generate(self, prefix: torch.Tensor, max_new_tokens: int | None = None) -> torch.Tensor:
        """Greedy tokens for one prompt: prefix = inputs_embeds rows [S0, d] f32 on the device. Returns the
        sampled ids (int64, CPU) including the EOS token if it was produced (llm.py:225-248)."""
        cfg = self.cfg
        n_max = self.max_new if max_new_tokens is None else min(int(max_new_tokens), self.max_new)
        S0 = prefix.shape[0]
        if S0 + n_max > self.max_len:
            raise ValueError(f"prompt {S0} + {n_max} new tokens exceeds the cache ({self.max_len} rows)")
        if n_max <= 0:
            return torch.zeros(0, dtype=torch.long)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        ev[0].record()
        Xl = self._llm_batched(prefix, self.cache)
        # first token from the last prompt row (its argmax key is read by the first begin)
        self.state.copy_(torch.tensor([S0 - 1, 0, 0, n_max, self.eos, 0, 0, 0], dtype=torch.int32))
        self.keys.zero_()
        head = _gemv_desc(DEC_ARGMAX, self.eng.W["llm.lm_head"], cfg.vocab, cfg.llm_dim, X=Xl[S0 - 1],
                          gamma=self.eng.P["llm.norm"], eps=cfg.rms_eps, keys=self.keys, state=self.state)
        K.check(K.lib().slx_dec_gemv(ctypes.byref(head), K.stream_ptr()), "slx_dec_gemv")
        ev[1].record()
        done_steps = 0
        while done_steps < n_max - 1:
            chunk = min(self.check_every, n_max - 1 - done_steps)
            for _ in range(chunk):
                if self.graph is not None:
                    self.graph.replay()
                else:
                    self._step()
            done_steps += chunk
            if int(self.state[2].item()):
                break
        self._begin()  # records the last token (no-op after EOS)
        ev[2].record()
        n = int(self.state[1].item())
        self.last_timing = {"prefill_ms": ev[0].elapsed_time(ev[1]), "decode_ms": ev[1].elapsed_time(ev[2]),
                            "decode_steps": done_steps}
        return self.tokens[:n].long().cpu()

    def drive(self, prefix: torch.Tensor, queries: torch.Tensor, tokens: torch.Tensor):
        """driving.py:156-165: forward(prompt + generated + queries) -> route [20,2], speed_wps [n_speed, dims]."""
        eng, cfg = self.eng, self.cfg
        d = cfg.llm_dim
        S0, n, nq = prefix.shape[0], int(tokens.numel()), queries.shape[0]
        Xf = eng._e(S0 + n + nq, d, dtype=F32)
        Xf[:S0].copy_(prefix)
        if n:
            idx = tokens.to(torch.int32).to(self.dev)
            K.call("slx_gather_rows_b2f", K.P(eng.W["llm.embed"]), d, K.P(idx), n, d, K.P(Xf[S0:S0 + n]), d,
                   K.stream_ptr())
        Xf[S0 + n:].copy_(queries)
        Xo = self._llm_batched(Xf)
        feat, _ = eng._norm(Xo[S0 + n:], eng.P["llm.norm"], None, nq, d, cfg.rms_eps, rms=True)
        nr, ns = cfg.n_route, cfg.n_speed
        ridx = torch.arange(nr, dtype=torch.int32, device=self.dev)
        sidx = torch.arange(nr, nr + ns, dtype=torch.int32, device=self.dev)
        fr, fs = eng._e(nr, d, dtype=F32), eng._e(ns, d, dtype=F32)
        K.call("slx_gather_rows_b2f", K.P(feat), d, K.P(ridx), nr, d, K.P(fr), d, K.stream_ptr())
        K.call("slx_gather_rows_b2f", K.P(feat), d, K.P(sidx), ns, d, K.P(fs), d, K.stream_ptr())
        m = cfg.head_mlp
        hd = eng._mlp_fwd(fr, [("route.0", 2 * m, K.ACT_SILU), ("route.1", m, K.ACT_SILU), ("route.2", 2, K.ACT_NONE)])
        sd_ = eng._mlp_fwd(fs, [("speed.0", m, K.ACT_SILU), ("speed.1", cfg.speed_dims, K.ACT_NONE)])
        route, speed = eng._e(1, nr, 2, dtype=F32), eng._e(1, ns, cfg.speed_dims, dtype=F32)
        dummy = eng._e(max(nr, ns), dtype=F32)
        lab_r, lab_s = torch.zeros(1, nr, 2, device=self.dev), torch.zeros(1, ns, cfg.speed_dims, device=self.dev)
        K.call("slx_wp_loss_fwd", K.P(hd[0][0]), K.P(lab_r), 1, nr, 2, 0, K.P(route), K.P(dummy), K.stream_ptr())
        K.call("slx_wp_loss_fwd", K.P(sd_[0][0]), K.P(lab_s), 1, ns, cfg.speed_dims, 0, K.P(speed), K.P(dummy),
               K.stream_ptr())
        return route[0], speed[0]


def infer_example(engine, decoder: GreedyDecoder, example, max_new_tokens: int | None = None):
    """DrivingModel.forward (predict_language=True) on a batch: -> (speed_wps [B,ns,dims], route [B,nr,2],
    token id lists). One ViT pass for the whole batch, then greedy decode + driving forward per sample."""
    from .plan import plan_from_example
    cfg = engine.cfg
    plan = plan_from_example(cfg, example, inference=True)
    dplan = plan.to_device(engine.device)
    di = example.driving_input if hasattr(example, "driving_input") else example
    X = engine.encode_inputs(di.camera_images.to(engine.device), plan, dplan, {})
    routes, speeds, toks = [], [], []
    NQ = cfg.n_queries
    for b in range(plan.B):
        nv = int(plan.seqlens[b]) - NQ
        r0 = b * plan.S
        prefix = X[r0:r0 + nv]
        queries = X[r0 + nv:r0 + nv + NQ]
        t = decoder.generate(prefix, max_new_tokens)
        route, speed = decoder.drive(prefix, queries, t)
        routes.append(route)
        speeds.append(speed)
        toks.append(t.tolist())
    return torch.stack(speeds), torch.stack(routes), toks
