"""VLA training-step engine: the SimLingo hot path as an explicit sequence of gfx950 HIP kernels.

One step = InternViT (24 blocks) -> pixel_shuffle + mlp1 -> token assembly -> Qwen2 (24 blocks, LoRA)
-> final RMSNorm -> LM head on the loss rows + driving heads -> losses, then the hand-written backward.
It replaces, as one unit, DrivingModel.forward_loss (simlingo_training/models/driving.py:236-261)
and the autograd backward Lightning/DeepSpeed run after it.

Memory layout (sized for 288 GB HBM3E; no activation recompute):
  * trainable parameters live in ONE flat f32 master buffer in backward-completion order
    (param_specs), mirrored by a flat bf16 working copy (GEMM operands) and a flat f32 gradient
    buffer, so the optimizer is a single kernel and gradient buckets are contiguous ranges;
  * frozen Qwen2 weights are bf16 only (q/k/v and gate/up stored fused), 1-D frozen params f32;
  * residual streams are f32, GEMM operands and saved activations bf16, token-major everywhere
    (attention reads the fused QKV GEMM output in place).
All arithmetic is in libslx_hip.so; torch only allocates and supplies the stream.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field

import numpy as np
import torch

from . import kernels as K
from .config import VLAConfig
from .ddp import GradBucketer
from .dropmask import lora_site_seed
from .engine_ops import EngineOps
from .params import LORA_SITES, lora_io, param_specs
from .plan import Plan

BF16, F32 = torch.bfloat16, torch.float32
# InternViT weight gradients as paired launches (slx_gemm_bf16_pair); SLX_PAIR_WGRAD=0 runs them one by one (A/B)
PAIR_WGRAD = os.environ.get("SLX_PAIR_WGRAD", "1") != "0"
# main loop of the K = 64 LoRA GEMM that carries the SwiGLU backward epilogue (an HBM-bound elementwise pass): v2 128^2
# tiles, two blocks per CU, +0.1-0.15 % over the cost model's v3 (profiles/round2_s3_swiglu_bwd_ab.txt)
SWIGLU_BWD_VARIANT = int(os.environ.get("SLX_SWIGLU_BWD_VARIANT", "2"))
# LoRA B-gradient GEMMs (N = r = 32, K = the 6384 tokens): most K splits per launch (0 = the host cost model's choice).
# A/B hook: these launches are bound by HBM and latency, not by the MFMA work the cost model prices.
LORA_DB_SPLIT = int(os.environ.get("SLX_LORA_DB_SPLIT", "0"))
# Qwen2 RoPE fused into the q|k|v GEMM epilogue (0: the separate slx_rope pass, A/B hook)
FUSED_ROPE = os.environ.get("SLX_FUSED_ROPE", "1") != "0"
# Data-gradient GEMMs dX = dY W over [in][out] copies of the weights (NT main loop, 6-21% faster than NN on the step's
# shapes: profiles/round3_nn_vs_nt.txt); 0 runs them NN over W itself (A/B hook)
NT_DGRAD = os.environ.get("SLX_NT_DGRAD", "1") != "0"
# Every LoRA parameter gradient (dB_j = s dy_j^T t_j, dA_j = dT_j^T drop_j(x)) of a layer half (the MLP sites, then the
# attention sites) is deferred to ONE slx_lora_grad launch issued before the norm backward that overwrites their shared
# operand, instead of a split-K GEMM per B gradient and a dA pass per site group: +1.75 % on the step (102.0 -> 103.8
# samples/s in alternating runs, profiles/round4_lora_grad_group_ab.txt); SLX_LORA_GRAD_GROUP=0 restores the per-site path
LORA_GRAD_GROUP = os.environ.get("SLX_LORA_GRAD_GROUP", "1") == "1"
# The InternViT fc1 GEMM (and SimLingo-Base's CLIP fc1) stores act'(h) (bf16) as its aux instead of h, so the fc2
# data-gradient epilogue multiplies it in instead of evaluating act' (an rcp, an exp2 and ~10 FMA per element of
# 16400 x 4096): +0.5 % on the step (104.27 -> 104.83 samples/s, profiles/round4_gelu_aux_grad_ab.txt);
# SLX_GELU_AUX_GRAD=0 stores the pre-activation as before
GELU_AUX_GRAD = os.environ.get("SLX_GELU_AUX_GRAD", "1") == "1"
# The down site's LoRA dgrad + the SwiGLU backward as one streaming kernel (slx_lora_swiglu_bwd: 32 x 256 tiles, the K = 32
# product on the MFMA, 16-B row streams) instead of the K = 64 GEMM with the DROPMASK_SWIGLU epilogue over 128^2 tiles;
# SLX_LORA_SWIGLU_BWD=0 restores the GEMM (A/B)
LORA_SWIGLU_BWD = os.environ.get("SLX_LORA_SWIGLU_BWD", "1") == "1"
# ... and that pass also forms dA_down, dB_gate and dB_up (slx_lora_swiglu_bwd_grads), which slx_lora_grad's MLP-half
# launch otherwise computes by streaming dgu and act again; SLX_LORA_SWIGLU_GRADS=0 restores those jobs (A/B)
LORA_SWIGLU_GRADS = os.environ.get("SLX_LORA_SWIGLU_GRADS", "1") == "1"
# The SwiGLU forward and the down site's LoRA down-projection as one streaming kernel (slx_swiglu_lora_down: act is
# written once and never read back for t); SLX_SWIGLU_LORA_DOWN=0 runs slx_swiglu_fwd + slx_lora_down (A/B)
SWIGLU_LORA_DOWN = os.environ.get("SLX_SWIGLU_LORA_DOWN", "1") == "1"
# SLX_LORA_GRAD_DEFER=1: a layer's attention-half LoRA gradient jobs ride in the NEXT layer's (in backward order)
# MLP-half slx_lora_grad launch instead of a launch of their own (~50 MB, latency-bound alone); the norm backwards
# then write a fresh bf16 dX buffer, so the deferred o-site job keeps the one it read
LORA_GRAD_DEFER = os.environ.get("SLX_LORA_GRAD_DEFER", "0") == "1"
# SLX_VIT_RESID_VARIANT / SLX_LLM_RESID_VARIANT: main-loop member for the residual-epilogue GEMMs (InternViT proj / fc2
# forward, Qwen2 o / down forward); 0 = the cost model's choice (A/B hook)
VIT_RESID_VARIANT = int(os.environ.get("SLX_VIT_RESID_VARIANT", "0"))
LLM_RESID_VARIANT = int(os.environ.get("SLX_LLM_RESID_VARIANT", "0"))
# SLX_DETERMINISTIC=1: the library's deterministic-reduction mode (kernels.set_deterministic) from the first engine on:
# bitwise-reproducible gradients (ordered partial sums instead of f32 atomics), at some speed
DETERMINISTIC = os.environ.get("SLX_DETERMINISTIC", "0") == "1"
ALIGN = 64  # elements; keeps every parameter view 256-B aligned


def _f32_frozen(s) -> bool:
    """Frozen parameters the kernels read as f32 (1-D vectors and, with vision_model.freeze, the ViT position table
    added by slx_vit_embed_fwd); every other frozen tensor is a bf16 GEMM operand."""
    return len(s.shape) == 1 or s.name == "vit.pos"


def _pad8(n):
    return (n + 7) // 8 * 8


def _pad64(n):
    return (n + 63) // 64 * 64


class VLAEngine(EngineOps):
    def __init__(self, cfg: VLAConfig, device, params: dict[str, torch.Tensor] | None = None, seed: int = 0,
                 bucket_bytes: int = 32 << 20, precise: bool = False, wire: str = "f32"):
        """precise=True: fp32 parity mode — the same launch sequence with f32 activations and weights (the f32
        twins of csrc/precise.hip), forward, backward and optimizer; used to hold the trained path to the north-star
        tolerance (LoRA dropout must be 0: the parity mode has no keep masks)."""
        from .params import init_params
        self.cfg = cfg
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise RuntimeError("VLAEngine runs on the MI355X (HIP) only; there is no CPU path")
        self.precise = bool(precise)
        self.adt = F32 if self.precise else BF16   # activation / GEMM-operand dtype
        K.lib()  # fail loudly if the HIP library is missing
        if DETERMINISTIC:
            K.set_deterministic(True, self.device)
        params = params if params is not None else init_params(cfg, seed)
        self.specs = param_specs(cfg)
        # ---- flat trainable storage ----
        offs, off = {}, 0
        for s in self.specs:
            if s.trainable:
                offs[s.name] = off
                off += (math.prod(s.shape) + ALIGN - 1) // ALIGN * ALIGN
        self.n_flat = off
        dev = self.device
        self.master = torch.zeros(off, dtype=F32, device=dev)
        self.grad = torch.zeros(off, dtype=F32, device=dev)
        self.wbf = torch.zeros(off, dtype=BF16, device=dev)
        self.P, self.G, self.W = {}, {}, {}
        self.offsets = offs
        for s in self.specs:
            n = math.prod(s.shape)
            if s.trainable:
                o = offs[s.name]
                self.P[s.name] = self.master[o:o + n].view(s.shape)
                self.G[s.name] = self.grad[o:o + n].view(s.shape)
                self.W[s.name] = self.P[s.name] if self.precise else self.wbf[o:o + n].view(s.shape)
                self.P[s.name].copy_(params[s.name].to(dev))
            else:
                t = params[s.name].to(dev)
                if _f32_frozen(s):
                    self.P[s.name] = t.float().contiguous()
                else:
                    self.W[s.name] = t.to(self.adt).contiguous()
        self.wbf.copy_(self.master.to(BF16))
        # LM head padded to a multiple of 128 rows: its dgrad GEMM reads K = V rows as [K][N], and the fused CE
        # gradient epilogue (slx_lmhead_ce_bwd) writes whole 128-column tiles of dlog, so ldd >= round_up(V, 128)
        V, d = cfg.vocab, cfg.llm_dim
        self.Vp = (V + 127) // 128 * 128
        if self.Vp != V:
            lm = torch.zeros(self.Vp, d, dtype=self.adt, device=dev)
            lm[:V].copy_(self.W["llm.lm_head"])
            self.W["llm.lm_head"] = lm
        # patch-embedding weight padded to K = kpad columns for the im2col GEMM
        self.wpatch = torch.zeros(cfg.vit_dim, cfg.patch_kpad, dtype=self.adt, device=dev)
        self._refresh_derived()
        self.ones_d = torch.ones(d, dtype=F32, device=dev)
        # contiguity needed by the assembly kernel: the 30 query rows are one [30, d] block
        qr, qs = offs["drv.query_route"], offs["drv.query_speed"]
        assert qs == qr + cfg.n_route * d, "query parameters must be adjacent"
        # ---- gradient buckets (contiguous ranges, backward-completion order) ----
        self.group_ranges = {}
        for s in self.specs:
            if not s.trainable:
                continue
            o = offs[s.name]
            e = o + (math.prod(s.shape) + ALIGN - 1) // ALIGN * ALIGN
            a, b = self.group_ranges.get(s.group, (o, e))
            self.group_ranges[s.group] = (min(a, o), max(b, e))
        self.bucketer = GradBucketer(self.grad, self.group_ranges, bucket_bytes, wire=wire)
        self.world = 1
        self.step_seed = 0
        self.saved = None
        self._cos_sin = {}
        self._build_lora_cat()
        self._build_transposes()
        self._lg_jobs = []         # deferred slx_lora_grad jobs of the current layer half (LORA_GRAD_GROUP)
        self.probe_site = None     # name of a call site to bracket with HIP events (bench roofline)
        self.probe_events = []

    def load_params(self, params: dict):
        """Overwrite every parameter from {internal name: tensor} (checkpoint load): trainable -> f32 master + bf16
        working copy, frozen -> bf16 (1-D f32); derived operands (padded LM head, patch weight, LoRA-concatenated
        weights) are rebuilt and the optimizer moments reset."""
        with torch.no_grad():
            for s in self.specs:
                t = params[s.name]
                if tuple(t.shape) != tuple(s.shape):
                    raise ValueError(f"{s.name}: shape {tuple(t.shape)} != {tuple(s.shape)}")
                if s.trainable:
                    self.P[s.name].copy_(t.to(self.device, torch.float32))
                elif _f32_frozen(s):
                    self.P[s.name].copy_(t.to(self.device, torch.float32))
                elif s.name == "llm.lm_head":
                    self.W[s.name][: self.cfg.vocab].copy_(t.to(self.device, self.adt))
                else:
                    self.W[s.name].copy_(t.to(self.device, self.adt))
            self.wbf.copy_(self.master.to(BF16))
            self._build_lora_cat()
            self._build_transposes()
            self._refresh_derived()
        for name in ("m_state", "v_state"):
            if hasattr(self, name):
                delattr(self, name)

    def params_cpu(self) -> dict:
        """{internal name: f32 CPU tensor} of the current parameters (trainable from the f32 master, frozen from the
        engine's bf16 copies) - the inverse of load_params."""
        out = {}
        for s in self.specs:
            if s.trainable or _f32_frozen(s):
                out[s.name] = self.P[s.name].detach().float().cpu().clone()
            elif s.name == "llm.lm_head":
                out[s.name] = self.W[s.name][: self.cfg.vocab].detach().float().cpu()
            else:
                out[s.name] = self.W[s.name].detach().float().cpu()
        return out

    # ------------------------------------------------------------------------------------------
    def _refresh_derived(self):
        """bf16 views that are not plain slices of the flat buffer (after every optimizer step)."""
        cfg = self.cfg
        self.wpatch[:, : cfg.patch_k].copy_(self.W["vit.patch.w"])
        if getattr(self, "_pack_tab", None) is not None:
            K.call("slx_pack_scaled", K.P(self._pack_tab), self._pack_n, K.stream_ptr())
        self._refresh_transposes()

    def _build_transposes(self):
        """[in][out] copies W^T of the Linear weights whose data-gradient GEMM dX = dY W then runs NT (NT_DGRAD): the
        mlp1 / InternViT (and, without LoRA, Qwen2) weights, re-transposed from their bf16 working copies after every
        optimizer step by one batched launch (_refresh_derived). The LoRA-concatenated Qwen2 operands get theirs in
        _build_lora_cat."""
        if self.precise or not NT_DGRAD:
            self._transposed_copies([])
            return
        cfg = self.cfg
        names = ["proj.fc1.w", "proj.fc2.w"]
        if not cfg.vit_freeze:
            names += [f"vit.{i}.{n}" for i in range(cfg.vit_layers) for n in ("qkv.w", "proj.w", "fc1.w", "fc2.w")]
        if not cfg.lora:
            names += [f"llm.{i}.{n}" for i in range(cfg.llm_layers) for n in ("qkv_w", "o_w", "gate_up_w", "down_w")]
        self._transposed_copies(names)

    def _dxw(self, cat, group, name):
        """(w, w^T or None) of a Qwen2 data-gradient GEMM: the LoRA-concatenated operand of `group` or the weight."""
        if cat is not None:
            return cat[group], cat["T." + group]
        return self.W[name], self.WT.get(name)


    # LoRA folded into the frozen GEMMs by K-concatenation: y = [x | t] . [W | s*B_blockdiag]^T with
    # t = drop(x) A^T written into the extra columns of the activation buffer. Per layer and group:
    #   qkv  : x = RMSNorm1(X) [M, d]   -> W_cat [d + 2kv, d + 128]   (t_q, t_k, t_v, pad)
    #   o    : x = attention out [M, d] -> W_cat [d, d + 64]         (t_o, pad)
    #   gu   : x = RMSNorm2 [M, d]      -> W_cat [2F, d + 64]        (t_gate, t_up)
    #   down : x = SwiGLU act [M, F]    -> W_cat [d, F + 64]         (t_down, pad)
    # The dgrad GEMM dy . W_cat then returns [dx_base | s * dy_s B_s] = [dx_base | dt] in one pass.
    LORA_GROUPS = (("qkv", ("q", "k", "v"), 128), ("o", ("o",), 64), ("gu", ("gate", "up"), 64), ("down", ("down",), 64))

    def _build_lora_cat(self):
        cfg = self.cfg
        self.cat = []
        self._pack_tab = None
        if not cfg.lora:
            return
        d, F = cfg.llm_dim, cfg.llm_ffn
        qn, kn = cfg.llm_heads * 64, cfg.llm_kv_heads * 64
        s = float(cfg.lora_scale)
        entries = []
        r = cfg.lora_r
        nt = NT_DGRAD and not self.precise
        once = []
        for i in range(cfg.llm_layers):
            p = f"llm.{i}."
            cats = {}
            for g, sites, pad in self.LORA_GROUPS:
                base = {"qkv": self.W[p + "qkv_w"], "o": self.W[p + "o_w"], "gu": self.W[p + "gate_up_w"],
                        "down": self.W[p + "down_w"]}[g]
                N, Kin = base.shape
                w = torch.zeros(N, Kin + pad, dtype=self.adt, device=self.device)
                w[:, :Kin].copy_(base)
                # [W | s*B]^T for the NT data-gradient GEMM: the frozen W^T once, the s*B^T rows with every pack
                wt = torch.zeros(Kin + pad, N, dtype=self.adt, device=self.device) if nt else None
                if nt:
                    once.append((base, wt[:Kin]))
                row = 0
                for j, site in enumerate(sites):
                    out_s = lora_io(cfg, site)[1]
                    b = self.P[p + f"lora.{site}.b"]  # [out_s, r] f32 master
                    dst = w[row:row + out_s, Kin + r * j: Kin + r * (j + 1)]
                    entries.append([b.data_ptr(), b.stride(0), dst.data_ptr(), dst.stride(0), out_s, r,
                                    int(np.float32(s).view(np.int32)), int(self.precise)])
                    if nt:
                        dt = wt[Kin + r * j: Kin + r * (j + 1), row:row + out_s]
                        entries.append([b.data_ptr(), b.stride(0), dt.data_ptr(), dt.stride(0), out_s, r,
                                        int(np.float32(s).view(np.int32)), 4])
                    row += out_s
                cats[g] = w
                cats["T." + g] = wt
            # A_s zero-padded to 64 rows: the dropout-masked dgrad dx += drop'(dT_s A_s) then runs as a K=64 GEMM
            # whose A operand is the 64-column window of the group's dT buffer starting at site s (the columns past
            # the site multiply the zero rows), which keeps it on the LDS-DMA path.
            for site in LORA_SITES:
                a = self.P[p + f"lora.{site}.a"]  # [r, in] f32 master
                ap = torch.zeros(64, a.shape[1], dtype=self.adt, device=self.device)
                entries.append([a.data_ptr(), a.stride(0), ap.data_ptr(), ap.stride(0), r, a.shape[1],
                                int(np.float32(1.0).view(np.int32)), int(self.precise)])
                cats["apad." + site] = ap
                if not self.precise:  # fragment-ordered copies read by slx_lora_down (mode 2) and slx_lora_bwd (3)
                    for mode, key in ((2, "afrag."), (3, "axfrag.")):
                        af = torch.empty(r * a.shape[1], dtype=torch.bfloat16, device=self.device)
                        entries.append([a.data_ptr(), a.stride(0), af.data_ptr(), 0, r, a.shape[1],
                                        int(np.float32(1.0).view(np.int32)), mode])
                        cats[key + site] = af
                    if site == "down":  # A^T [F][32] for slx_lora_swiglu_bwd (mode 4: transposed)
                        at = torch.empty(a.shape[1], r, dtype=torch.bfloat16, device=self.device)
                        entries.append([a.data_ptr(), a.stride(0), at.data_ptr(), r, r, a.shape[1],
                                        int(np.float32(1.0).view(np.int32)), 4])
                        cats["aT.down"] = at
            self.cat.append(cats)
        self._pack_tab = torch.tensor(entries, dtype=torch.int64, device=self.device)
        self._pack_n = len(entries)
        K.call("slx_pack_scaled", K.P(self._pack_tab), self._pack_n, K.stream_ptr())
        if once:
            tab, tiles = self._transpose_table(once)
            K.call("slx_transpose_bf16", K.P(tab), len(once), tiles, K.stream_ptr())
            torch.cuda.current_stream(self.device).synchronize()  # the one-time table dies here

    def rope_tables(self, S):
        if S not in self._cos_sin:
            self._cos_sin[S] = K.rope_tables(S, self.cfg.rope_theta, self.device)
        return self._cos_sin[S]

    # ------------------------------------------------------------------------------------------
    # helpers





    # ==========================================================================================
    # forward
    def forward(self, pix: torch.Tensor, plan: Plan, dplan: dict, path: torch.Tensor, waypoints: torch.Tensor,
                training: bool = True):
        cfg = self.cfg
        sv = {}
        B = plan.B
        self.step_seed += 1
        sv["step_seed"] = self.step_seed
        sv["drop"] = cfg.lora_dropout if (training and cfg.lora) else 0.0
        X = self.encode_inputs(pix, plan, dplan, sv)
        S, d = plan.S, cfg.llm_dim
        Ml = B * S
        X, llm_saved = self.llm_stack(X, B, S, dplan["seqlens"], sv)
        sv["llm"] = llm_saved
        # final RMSNorm kept in f32: the driving heads read it unrounded (only the LM-head rows are cast to bf16)
        feat, nf = self._norm(X, self.P["llm.norm"], None, Ml, d, cfg.rms_eps, rms=True, out=self._e(Ml, d, dtype=F32))
        sv.update(X_last=X, feat=feat, nf=nf)
        # ---------------- language loss rows ----------------
        R = plan.loss_pos.shape[0]
        ce_loss = self._e(max(R, 1), dtype=F32)
        if R:
            fl = self._e(R, d)
            self._gather_feat(feat, d, dplan["loss_pos"], R, d, fl)
            lse_ce = self._e(R, dtype=F32)
            if self.precise:  # fp32 parity mode: materialised f32 logits + slx_ce_fwd
                logits = self._e(R, self.Vp, dtype=F32)
                K.mm(fl, self.W["llm.lm_head"][: cfg.vocab], logits)
                K.call("slx_ce_fwd", K.P(logits), self.Vp, K.P(dplan["loss_labels"]), R, cfg.vocab, K.P(ce_loss),
                       K.P(lse_ce), K.stream_ptr())
                sv.update(logits=logits)
            else:  # fused LM head + CE: no [R, V] logits buffer (slx_lmhead_ce_fwd)
                nws = K.lib().slx_lmhead_ce_ws_floats(R, cfg.vocab)
                ws = self._e(nws, dtype=F32)
                K.call("slx_lmhead_ce_fwd", K.P(fl), d, K.P(self.W["llm.lm_head"]), d, K.P(dplan["loss_labels"]), R,
                       cfg.vocab, d, K.P(ce_loss), K.P(lse_ce), K.P(ws), nws, K.stream_ptr())
            sv.update(fl=fl, lse_ce=lse_ce)
        # ---------------- driving heads ----------------
        nr, ns = cfg.n_route, cfg.n_speed
        qpos = dplan["query_pos"].view(B, cfg.n_queries)
        rpos = qpos[:, :nr].contiguous().view(-1)
        spos = qpos[:, nr:].contiguous().view(-1)
        m = cfg.head_mlp
        fr = self._e(B * nr, d, dtype=F32)
        fs = self._e(B * ns, d, dtype=F32)
        self._gather_feat(feat, d, rpos, B * nr, d, fr)
        self._gather_feat(feat, d, spos, B * ns, d, fs)
        hd = self._mlp_fwd(fr, [("route.0", 2 * m, K.ACT_SILU), ("route.1", m, K.ACT_SILU), ("route.2", 2, K.ACT_NONE)])
        sd_ = self._mlp_fwd(fs, [("speed.0", m, K.ACT_SILU), ("speed.1", cfg.speed_dims, K.ACT_NONE)])
        route_pred = self._e(B, nr, 2, dtype=F32)
        route_loss = self._e(B * nr, dtype=F32)
        lab_r = path.float().contiguous()
        lab_s = waypoints[:, : nr + 1].float().contiguous()
        K.call("slx_wp_loss_fwd", K.P(hd[0][0]), K.P(lab_r), B, nr, 2, 0, K.P(route_pred), K.P(route_loss), K.stream_ptr())
        speed_pred = self._e(B, ns, cfg.speed_dims, dtype=F32)
        speed_loss = self._e(B * ns, dtype=F32)
        K.call("slx_wp_loss_fwd", K.P(sd_[0][0]), K.P(lab_s), B, ns, cfg.speed_dims, 0, K.P(speed_pred), K.P(speed_loss),
               K.stream_ptr())
        out4 = self._e(4, dtype=F32)
        K.call("slx_loss_finalize", K.P(ce_loss), R, K.P(route_loss), B * nr, K.P(speed_loss), B * ns, K.P(out4),
               K.stream_ptr())
        sv.update(plan=plan, dplan=dplan, rpos=rpos, spos=spos, fr=fr, fs=fs, hd=hd, sd=sd_, lab_r=lab_r, lab_s=lab_s,
                  route_pred=route_pred, speed_pred=speed_pred, R=R, S=S, Ml=Ml,
                  ce_loss=ce_loss, route_loss=route_loss, speed_loss=speed_loss)
        self.saved = sv
        return out4, route_pred, speed_pred

    def llm_stack(self, X: torch.Tensor, B: int, S: int, seql: torch.Tensor, sv: dict):
        """Qwen2 decoder x24 + LoRA (language_model.model, driving.py:217-223) over the assembled rows X [B*S, d] f32,
        causal with key padding (seql [B] valid leading rows). Returns the last residual stream and the per-layer
        activations the backward reads (sv["drop"] / sv["step_seed"] select the LoRA dropout masks)."""
        cfg = self.cfg
        d = cfg.llm_dim
        Ml = B * S
        # ---------------- Qwen2 + LoRA ----------------
        Hq, Hk, Fl = cfg.llm_heads, cfg.llm_kv_heads, cfg.llm_ffn
        qn, kn = Hq * 64, Hk * 64
        nqkv = qn + 2 * kn
        cos, sin = self.rope_tables(S)
        llm_saved = []
        lora = cfg.lora
        r = cfg.lora_r
        for i in range(cfg.llm_layers):
            p = f"llm.{i}."
            L = {}
            cat = self.cat[i] if lora else None
            Pq, Po, Pg, Pd = (128, 64, 64, 64) if lora else (0, 0, 0, 0)
            hx = self._buf(("hx", i), Ml, d + Pq, zero=lora)
            h, nrm1 = self._norm(X, self.P[p + "ln1"], None, Ml, d, cfg.rms_eps, rms=True, out=hx[:, :d])
            if lora:
                L.update(self._lora_down(hx[:, :d], i, ("q", "k", "v"), hx[:, d:], sv))
            qkv = self._e(Ml, nqkv)
            # q|k|v projection with RoPE on the q and k head slots (the first Hq+Hk) fused into its epilogue
            K.mm(hx, cat["qkv"] if lora else self.W[p + "qkv_w"], qkv, bias=self.P[p + "qkv_b"],
                 rope=(cos, sin, S, (Hq + Hk) * 64) if FUSED_ROPE else None)
            if not FUSED_ROPE:
                K.rope(qkv, Ml, S, Hq + Hk, cos, sin)
            ox = self._buf(("ox", i), Ml, qn + Po, zero=lora)
            o = ox[:, :qn]
            lse = self._e(B * Hq * S, dtype=F32)
            K.attn_fwd(qkv[:, :qn], qkv[:, qn:qn + kn], qkv[:, qn + kn:], o, lse, B=B, S=S, Hq=Hq, Hkv=Hk, causal=True,
                       seqlens=seql)
            if lora:
                L.update(self._lora_down(o, i, ("o",), ox[:, qn:], sv))
            Xm = self._e(Ml, d, dtype=F32)
            K.mm(ox, cat["o"] if lora else self.W[p + "o_w"], Xm, epi=K.EPI_RESID_LS, resid=X, ldr=d, ls=self.ones_d,
                 variant=LLM_RESID_VARIANT or None)
            h2x = self._buf(("h2x", i), Ml, d + Pg, zero=lora)
            h2, nrm2 = self._norm(Xm, self.P[p + "ln2"], None, Ml, d, cfg.rms_eps, rms=True, out=h2x[:, :d])
            if lora:
                L.update(self._lora_down(h2, i, ("gate", "up"), h2x[:, d:], sv))
            gu = self._e(Ml, 2 * Fl)
            K.mm(h2x, cat["gu"] if lora else self.W[p + "gate_up_w"], gu)
            ax = self._buf(("ax", i), Ml, Fl + Pd, zero=lora)
            act = ax[:, :Fl]
            if lora and SWIGLU_LORA_DOWN and not self.precise and Fl % 256 == 0:
                bits = self._lora_bits(i, "down", Ml, sv)
                ws = self._buf(("sld_ws",), K.lib().slx_swiglu_lora_down_ws_floats(Ml, Fl), dtype=F32)
                K.swiglu_lora_down(gu, act, self.cat[i]["apad.down"], ax[:, Fl:Fl + cfg.lora_r], bits, sv["drop"], ws)
                L["down"] = bits
            else:
                self._swiglu(gu, act, Ml, Fl)
                if lora:
                    L.update(self._lora_down(act, i, ("down",), ax[:, Fl:], sv))
            Xo = self._e(Ml, d, dtype=F32)
            K.mm(ax, cat["down"] if lora else self.W[p + "down_w"], Xo, epi=K.EPI_RESID_LS, resid=Xm, ldr=d,
                 ls=self.ones_d, variant=LLM_RESID_VARIANT or None)
            llm_saved.append(dict(X=X, hx=hx, n1=nrm1, qkv=qkv, ox=ox, lse=lse, Xm=Xm, h2x=h2x, n2=nrm2, gu=gu, ax=ax,
                                  lora=L))
            X = Xo
        return X, llm_saved

    def vit_features(self, pix: torch.Tensor, sv: dict | None = None) -> torch.Tensor:
        """InternViT (24 layers) -> drop CLS -> pixel_shuffle(0.5) + mlp1 (extract_feature, internvl2_model.py:114):
        pixel tiles [N, 3, 448, 448] -> image tokens [N*256, d] (bf16, or f32 in parity mode). Saves what the backward
        reads into `sv`."""
        cfg = self.cfg
        sv = {} if sv is None else sv
        pix = pix.reshape(-1, 3, cfg.img_size, cfg.img_size)
        if pix.dtype != F32 or not pix.is_contiguous():
            pix = pix.float().contiguous()
        N = pix.shape[0]
        sv["N"] = N
        # ---------------- InternViT ----------------
        D, T, F_, H = cfg.vit_dim, cfg.vit_tokens, cfg.vit_ffn, cfg.vit_heads
        g = cfg.vit_grid
        Mv = N * T
        col = self._e(N * g * g, cfg.patch_kpad)
        K.call("slx_im2col_patch_f32" if self.precise else "slx_im2col_patch", K.P(pix), N, cfg.img_size, cfg.img_size, cfg.patch, cfg.patch_kpad, K.P(col), K.stream_ptr())
        pe = self._e(N * g * g, D, dtype=F32)
        K.mm(col, self.wpatch, pe, bias=self.P["vit.patch.b"])
        x = self._e(Mv, D, dtype=F32)
        K.call("slx_vit_embed_fwd", K.P(pe), K.P(self.P["vit.cls"]), K.P(self.P["vit.pos"]), K.P(x), N, T, D, K.stream_ptr())
        sv["col"] = col
        vit_saved = []
        for i in range(cfg.vit_layers):
            p = f"vit.{i}."
            h1, n1 = self._norm(x, self.P[p + "ln1.w"], self.P[p + "ln1.b"], Mv, D, cfg.vit_eps)
            qkv = self._e(Mv, 3 * D)
            K.mm(h1, self.W[p + "qkv.w"], qkv, bias=self.P[p + "qkv.b"])
            o = self._e(Mv, D)
            lse = self._e(N * H * T, dtype=F32)
            with self._probe("vit.attn"):
                K.attn_fwd(qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:], o, lse, B=N, S=T, Hq=H, Hkv=H, causal=False)
            xm = self._e(Mv, D, dtype=F32)
            y1 = self._e(Mv, D)
            K.mm(o, self.W[p + "proj.w"], xm, bias=self.P[p + "proj.b"], epi=K.EPI_RESID_LS, resid=x, ldr=D,
                 ls=self.P[p + "ls1"], aux_out=y1, ldaux_out=D, variant=VIT_RESID_VARIANT or None)
            h2, n2 = self._norm(xm, self.P[p + "ln2.w"], self.P[p + "ln2.b"], Mv, D, cfg.vit_eps)
            hpre = self._e(Mv, F_)
            hact = self._e(Mv, F_)
            hgrad = GELU_AUX_GRAD and not self.precise  # hpre then holds gelu'(h) (see GELU_AUX_GRAD)
            with self._probe("vit.fc1"):
                K.mm(h2, self.W[p + "fc1.w"], hact, bias=self.P[p + "fc1.b"], epi=K.EPI_GELU, aux_out=hpre, ldaux_out=F_,
                     aux_grad=hgrad)
            xo = self._e(Mv, D, dtype=F32)
            y2 = self._e(Mv, D)
            K.mm(hact, self.W[p + "fc2.w"], xo, bias=self.P[p + "fc2.b"], epi=K.EPI_RESID_LS, resid=xm, ldr=D,
                 ls=self.P[p + "ls2"], aux_out=y2, ldaux_out=D, variant=VIT_RESID_VARIANT or None)
            vit_saved.append(dict(x=x, h1=h1, n1=n1, qkv=qkv, o=o, lse=lse, y1=y1, xm=xm, h2=h2, n2=n2, hpre=hpre,
                                  hact=hact, y2=y2, hgrad=hgrad))
            x = xo
        sv["vit"] = vit_saved
        sv["vit_out"] = x
        # ---------------- pixel_shuffle + mlp1 ----------------
        d = cfg.llm_dim
        Mi = N * cfg.img_tokens_per_tile
        z, nz = self._norm(x, self.P["proj.ln.w"], self.P["proj.ln.b"], Mi, 4 * D, cfg.proj_eps, ps=g, tpi=T, ldx=D)
        a1pre = self._e(Mi, d)
        a1 = self._e(Mi, d)
        K.mm(z, self.W["proj.fc1.w"], a1, bias=self.P["proj.fc1.b"], epi=K.EPI_GELU, aux_out=a1pre, ldaux_out=d)
        img = self._e(Mi, d)
        K.mm(a1, self.W["proj.fc2.w"], img, bias=self.P["proj.fc2.b"])
        sv.update(z=z, nz=nz, a1pre=a1pre, a1=a1, Mi=Mi, Mv=Mv)
        return img

    def encode_inputs(self, pix: torch.Tensor, plan: Plan, dplan: dict, sv: dict) -> torch.Tensor:
        """InternViT -> pixel_shuffle + mlp1 -> wp_encoder -> token assembly: the LLM input rows X [B*S, d] f32
        (extract_feature internvl2_model.py:114, replace_placeholder_tokens :17-144, AdaptorList.forward
        adaptors.py:301-331). Saves what the backward needs into `sv`."""
        cfg = self.cfg
        B = plan.B
        sv["B"] = B
        img = self.vit_features(pix, sv)
        d = cfg.llm_dim
        Mi = sv["Mi"]
        # ---------------- waypoint encoder (placeholder coords) ----------------
        nwp = plan.wp_coords.shape[0]
        wp_out = self._e(max(nwp, 1), d, dtype=F32)
        if nwp:
            c = dplan["wp_coords"]
            w1pre = self._e(nwp, cfg.wp_hidden, dtype=F32)
            w1 = self._e(nwp, cfg.wp_hidden, dtype=F32)
            K.sgemm(c, 2, 1, self.P["wp.0.w"], 1, 2, w1, cfg.wp_hidden, 1, nwp, cfg.wp_hidden, 2, bias=self.P["wp.0.b"],
                    act=K.ACT_RELU, pre=w1pre, ldpre=cfg.wp_hidden)
            w2pre = self._e(nwp, cfg.wp_hidden2, dtype=F32)
            w2 = self._e(nwp, cfg.wp_hidden2, dtype=F32)
            K.sgemm(w1, cfg.wp_hidden, 1, self.P["wp.1.w"], 1, cfg.wp_hidden, w2, cfg.wp_hidden2, 1, nwp, cfg.wp_hidden2,
                    cfg.wp_hidden, bias=self.P["wp.1.b"], act=K.ACT_RELU, pre=w2pre, ldpre=cfg.wp_hidden2)
            K.sgemm(w2, cfg.wp_hidden2, 1, self.P["wp.2.w"], 1, cfg.wp_hidden2, wp_out, d, 1, nwp, d, cfg.wp_hidden2,
                    bias=self.P["wp.2.b"])
            sv.update(w1pre=w1pre, w1=w1, w2pre=w2pre, w2=w2)
        # ---------------- token assembly ----------------
        S = plan.S
        Ml = B * S
        X = self._e(Ml, d, dtype=F32)
        K.call("slx_assemble_tokens_f32" if self.precise else "slx_assemble_tokens", K.P(dplan["code"]), Ml, d, K.P(self.W["llm.embed"]), cfg.vocab, K.P(img),
               K.P(wp_out), K.P(self.P["drv.query_route"]), K.P(X), K.stream_ptr())
        sv["nwp"] = nwp
        return X

    def llm_features(self, X: torch.Tensor, B: int, S: int, seql: torch.Tensor, logits: bool = False):
        """Eval forward of the Qwen2 stack on arbitrary input rows X [B*S, d] f32 (LoRA dropout off): post-norm
        features [B*S, d] f32 and, if asked, the full-vocabulary logits [B*S, V] f32 (language_model.model(...),
        driving.py:217-225 / llm.py:126-143)."""
        cfg = self.cfg
        d, Ml = cfg.llm_dim, B * S
        Xl, _ = self.llm_stack(X, B, S, seql, {"step_seed": 0, "drop": 0.0})
        feat, _ = self._norm(Xl, self.P["llm.norm"], None, Ml, d, cfg.rms_eps, rms=True, out=self._e(Ml, d, dtype=F32))
        if not logits:
            return feat, None
        fb = self._e(Ml, d)
        if self.precise:
            fb.copy_(feat)
        else:
            K.call("slx_cast_rows", K.P(feat), d, K.P(fb), d, Ml, d, K.stream_ptr())
        lg = self._e(Ml, self.Vp, dtype=F32)
        K.mm(fb, self.W["llm.lm_head"][: cfg.vocab], lg)
        return feat, lg[:, : cfg.vocab]

    def _lora_down(self, x, i, sites, t_out, sv):
        """t_out[:, 32j:32j+32] = drop_j(x) A_j^T for the sites sharing x (bf16, written into the extra columns of
        the activation buffer), one launch. Dropout is applied while loading x (hash mask); the keep masks are also
        stored as bits (persistent per layer and site) for the backward. Returns {site: keep bits or None}."""
        seeds = [lora_site_seed(sv["step_seed"], i, LORA_SITES.index(site)) for site in sites]
        if self.precise:  # parity mode runs the eval forward: dropout off, t = x A^T as f32 GEMMs
            if sv["drop"] > 0:
                raise RuntimeError("fp32 parity mode runs the eval forward (LoRA dropout off): forward(training=False)")
            r = self.cfg.lora_r
            for j, site in enumerate(sites):
                K.mm(x, self.W[f"llm.{i}.lora.{site}.a"], t_out[:, r * j:r * (j + 1)])
            return {site: None for site in sites}
        bits = [self._lora_bits(i, site, x.shape[0], sv) for site in sites]
        K.lora_down(x, [self.cat[i]["afrag." + site] for site in sites], t_out, seeds, p=sv["drop"], bits=bits,
                    packed=True)
        return dict(zip(sites, bits))

    def _bits_layer(self, i, M, sv):
        jobs = []
        for j, s in enumerate(LORA_SITES):
            kin = lora_io(self.cfg, s)[0]
            b = self._buf(("bits", i, s), M, kin // 32, dtype=torch.int32)
            jobs.append((lora_site_seed(sv["step_seed"], i, j), b, kin, kin))
        K.dropout_bits(jobs, M, sv["drop"])

    def _lora_bits(self, i, site, M, sv):
        """Keep-bit mask of one (layer, site) for this step (persistent buffer; None without dropout). The 7 sites of
        a layer are generated by one slx_dropout_bits launch, the first time any of them is asked for in a step."""
        if sv["drop"] <= 0:
            return None
        key = sv.setdefault("bits_done", set())
        if i not in key:
            self._bits_layer(i, M, sv)
            key.add(i)
        return self._buf(("bits", i, site), M, lora_io(self.cfg, site)[0] // 32, dtype=torch.int32)


    # ==========================================================================================
    # backward
    def backward(self, dlosses: torch.Tensor | None = None):
        cfg = self.cfg
        sv = self.saved
        assert sv is not None, "backward() without forward()"
        pr = self.precise  # fp32 parity mode: the same sequence over f32 operands (csrc/precise.hip twins)
        if pr and sv["drop"] > 0:
            raise RuntimeError("the fp32 parity mode has no LoRA dropout (lora_dropout = 0)")
        B, S, Ml, Mv, Mi, R = sv["B"], sv["S"], sv["Ml"], sv["Mv"], sv["Mi"], sv["R"]
        d, D = cfg.llm_dim, cfg.vit_dim
        nr, ns = cfg.n_route, cfg.n_speed
        dplan = sv["dplan"]
        self.grad.zero_()  # one memset per step; every gradient producer below accumulates
        gs = self._e(3, dtype=F32)
        if dlosses is not None:
            dlosses = dlosses.float().contiguous()
        K.call("slx_loss_gscale", K.P(dlosses), R, B * nr, B * ns, K.P(gs), K.stream_ptr())
        # ---------------- driving heads ----------------
        dfeat = self._z(Ml + 1, d)  # + one zero row for unreferenced gathers
        for tag, npts, dims, saved, lab, pos in (("route", nr, 2, sv["hd"], sv["lab_r"], sv["rpos"]),
                                                 ("speed", ns, cfg.speed_dims, sv["sd"], sv["lab_s"], sv["spos"])):
            dout = self._e(B * npts, dims, dtype=F32)
            pred = sv["route_pred"] if tag == "route" else sv["speed_pred"]
            K.call("slx_wp_loss_bwd", K.P(pred), K.P(lab), B, npts, dims, 0, K.P(gs[1:2] if tag == "route" else gs[2:3]),
                   K.P(dout), K.stream_ptr())
            dx = self._mlp_bwd(dout, saved)
            K.call("slx_scatter_rows", K.P(dx), d, K.P(pos), B * npts, d, K.P(dfeat), d, 1, K.stream_ptr())
        self._group_done("heads")
        # ---------------- language loss ----------------
        if R:
            dlog = self._e(R, self.Vp)
            if "logits" in sv:
                K.call("slx_ce_bwd_f32" if pr else "slx_ce_bwd", K.P(sv["logits"]), self.Vp, K.P(dplan["loss_labels"]), K.P(sv["lse_ce"]), R,
                       cfg.vocab, K.P(gs[0:1]), K.P(dlog), self.Vp, K.stream_ptr())
            else:  # the LM-head GEMM recomputed with the softmax-gradient epilogue (slx_lmhead_ce_bwd)
                K.call("slx_lmhead_ce_bwd", K.P(sv["fl"]), d, K.P(self.W["llm.lm_head"]), d, K.P(dplan["loss_labels"]),
                       K.P(sv["lse_ce"]), R, cfg.vocab, d, K.P(gs[0:1]), K.P(dlog), self.Vp, K.stream_ptr())
            dfl = self._e(R, d, dtype=F32)
            K.mm(dlog, self.W["llm.lm_head"], dfl, tb=False)  # [R,Vp] @ [Vp,d]
            K.call("slx_scatter_rows", K.P(dfl), d, K.P(dplan["loss_pos"]), R, d, K.P(dfeat), d, 1, K.stream_ptr())
        # ---------------- final RMSNorm ----------------
        dX = self._z(Ml + 1, d)
        # bf16 copy of dX, written by every norm backward that updates dX (dgrad operand); parity mode: dX itself
        dxb = dX[:Ml] if pr else self._e(Ml, d)
        nb = None if pr else dxb
        K.norm_bwd(sv["nf"], dfeat, dX, dx_bf16=nb)
        # ---------------- Qwen2 layers ----------------
        Hq, Hk, Fl = cfg.llm_heads, cfg.llm_kv_heads, cfg.llm_ffn
        qn, kn = Hq * 64, Hk * 64
        nqkv = qn + 2 * kn
        cos, sin = self.rope_tables(S)
        ws = K.attn_ws(B, S, Hq, Hk, self.device)
        lora = cfg.lora
        r = cfg.lora_r
        defer = (lora and LORA_GRAD_GROUP and LORA_GRAD_DEFER and not self.precise and self._lg_shapes_ok())
        done_pending = None
        for i in reversed(range(cfg.llm_layers)):
            p = f"llm.{i}."
            Ls = sv["llm"][i]
            cat = self.cat[i] if lora else None
            Pq, Po, Pg, Pd = (128, 64, 64, 64) if lora else (0, 0, 0, 0)
            hx, ox, h2x, ax = Ls["hx"], Ls["ox"], Ls["h2x"], Ls["ax"]
            # down projection: Xo = Xm + [act | t_d] . [Wd | s B_d]^T   (dxb = bf16(dX), from the last norm backward)
            # bf16 with LoRA: the gradient of act that a bf16 Linear backward produces under autocast (read once by the
            # SwiGLU epilogue and, columns Fl.., as the dT operand); f32 for the plain slx_swiglu_bwd path
            dax = self._e(Ml, Fl + Pd, dtype=BF16 if (lora and not pr) else F32)
            self._mm_dx(dxb, *self._dxw(cat, "down", p + "down_w"), dax)
            dgu = self._e(Ml, 2 * Fl)
            if lora:  # the down-site dropout dgrad and the SwiGLU backward share one GEMM epilogue
                self._lora_bwd(i, ("down",), [dxb], ax[:, Fl:], ax[:, :Fl], dax[:, Fl:], dax[:, :Fl], sv,
                               swiglu=(Ls["gu"], dgu), gu_t=h2x[:, d:])
            else:
                K.call("slx_swiglu_bwd_f32" if pr else "slx_swiglu_bwd", K.P(dax), dax.stride(0), K.P(Ls["gu"]), 2 * Fl,
                       K.P(dgu), 2 * Fl, Ml, Fl, K.stream_ptr())
            del dax
            dh2x = self._e(Ml, d + Pg, dtype=F32)
            self._mm_dx(dgu, *self._dxw(cat, "gu", p + "gate_up_w"), dh2x)
            if lora:
                self._lora_bwd(i, ("gate", "up"), [dgu[:, :Fl], dgu[:, Fl:]], h2x[:, d:], h2x[:, :d], dh2x[:, d:],
                               dh2x[:, :d], sv)
            del dgu
            self._lg_flush(Ml)  # before dxb (the down site's dy) is overwritten
            if done_pending is not None:  # the previous layer's deferred attention-half jobs were in that launch
                self._group_done(done_pending)
                done_pending = None
            if defer:
                dxb = nb = self._e(Ml, d)
            K.norm_bwd(Ls["n2"], dh2x, dX, dx_accumulate=True, dx_bf16=nb)
            # o projection
            dox = self._e(Ml, qn + Po, dtype=F32)
            self._mm_dx(dxb, *self._dxw(cat, "o", p + "o_w"), dox)
            dob = dox[:, :qn] if pr else self._e(Ml, qn)
            if lora:  # the LoRA dx term and the bf16 cast of dO in one pass
                self._lora_bwd(i, ("o",), [dxb], ox[:, qn:], ox[:, :qn], dox[:, qn:], dox[:, :qn], sv,
                               dx_bf16=None if pr else dob)
            elif not pr:
                K.call("slx_cast_rows", K.P(dox), dox.stride(0), K.P(dob), qn, Ml, qn, K.stream_ptr())
            del dox
            qkv = Ls["qkv"]
            dqkv = self._e(Ml, nqkv)
            K.attn_bwd(qkv[:, :qn], qkv[:, qn:qn + kn], qkv[:, qn + kn:], ox[:, :qn], Ls["lse"], dob,
                       dqkv[:, :qn], dqkv[:, qn:qn + kn], dqkv[:, qn + kn:], ws, rope_cos=cos, rope_sin=sin,
                       B=B, S=S, Hq=Hq, Hkv=Hk, causal=True, seqlens=dplan["seqlens"])
            dhx = self._e(Ml, d + Pq, dtype=F32)
            self._mm_dx(dqkv, *self._dxw(cat, "qkv", p + "qkv_w"), dhx)
            if lora:
                self._lora_bwd(i, ("q", "k", "v"), [dqkv[:, :qn], dqkv[:, qn:qn + kn], dqkv[:, qn + kn:]], hx[:, d:],
                               hx[:, :d], dhx[:, d:], dhx[:, :d], sv)
            if defer:  # the attention-half jobs wait for the next layer's MLP-half launch; the o site keeps its dxb
                dxb = nb = self._e(Ml, d)
            else:
                self._lg_flush(Ml)  # before dxb (the o site's dy) is overwritten
            K.norm_bwd(Ls["n1"], dhx, dX, dx_accumulate=True, dx_bf16=nb)
            del dqkv, dhx, dh2x
            if lora:
                if defer:
                    done_pending = f"llm{i}"
                else:
                    self._group_done(f"llm{i}")
        if done_pending is not None:
            self._lg_flush(Ml)
            self._group_done(done_pending)
        # ---------------- token assembly backward ----------------
        qg = self.G["drv.query_route"]  # [20, d] followed by [10, d] (adjacent)
        K.call("slx_gather_sum", K.P(dX), d, K.P(dplan["query_pos"]), B, cfg.n_queries, d, K.P(qg), 0, K.stream_ptr())
        nwp = sv["nwp"]
        if nwp:
            dwp = self._e(nwp, d, dtype=F32)
            K.call("slx_gather_rows", K.P(dX), d, K.P(dplan["wp_pos"]), nwp, d, K.P(dwp), d, 0, K.stream_ptr())
            saved = [(None, None, sv["w2"], "wp.2", K.ACT_NONE), (sv["w2"], sv["w2pre"], sv["w1"], "wp.1", K.ACT_RELU),
                     (sv["w1"], sv["w1pre"], dplan["wp_coords"], "wp.0", K.ACT_RELU)]
            self._mlp_bwd(dwp, saved, need_dx=False)
        else:
            for n in ("wp.0.w", "wp.0.b", "wp.1.w", "wp.1.b", "wp.2.w", "wp.2.b"):
                self.G[n].zero_()
        self._group_done("assembly")
        dimg = self._e(Mi, d)
        K.call("slx_gather_rows", K.P(dX), d, K.P(dplan["img_pos"]), Mi, d, K.P(dimg), d, int(not pr), K.stream_ptr())
        del dX, dfeat
        # ---------------- mlp1 backward ----------------
        K.mm(dimg, sv["a1"], self.G["proj.fc2.w"], ta=True, tb=False, accumulate=True)
        self._colsum(dimg, self.G["proj.fc2.b"])
        da1 = self._e(Mi, d)
        self._mm_dx(dimg, self.W["proj.fc2.w"], self.WT.get("proj.fc2.w"), da1, epi=K.EPI_GELU_BWD, aux=sv["a1pre"],
                    ldaux=d, colsum=self.G["proj.fc1.b"])
        K.mm(da1, sv["z"], self.G["proj.fc1.w"], ta=True, tb=False, accumulate=True)
        dz = self._e(Mi, 4 * D, dtype=F32)
        self._mm_dx(da1, self.W["proj.fc1.w"], self.WT.get("proj.fc1.w"), dz)
        T = cfg.vit_tokens
        dxv = self._z(Mv, D)
        ws_n = self._ws(K.norm_ws_floats(4 * D))
        K.norm_bwd(sv["nz"], dz, dxv, dgamma=self.G["proj.ln.w"], dbeta=self.G["proj.ln.b"], ws=ws_n, lddx=D,
                   param_accumulate=True)
        del dz, da1, dimg
        self._group_done("proj")
        if cfg.vit_freeze:  # vision_model.freeze: mlp1 is the last trainable module; no InternViT backward at all
            self.bucketer.mark("backward_end")
            self.saved = None
            return
        # ---------------- InternViT layers ----------------
        F_, H, N = cfg.vit_ffn, cfg.vit_heads, sv["N"]
        vws = K.attn_ws(N, T, H, H, self.device)
        g = self._e(Mv, D)
        lnws = self._ws(max(K.norm_ws_floats(D), K.lib().slx_colsum_ws_floats(F_) + 0))
        for i in reversed(range(cfg.vit_layers)):
            p = f"vit.{i}."
            Ls = sv["vit"][i]
            # x_out = x_mid + ls2 * (fc2(gelu(fc1(ln2(x_mid)))) ); below the top layer this branch backward ran fused
            # into the previous LN1 backward (slx_norm_desc.ls*)
            if i == cfg.vit_layers - 1 and pr:
                self._ls_branch_precise(dxv, self.P[p + "ls2"], Ls["y2"], g, self.G[p + "ls2"], self.G[p + "fc2.b"])
            elif i == cfg.vit_layers - 1:
                K.call("slx_ls_branch_bwd", K.P(dxv), D, K.P(self.P[p + "ls2"]), K.P(Ls["y2"]), D, K.P(g), D, Mv, D,
                       K.P(self.G[p + "ls2"]), K.P(self.G[p + "fc2.b"]), 1, K.P(self._ws(2 * 256 * D)), K.stream_ptr())
            pair = PAIR_WGRAD and not pr
            if not pair:
                K.mm(g, Ls["hact"], self.G[p + "fc2.w"], ta=True, tb=False, accumulate=True)
            dh = self._e(Mv, F_)
            self._mm_dx(g, self.W[p + "fc2.w"], self.WT.get(p + "fc2.w"), dh, epi=K.EPI_GELU_BWD, aux=Ls["hpre"],
                        ldaux=F_, colsum=self.G[p + "fc1.b"],  # fc1.b grad = column sums of dh, in the same epilogue
                        aux_grad=Ls["hgrad"])
            if pair:  # fc2.w and fc1.w gradients as one launch (two under-filled grids fill the chip together)
                with self._probe("vit.wgrad_fc"):
                    K.mm_pair((g, Ls["hact"], self.G[p + "fc2.w"]), (dh, Ls["h2"], self.G[p + "fc1.w"]))
            else:
                K.mm(dh, Ls["h2"], self.G[p + "fc1.w"], ta=True, tb=False, accumulate=True)
            dh2 = self._e(Mv, D)  # bf16: the gradient a bf16 Linear backward hands the fp32 LayerNorm under autocast
            self._mm_dx(dh, self.W[p + "fc1.w"], self.WT.get(p + "fc1.w"), dh2)
            del dh
            # x_mid = x_in + ls1 * proj(attn(ln1(x_in))): its branch backward (g = ls1 * dx_mid, dls1, proj.b grad)
            # fused into the LN2 backward that produces dx_mid
            lsb = (self.P[p + "ls1"], Ls["y1"], g, self.G[p + "ls1"], self.G[p + "proj.b"])
            K.norm_bwd(Ls["n2"], dh2, dxv, dx_accumulate=True, dgamma=self.G[p + "ln2.w"], dbeta=self.G[p + "ln2.b"],
                       ws=self._ws(K.norm_ws_floats(D)), param_accumulate=True, ls_branch=None if pr else lsb)
            if pr:
                self._ls_branch_precise(dxv, *lsb)
            if not pair:
                K.mm(g, Ls["o"], self.G[p + "proj.w"], ta=True, tb=False, accumulate=True)
            do = self._e(Mv, D)
            self._mm_dx(g, self.W[p + "proj.w"], self.WT.get(p + "proj.w"), do)
            qkv = Ls["qkv"]
            dqkv = self._e(Mv, 3 * D)
            K.attn_bwd(qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:], Ls["o"], Ls["lse"], do,
                       dqkv[:, :D], dqkv[:, D:2 * D], dqkv[:, 2 * D:], vws, B=N, S=T, Hq=H, Hkv=H, causal=False,
                       dbias=self.G[p + "qkv.b"])  # qkv.b grad = column sums of dq | dk | dv, in the same kernels
            del do
            if pair:  # proj.w (g still holds ls1 * dx_mid) and qkv.w gradients as one launch
                with self._probe("vit.wgrad_attn"):
                    K.mm_pair((g, Ls["o"], self.G[p + "proj.w"]), (dqkv, Ls["h1"], self.G[p + "qkv.w"]))
            else:
                K.mm(dqkv, Ls["h1"], self.G[p + "qkv.w"], ta=True, tb=False, accumulate=True)
            self._mm_dx(dqkv, self.W[p + "qkv.w"], self.WT.get(p + "qkv.w"), dh2)
            del dqkv
            nxt = None
            if i > 0:  # the next (lower) layer's ls2 branch backward, fused onto dx_in
                q = f"vit.{i - 1}."
                nxt = (self.P[q + "ls2"], sv["vit"][i - 1]["y2"], g, self.G[q + "ls2"], self.G[q + "fc2.b"])
            K.norm_bwd(Ls["n1"], dh2, dxv, dx_accumulate=True, dgamma=self.G[p + "ln1.w"], dbeta=self.G[p + "ln1.b"],
                       ws=self._ws(K.norm_ws_floats(D)), param_accumulate=True, ls_branch=None if pr else nxt)
            if pr and nxt is not None:
                self._ls_branch_precise(dxv, *nxt)
            del dh2
            self._group_done(f"vit{i}")
        # ---------------- embeddings ----------------
        g_ = cfg.vit_grid
        dpatch = self._e(N * g_ * g_, D)
        K.call("slx_vit_embed_bwd_f32" if pr else "slx_vit_embed_bwd", K.P(dxv), N, T, D, K.P(self.G["vit.pos"]),
               K.P(self.G["vit.cls"]), K.P(dpatch), K.stream_ptr())
        dwp = self._e(D, cfg.patch_kpad, dtype=F32)
        K.mm(dpatch, sv["col"], dwp, ta=True, tb=False)
        self.G["vit.patch.w"].copy_(dwp[:, : cfg.patch_k])
        self._colsum(dpatch, self.G["vit.patch.b"])
        self._group_done("vit_embed")
        self.bucketer.mark("backward_end")
        self.saved = None

    def _lora_db(self, i, sites, dys, tx):
        """dB_j = s dy_j^T t_j. Sites of equal width whose dy columns are adjacent (k|v, gate|up) and whose B-gradient
        slices sit a fixed stride apart in the flat buffer (a, b interleaved per site) run as one batched split-K
        launch instead of one each."""
        s = self.cfg.lora_scale
        r = self.cfg.lora_r
        j = 0
        while j < len(sites):
            gb = self.G[f"llm.{i}.lora.{sites[j]}.b"]
            if j + 1 < len(sites):
                gn = self.G[f"llm.{i}.lora.{sites[j + 1]}.b"]
                out = dys[j].shape[1]
                if (dys[j + 1].shape[1] == out and dys[j + 1].data_ptr() == dys[j].data_ptr() + 2 * out
                        and gn.shape == gb.shape and gn.data_ptr() > gb.data_ptr()):
                    sC = (gn.data_ptr() - gb.data_ptr()) // 4
                    K.gemm(dys[j], tx[:, r * j:], gb, out, r, dys[j].shape[0], K.GEMM_TN, dys[j].stride(0),
                           tx.stride(0), r, alpha=s, accumulate=True, batch=2, sA=out, sB=r, sC=sC,
                           ksplit_max=LORA_DB_SPLIT)
                    j += 2
                    continue
            K.mm(dys[j], tx[:, r * j:r * (j + 1)], gb, ta=True, tb=False, alpha=s, accumulate=True,
                 ksplit_max=LORA_DB_SPLIT)
            j += 1

    def _lora_bwd(self, i, sites, dys, tx, x, dtx, dx, sv, swiglu=None, dx_bf16=None, gu_t=None):
        """LoRA sites of one group sharing the input x. dys[j] bf16 [M, out_j] (views of the output grad),
        tx bf16 [M, P] (forward down-projections t_j in columns 32j..), x bf16 [M, in] (undropped input),
        dtx f32 [M, P] (columns 32j.. hold dt_j = s dy_j B_j, produced by the fused dgrad GEMM; padding columns
        are exactly 0 because W_cat's are), dx f32 [M, in] (the base input gradient):
        dB_j = s dy_j^T t_j (GEMMs) ; dA_j = dt_j^T drop_j(x) and dx += drop_j'(dt_j A_j) in one slx_lora_bwd launch
        (dx_bf16: write bf16(dx + ...) there instead of updating dx).
        swiglu=(gu, dgu) (down projection only): the dx term and the SwiGLU backward run in one GEMM epilogue instead:
        dgu = swiglu'(gu) applied to dx + drop'(dt A). gu_t (with swiglu): the gate / up sites' forward t [M, 64], for
        slx_lora_swiglu_bwd_grads (the grouped path then forms dA_down, dB_gate and dB_up in the SwiGLU pass)."""
        cfg = self.cfg
        if self.precise:
            self._lora_bwd_precise(i, sites, dys, tx, x, dtx, dx, swiglu)
            return
        drop = sv["drop"]
        keep = sv["llm"][i]["lora"]
        bits = [keep[site] for site in sites]
        As = [self.cat[i]["axfrag." + site] for site in sites]
        if LORA_GRAD_GROUP and not self.precise and self._lg_shapes_ok():
            self._lora_bwd_grouped(i, sites, dys, tx, x, dtx, dx, swiglu, dx_bf16, drop, bits, As, sv["step_seed"],
                                   gu_t)
            return
        self._lora_db(i, sites, dys, tx)
        # dA and the dx term in one launch. (Running the parameter-only part - dB GEMMs, dA - on a side stream was
        # measured 6 ms/step slower: per-call event/stream overhead on the host and slower main-stream GEMMs.)
        K.lora_bwd(x, dtx, As, bits, [self.G[f"llm.{i}.lora.{site}.a"] for site in sites],
                   dx=None if swiglu is not None else dx, dx_bf16=dx_bf16, p=drop, packed=True)
        if swiglu is not None:
            gu, dgu = swiglu
            M = x.shape[0]
            F = gu.shape[1] // 2
            if dtx.dtype == torch.bfloat16:  # the K=64 operand straight from the bf16 dgrad output (64 columns)
                assert dtx.shape[1] == 64
                dT = dtx
            else:
                dT = self._buf(("dT_down",), M, 64)  # bf16 K=64 operand: dt_down | 32 zero columns (W_cat padding)
                K.call("slx_cast_rows", K.P(dtx), dtx.stride(0), K.P(dT), dT.stride(0), M, 64, K.stream_ptr())
            K.gemm(dT, self.cat[i]["apad.down"], dgu, M, F, 64, K.GEMM_NN, dT.stride(0), x.shape[1], dgu.stride(0),
                   epi=K.EPI_DROPMASK_SWIGLU, resid=dx, ldr=dx.stride(0), aux=gu, ldaux=gu.stride(0),
                   seed=lora_site_seed(sv["step_seed"], i, LORA_SITES.index("down")), drop_p=drop,
                   ldmask=x.shape[1], maskbits=bits[0], variant=SWIGLU_BWD_VARIANT)


    def _lora_bwd_precise(self, i, sites, dys, tx, x, dtx, dx, swiglu):
        """fp32 parity mode of _lora_bwd (no dropout): dB_j = s dy_j^T t_j, dA_j += dt_j^T x, dx += dt_j A_j as f32 GEMMs,
        then (down site) the SwiGLU backward of dx."""
        r = self.cfg.lora_r
        self._lora_db(i, sites, dys, tx)
        for j, site in enumerate(sites):
            dt = dtx[:, r * j:r * (j + 1)]
            a = f"llm.{i}.lora.{site}.a"
            K.mm(dt, x, self.G[a], ta=True, tb=False, accumulate=True)
            K.mm(dt, self.W[a], dx, tb=False, accumulate=True)
        if swiglu is not None:
            gu, dgu = swiglu
            K.call("slx_swiglu_bwd_f32", K.P(dx), dx.stride(0), K.P(gu), gu.stride(0), K.P(dgu), dgu.stride(0), x.shape[0],
                   gu.shape[1] // 2, K.stream_ptr())

    def _lora_bwd_grouped(self, i, sites, dys, tx, x, dtx, dx, swiglu, dx_bf16, drop, bits, As, step_seed, gu_t=None):
        """LORA_GRAD_GROUP: the dx term (or the down site's SwiGLU epilogue) now; dB_j and dA_j as slx_lora_grad jobs
        deferred to the layer half's _lg_flush. A dT that lives in f32 (the fused dgrad GEMM's extra columns) is
        written as bf16 by the dx kernel, the rounding the dA pass applied to it. With LORA_SWIGLU_GRADS the down site's
        SwiGLU pass forms dA_down, dB_gate and dB_up itself (the gate / up sites, which come next, then skip their dB)."""
        cfg = self.cfg
        r = cfg.lora_r
        M = x.shape[0]
        F = swiglu[0].shape[1] // 2 if swiglu is not None else 0
        fuse = (swiglu is not None and gu_t is not None and LORA_SWIGLU_BWD and LORA_SWIGLU_GRADS and F % 128 == 0
                and dtx.dtype == torch.bfloat16)
        skip_db = sites == ("gate", "up") and getattr(self, "_gu_db_fused", None) == i
        if sites == ("gate", "up"):
            self._gu_db_fused = None
        for j, site in enumerate(sites):
            if not skip_db:
                self._lg_jobs.append(dict(x=dys[j], t=tx[:, r * j:r * (j + 1)], outs=[self.G[f"llm.{i}.lora.{site}.b"]],
                                          out_nr=True, alpha=float(cfg.lora_scale)))
        if dtx.dtype == torch.bfloat16:
            dTb = dtx
        else:
            dTb = self._buf(("lg_dT",) + tuple(sites), M, r * len(sites), dtype=torch.bfloat16)
        if fuse:
            gu, dgu = swiglu
            K.lora_swiglu_bwd_grads(dtx, self.cat[i]["aT.down"], dx, gu, dgu, bits[0], drop, gu_t[:, :r],
                                    gu_t[:, r:2 * r], self.G[f"llm.{i}.lora.down.a"], self.G[f"llm.{i}.lora.gate.b"],
                                    self.G[f"llm.{i}.lora.up.b"], float(cfg.lora_scale))
            self._gu_db_fused = i
            return
        self._lg_jobs.append(dict(x=x, t=dTb, outs=[self.G[f"llm.{i}.lora.{site}.a"] for site in sites], out_nr=False,
                                  alpha=1.0, p=drop, bits=bits))
        if swiglu is None:
            K.lora_bwd(x, dtx, As, bits, None, dx=dx, dx_bf16=dx_bf16, p=drop, packed=True,
                       dt_out=None if dTb is dtx else dTb)
            return
        assert dTb is dtx, "the SwiGLU path takes dT from the bf16 dgrad output"
        gu, dgu = swiglu
        F = gu.shape[1] // 2
        if LORA_SWIGLU_BWD and F % 256 == 0:
            K.lora_swiglu_bwd(dtx, self.cat[i]["aT.down"], dx, gu, dgu, bits[0], drop)
            return
        K.gemm(dtx, self.cat[i]["apad.down"], dgu, M, F, 64, K.GEMM_NN, dtx.stride(0), x.shape[1], dgu.stride(0),
               epi=K.EPI_DROPMASK_SWIGLU, resid=dx, ldr=dx.stride(0), aux=gu, ldaux=gu.stride(0),
               seed=lora_site_seed(step_seed, i, LORA_SITES.index("down")), drop_p=drop,
               ldmask=x.shape[1], maskbits=bits[0], variant=SWIGLU_BWD_VARIANT)

    def _lg_shapes_ok(self):
        """slx_lora_grad takes 128-column blocks: every LoRA site's input and output width a multiple of 128 (the
        InternVL2-1B widths are; the tiny test geometries run the per-site path)."""
        cfg = self.cfg
        widths = (cfg.llm_dim, cfg.llm_heads * 64, cfg.llm_kv_heads * 64, cfg.llm_ffn)
        return all(w % 128 == 0 for w in widths)

    def _lg_flush(self, M):
        if self._lg_jobs:
            K.lora_grad(self._lg_jobs, M)
            self._lg_jobs = []

    # ==========================================================================================
    # optimizer
    def adamw_step(self, lr, step, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.1, max_norm=0.3):
        self.wait_grads()
        if not hasattr(self, "m_state"):
            self.m_state = torch.zeros_like(self.master)
            self.v_state = torch.zeros_like(self.master)
            self.sumsq = torch.zeros(1, dtype=F32, device=self.device)
        # the summed gradients: the f32 buffer, or (bf16 all-reduce wire) the wire buffer itself, widened in the kernels;
        # the sum of squares in a fixed order, so every data-parallel replica computes the same clip factor
        g, g_bf16 = self.bucketer.optimizer_grad()
        ws = self._sumsq_ws()
        K.call("slx_sumsq_bf16_ws" if g_bf16 else "slx_sumsq_ws", K.P(g), self.n_flat, K.P(self.sumsq), 1, K.P(ws),
               ws.numel(), K.stream_ptr())
        K.call("slx_adamw_bf16g" if g_bf16 else "slx_adamw", K.P(self.master), K.P(g), K.P(self.m_state),
               K.P(self.v_state), K.P(self.wbf),
               self.n_flat, float(lr), float(betas[0]), float(betas[1]), float(eps), float(weight_decay), int(step),
               K.P(self.sumsq), float(max_norm if max_norm else 0.0), 1.0 / self.world, K.stream_ptr())
        self._refresh_derived()

