"""SimLingo-Base training step on MI355X (BASELINE.json configs[1]).

Replaces DrivingModel.forward_loss + backward of simlingo_base_training (models/driving.py:260-324,
encoder/llavanext.py:87-113, encoder/llavanext_model.py:45-178, language_model/llama.py:96-108,
adaptors/adaptors.py:96-287): CLIP ViT-L/14-336 over the anyres patches (first vit_layers-1 layers:
hidden_states[-2]), GELU projector, spatial unpad + avg_pool + image_newline, Linear(4096 -> 512) +
encodings, speed / target-point tokens, Llama 'tiny' (all weights trainable), driving heads + MSE, then the
hand-written backward and a fused AdamW over four parameter segments (decay / no-decay x vision / rest,
configure_params_groups), global-norm clip 1.0 (train.py:189).

Same kernel library as the VLA path (libslx_hip.so): CLIP layers are the InternViT kernels with ls = 1 and
the quick_gelu GEMM epilogues; the Llama is the Qwen2 kernel set (no biases, MHA, RoPE theta 1e4) plus
weight-gradient GEMMs. Layout: flat f32 master / f32 grad / bf16 working copies (base_params.flat_layout),
residual streams f32, GEMM operands and saved activations bf16, no activation recompute.
"""
from __future__ import annotations

import math
import os

import numpy as np
import torch

from . import engine as _engine
from . import kernels as K
from .base_config import BaseConfig
from .base_params import flat_layout, init_base_params
from .ddp import GradBucketer
from .engine_ops import EngineOps
from .plan import KIND_QUERY, KIND_WP

BF16, F32 = torch.bfloat16, torch.float32
ALIGN = 64
# data-gradient GEMMs over [in][out] weight copies (engine.NT_DGRAD; 0: NN over the weights, A/B hook)
NT_DGRAD = os.environ.get("SLX_NT_DGRAD", "1") != "0"


class BaseEngine(EngineOps):
    def __init__(self, cfg: BaseConfig, device, params: dict[str, torch.Tensor] | None = None, seed: int = 0,
                 bucket_bytes: int = 32 << 20, precise: bool = False):
        """precise=True: fp32 parity mode — the same launch sequence with f32 activations and weights (the f32
        twins of csrc/precise.hip), forward only; used to hold the forward to the north-star tolerance."""
        self.cfg = cfg
        self.precise = bool(precise)
        self.adt = F32 if self.precise else BF16   # activation / GEMM-operand dtype
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise RuntimeError("BaseEngine runs on the MI355X (HIP) only; there is no CPU path")
        K.lib()
        params = params if params is not None else init_base_params(cfg, seed)
        specs, offs, bounds, n, groups = flat_layout(cfg, ALIGN)
        self.specs, self.offsets, self.seg_bounds, self.n_flat = specs, offs, bounds, n
        dev = self.device
        self.master = torch.zeros(n, dtype=F32, device=dev)
        self.grad = torch.zeros(n, dtype=F32, device=dev)
        self.wbf = torch.zeros(n, dtype=BF16, device=dev)
        self.P, self.G, self.W = {}, {}, {}
        group_ranges = {}
        for s in specs:
            o, sz = offs[s.name], math.prod(s.shape)
            self.P[s.name] = self.master[o:o + sz].view(s.shape)
            self.G[s.name] = self.grad[o:o + sz].view(s.shape)
            self.W[s.name] = self.P[s.name] if self.precise else self.wbf[o:o + sz].view(s.shape)
            self.P[s.name].copy_(params[s.name].to(dev))
            e = o + (sz + ALIGN - 1) // ALIGN * ALIGN
            a, b = group_ranges.get(groups[s.name], (o, e))
            group_ranges[groups[s.name]] = (min(a, o), max(b, e))
        self.wbf.copy_(self.master.to(BF16))
        qr, qs = offs["drv.query_route"], offs["drv.query_speed"]
        assert qs == qr + cfg.n_route * cfg.llm_dim, "query parameters must be adjacent"
        self.wpatch = torch.zeros(cfg.vit_dim, cfg.patch_kpad, dtype=self.adt, device=dev)
        self.ones_D = torch.ones(cfg.vit_dim, dtype=F32, device=dev)
        self.ones_d = torch.ones(cfg.llm_dim, dtype=F32, device=dev)
        self.bias_eff = torch.zeros(cfg.embed_dim, dtype=F32, device=dev)
        self.bucketer = GradBucketer(self.grad, group_ranges, bucket_bytes)
        self.world = 1
        self.saved = None
        self._cos_sin = {}
        self._plans = {}
        self.probe_site = None
        self.probe_events = []
        names = []
        if NT_DGRAD and not self.precise:  # every weight is trainable: all copies refreshed after each optimizer step
            names = ["enc.proj.w", "mm.fc1.w", "mm.fc2.w"]
            names += [f"vit.{i}.{n}" for i in range(cfg.vit_used) for n in ("qkv.w", "proj.w", "fc1.w", "fc2.w")]
            names += [f"llm.{i}.{n}" for i in range(cfg.llm_layers) for n in ("qkv_w", "o_w", "gate_up_w")]
        self._transposed_copies(names)
        self._refresh_derived()

    def _refresh_derived(self):
        cfg = self.cfg
        self.wpatch[:, :cfg.patch_k].copy_(self.W["vit.patch.w"])
        self._refresh_transposes()

    def rope_tables(self, S):
        if S not in self._cos_sin:
            self._cos_sin[S] = K.rope_tables(S, self.cfg.rope_theta, self.device)
        return self._cos_sin[S]

    def _static_plan(self, B):
        """Index arrays of one batch geometry (host-built once): assembly codes, the rows of the
        fixed / query / head tokens, the non-CLS rows of the CLIP output."""
        if B in self._plans:
            return self._plans[B]
        cfg = self.cfg
        Ti, S, NQ = cfg.img_tokens, cfg.seq, cfg.n_queries
        Sf = S - NQ
        code = np.empty((B, S), dtype=np.int64)
        code[:, :Sf] = (KIND_WP << 28) | (np.arange(B)[:, None] * Sf + np.arange(Sf)[None])
        code[:, Sf:] = (KIND_QUERY << 28) | np.arange(NQ)[None]
        T, g2 = cfg.vit_tokens, cfg.vit_grid ** 2
        N = B * cfg.npatch
        nocls = (np.arange(N)[:, None] * T + 1 + np.arange(g2)[None]).reshape(-1)
        fixed_pos = (np.arange(B)[:, None] * S + np.arange(Sf)[None]).reshape(-1)
        vis_rows = (np.arange(B)[:, None] * Sf + np.arange(Ti)[None]).reshape(-1)
        spd_rows = np.arange(B) * Sf + Ti
        rte_rows = (np.arange(B)[:, None] * Sf + Ti + 1 + np.arange(cfg.n_tp)[None]).reshape(-1)
        qpos = (np.arange(B)[:, None] * S + Sf + np.arange(NQ)[None]).reshape(-1)
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(torch.int32).to(self.device)
        p = dict(code=t(code.reshape(-1)), nocls=t(nocls), fixed_pos=t(fixed_pos), vis_rows=t(vis_rows),
                 spd_rows=t(spd_rows), rte_rows=t(rte_rows), qpos=t(qpos), rpos=t(qpos.reshape(B, NQ)[:, :cfg.n_route]),
                 spos=t(qpos.reshape(B, NQ)[:, cfg.n_route:]))
        self._plans[B] = p
        return p

    # ==========================================================================================
    def forward(self, pix, speed, map_route, route_label, wps_label, image_size=None):
        """pix [B, 1, 1, npatch, 3, H, W] f32; speed [B, 1]; map_route [B, n_tp, 2]; labels route_adjusted
        [B, 20, 2], waypoints [B, >=10, 2] -> (out4 = [loss, 0, route_loss, speed_wps_loss], route, speed)."""
        cfg = self.cfg
        if image_size is not None and tuple(image_size) != (cfg.frame_h, cfg.frame_w):
            raise ValueError(f"image_sizes {tuple(image_size)} != configured frame {(cfg.frame_h, cfg.frame_w)}")
        B = pix.shape[0]
        pl = self._static_plan(B)
        sv = {"B": B}
        D, T, F_, H = cfg.vit_dim, cfg.vit_tokens, cfg.vit_ffn, cfg.vit_heads
        NP, g = cfg.npatch, cfg.vit_grid
        N = B * NP
        Mv = N * T
        pix = pix.reshape(N, 3, cfg.img_size, cfg.img_size)
        if pix.dtype != F32 or not pix.is_contiguous():
            pix = pix.float().contiguous()
        # ---- CLIP embeddings + pre_layrnorm ----
        col = self._e(N * g * g, cfg.patch_kpad)
        K.call("slx_im2col_patch_f32" if self.precise else "slx_im2col_patch", K.P(pix), N, cfg.img_size, cfg.img_size, cfg.patch, cfg.patch_kpad, K.P(col),
               K.stream_ptr())
        pe = self._e(N * g * g, D, dtype=F32)
        K.mm(col, self.wpatch, pe)
        x0 = self._e(Mv, D, dtype=F32)
        K.call("slx_vit_embed_fwd", K.P(pe), K.P(self.P["vit.cls"]), K.P(self.P["vit.pos"]), K.P(x0), N, T, D,
               K.stream_ptr())
        x, npre = self._norm(x0, self.P["vit.pre_ln.w"], self.P["vit.pre_ln.b"], Mv, D, cfg.vit_eps,
                             out=self._e(Mv, D, dtype=F32))
        sv.update(col=col, npre=npre)
        vit_saved = []
        for i in range(cfg.vit_used):
            p = f"vit.{i}."
            h1, n1 = self._norm(x, self.P[p + "ln1.w"], self.P[p + "ln1.b"], Mv, D, cfg.vit_eps)
            qkv = self._e(Mv, 3 * D)
            K.mm(h1, self.W[p + "qkv.w"], qkv, bias=self.P[p + "qkv.b"])
            o = self._e(Mv, D)
            lse = self._e(N * H * T, dtype=F32)
            K.attn_fwd(qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:], o, lse, B=N, S=T, Hq=H, Hkv=H, causal=False)
            xm = self._e(Mv, D, dtype=F32)
            K.mm(o, self.W[p + "proj.w"], xm, bias=self.P[p + "proj.b"], epi=K.EPI_RESID_LS, resid=x, ldr=D,
                 ls=self.ones_D)
            h2, n2 = self._norm(xm, self.P[p + "ln2.w"], self.P[p + "ln2.b"], Mv, D, cfg.vit_eps)
            hpre, hact = self._e(Mv, F_), self._e(Mv, F_)
            hgrad = _engine.GELU_AUX_GRAD and not self.precise  # hpre then holds qgelu'(h)
            with self._probe("vit.fc1"):
                K.mm(h2, self.W[p + "fc1.w"], hact, bias=self.P[p + "fc1.b"], epi=K.EPI_QGELU, aux_out=hpre,
                     ldaux_out=F_, aux_grad=hgrad)
            xo = self._e(Mv, D, dtype=F32)
            K.mm(hact, self.W[p + "fc2.w"], xo, bias=self.P[p + "fc2.b"], epi=K.EPI_RESID_LS, resid=xm, ldr=D,
                 ls=self.ones_D)
            vit_saved.append(dict(h1=h1, n1=n1, qkv=qkv, o=o, lse=lse, h2=h2, n2=n2, hpre=hpre, hact=hact, hgrad=hgrad))
            x = xo
        sv["vit"] = vit_saved
        # ---- projector + spatial merge + projection ----
        Pd, E, d = cfg.proj_dim, cfg.embed_dim, cfg.llm_dim
        Mf = N * g * g
        feat = self._e(Mf, D)
        self._gather_feat(x, D, pl["nocls"], Mf, D, feat)
        p1pre, p1 = self._e(Mf, Pd), self._e(Mf, Pd)
        K.mm(feat, self.W["mm.fc1.w"], p1, bias=self.P["mm.fc1.b"], epi=K.EPI_GELU, aux_out=p1pre, ldaux_out=Pd)
        p2 = self._e(Mf, Pd)
        K.mm(p1, self.W["mm.fc2.w"], p2, bias=self.P["mm.fc2.b"])
        r0, hu, c0, wu = cfg.unpad()
        Ti = cfg.img_tokens
        merged = self._e(B * Ti, Pd)
        K.call("slx_llava_merge_fwd_f32" if self.precise else "slx_llava_merge_fwd", K.P(p2), Pd, B, cfg.npatch_h, cfg.npatch_w, g, r0, hu, c0, wu, cfg.pool,
               K.P(self.P["mm.newline"]), K.P(merged), K.stream_ptr())
        S, NQ = cfg.seq, cfg.n_queries
        Sf = S - NQ
        pre = self._e(B * Sf, d, dtype=F32)
        K.call("slx_vec_sum3", K.P(self.P["enc.proj.b"]), K.P(self.P["enc.temporal"]), K.P(self.P["enc.camera"]), E,
               K.P(self.bias_eff), K.stream_ptr())
        K.gemm(merged, self.W["enc.proj.w"], pre, Ti, E, Pd, K.GEMM_NT, Pd, Pd, d, bias=self.bias_eff, batch=B,
               sA=Ti * Pd, sB=0, sC=Sf * d)
        sv.update(feat=feat, p1pre=p1pre, p1=p1, merged=merged)
        # ---- speed / target-point tokens (VectorInputAdaptor, WaypointInputAdaptor with NormZeroOne) ----
        sn = self._e(B, 1, dtype=F32)
        K.call("slx_affine", K.P(speed.reshape(B, 1).float().contiguous()), B, 1.0 / (cfg.speed_max - cfg.speed_min),
               -cfg.speed_min / (cfg.speed_max - cfg.speed_min), K.P(sn), K.stream_ptr())
        ntp = B * cfg.n_tp
        tn = self._e(ntp, 2, dtype=F32)
        K.call("slx_affine", K.P(map_route.reshape(ntp, 2).float().contiguous()), ntp * 2, 1.0 / (cfg.tp_max - cfg.tp_min),
               -cfg.tp_min / (cfg.tp_max - cfg.tp_min), K.P(tn), K.stream_ptr())
        h_ = cfg.in_hidden
        spd = self._mlp_fwd(sn, [("spd.0", h_, K.ACT_RELU), ("spd.1", d, K.ACT_NONE)])
        rte = self._mlp_fwd(tn, [("rte.0", h_, K.ACT_RELU), ("rte.1", d, K.ACT_NONE)])
        K.call("slx_scatter_rows", K.P(spd[0][0]), d, K.P(pl["spd_rows"]), B, d, K.P(pre), d, 0, K.stream_ptr())
        K.call("slx_scatter_rows", K.P(rte[0][0]), d, K.P(pl["rte_rows"]), ntp, d, K.P(pre), d, 0, K.stream_ptr())
        sv.update(spd=spd, rte=rte)
        # ---- [fixed | queries] -> Llama ----
        Ml = B * S
        X = self._e(Ml, d, dtype=F32)
        K.call("slx_assemble_tokens_f32" if self.precise else "slx_assemble_tokens", K.P(pl["code"]), Ml, d, K.P(None), 1, K.P(None), K.P(pre),
               K.P(self.P["drv.query_route"]), K.P(X), K.stream_ptr())
        Hh, Fl = cfg.llm_heads, cfg.llm_ffn
        cos, sin = self.rope_tables(S)
        llm_saved = []
        for i in range(cfg.llm_layers):
            p = f"llm.{i}."
            h, n1 = self._norm(X, self.P[p + "ln1"], None, Ml, d, cfg.rms_eps, rms=True)
            qkv = self._e(Ml, 3 * d)
            K.mm(h, self.W[p + "qkv_w"], qkv)
            K.rope(qkv, Ml, S, 2 * Hh, cos, sin)
            o = self._e(Ml, d)
            lse = self._e(B * Hh * S, dtype=F32)
            K.attn_fwd(qkv[:, :d], qkv[:, d:2 * d], qkv[:, 2 * d:], o, lse, B=B, S=S, Hq=Hh, Hkv=Hh, causal=True)
            Xm = self._e(Ml, d, dtype=F32)
            K.mm(o, self.W[p + "o_w"], Xm, epi=K.EPI_RESID_LS, resid=X, ldr=d, ls=self.ones_d)
            h2, n2 = self._norm(Xm, self.P[p + "ln2"], None, Ml, d, cfg.rms_eps, rms=True)
            gu = self._e(Ml, 2 * Fl)
            K.mm(h2, self.W[p + "gate_up_w"], gu)
            act = self._e(Ml, Fl)
            self._swiglu(gu, act, Ml, Fl)
            Xo = self._e(Ml, d, dtype=F32)
            K.mm(act, self.W[p + "down_w"], Xo, epi=K.EPI_RESID_LS, resid=Xm, ldr=d, ls=self.ones_d)
            llm_saved.append(dict(h=h, n1=n1, qkv=qkv, o=o, lse=lse, h2=h2, n2=n2, gu=gu, act=act))
            X = Xo
        sv["llm"] = llm_saved
        featL, nf = self._norm(X, self.P["llm.norm"], None, Ml, d, cfg.rms_eps, rms=True)
        # ---- driving heads + MSE (adaptors.py:163-232) ----
        nr, ns = cfg.n_route, cfg.n_speed
        fr, fs = self._e(B * nr, d, dtype=F32), self._e(B * ns, d, dtype=F32)
        self._gather_feat(featL, d, pl["rpos"], B * nr, d, fr)
        self._gather_feat(featL, d, pl["spos"], B * ns, d, fs)
        m = cfg.head_mlp
        hd = self._mlp_fwd(fr, [("route.0", m, K.ACT_SILU), ("route.1", 2, K.ACT_NONE)])
        sd_ = self._mlp_fwd(fs, [("speed.0", m, K.ACT_SILU), ("speed.1", cfg.speed_dims, K.ACT_NONE)])
        lab_r = route_label.float().contiguous()
        lab_s = wps_label[:, :ns].float().contiguous()
        route_pred, speed_pred = self._e(B, nr, 2, dtype=F32), self._e(B, ns, cfg.speed_dims, dtype=F32)
        route_loss, speed_loss = self._e(B * nr, dtype=F32), self._e(B * ns, dtype=F32)
        K.call("slx_wp_loss_fwd", K.P(hd[0][0]), K.P(lab_r), B, nr, 2, 1, K.P(route_pred), K.P(route_loss),
               K.stream_ptr())
        K.call("slx_wp_loss_fwd", K.P(sd_[0][0]), K.P(lab_s), B, ns, cfg.speed_dims, 1, K.P(speed_pred),
               K.P(speed_loss), K.stream_ptr())
        out4 = self._e(4, dtype=F32)
        K.call("slx_loss_finalize", K.P(route_loss), 0, K.P(route_loss), B * nr, K.P(speed_loss), B * ns, K.P(out4),
               K.stream_ptr())
        sv.update(X_last=X, nf=nf, hd=hd, sd=sd_, lab_r=lab_r, lab_s=lab_s, route_pred=route_pred,
                  speed_pred=speed_pred, Mv=Mv, N=N, Mf=Mf, Ml=Ml, pl=pl)
        self.saved = sv
        return out4, route_pred, speed_pred

    # ==========================================================================================
    def backward(self, dlosses: torch.Tensor | None = None):
        cfg = self.cfg
        sv = self.saved
        assert sv is not None, "backward() without forward()"
        if self.precise:
            raise RuntimeError("the fp32 parity mode is forward-only (it pins the forward outputs)")
        B, Mv, N, Mf, Ml, pl = sv["B"], sv["Mv"], sv["N"], sv["Mf"], sv["Ml"], sv["pl"]
        D, d, Pd, E = cfg.vit_dim, cfg.llm_dim, cfg.proj_dim, cfg.embed_dim
        nr, ns = cfg.n_route, cfg.n_speed
        S, NQ = cfg.seq, cfg.n_queries
        Sf, Ti = S - NQ, cfg.img_tokens
        self.grad.zero_()
        gs = self._e(3, dtype=F32)
        if dlosses is not None:
            dlosses = dlosses.float().contiguous()
        K.call("slx_loss_gscale", K.P(dlosses), 0, B * nr, B * ns, K.P(gs), K.stream_ptr())
        # ---- heads ----
        dfeat = self._z(Ml + 1, d)
        for tag, npts, dims, saved, lab, pos, pred in (("route", nr, 2, sv["hd"], sv["lab_r"], pl["rpos"], sv["route_pred"]),
                                                        ("speed", ns, cfg.speed_dims, sv["sd"], sv["lab_s"], pl["spos"],
                                                         sv["speed_pred"])):
            dout = self._e(B * npts, dims, dtype=F32)
            K.call("slx_wp_loss_bwd", K.P(pred), K.P(lab), B, npts, dims, 1,
                   K.P(gs[1:2] if tag == "route" else gs[2:3]), K.P(dout), K.stream_ptr())
            dx = self._mlp_bwd(dout, saved)
            K.call("slx_scatter_rows", K.P(dx), d, K.P(pos), B * npts, d, K.P(dfeat), d, 1, K.stream_ptr())
        self._group_done("heads")
        dX = self._z(Ml + 1, d)
        dxb = self._e(Ml, d)  # bf16 copy of dX written by every norm backward that updates dX
        K.norm_bwd(sv["nf"], dfeat, dX, dgamma=self.G["llm.norm"], param_accumulate=True,
                   ws=self._ws(K.norm_ws_floats(d)), dx_bf16=dxb)
        # ---- Llama (all weights trainable) ----
        Hh, Fl = cfg.llm_heads, cfg.llm_ffn
        cos, sin = self.rope_tables(S)
        ws = K.attn_ws(B, S, Hh, Hh, self.device, rope=True)
        for i in reversed(range(cfg.llm_layers)):
            p = f"llm.{i}."
            L = sv["llm"][i]
            K.mm(dxb, L["act"], self.G[p + "down_w"], ta=True, tb=False, accumulate=True)
            dgu = self._e(Ml, 2 * Fl)
            K.gemm(dxb, self.W[p + "down_w"], dgu, Ml, Fl, d, K.GEMM_NN, d, Fl, 2 * Fl, epi=K.EPI_SWIGLU_BWD,
                   aux=L["gu"], ldaux=2 * Fl)
            K.mm(dgu, L["h2"], self.G[p + "gate_up_w"], ta=True, tb=False, accumulate=True)
            dh2 = self._e(Ml, d, dtype=F32)
            self._mm_dx(dgu, self.W[p + "gate_up_w"], self.WT.get(p + "gate_up_w"), dh2)
            del dgu
            K.norm_bwd(L["n2"], dh2, dX, dx_accumulate=True, dgamma=self.G[p + "ln2"], param_accumulate=True,
                       ws=self._ws(K.norm_ws_floats(d)), dx_bf16=dxb)
            K.mm(dxb, L["o"], self.G[p + "o_w"], ta=True, tb=False, accumulate=True)
            do = self._e(Ml, d)
            self._mm_dx(dxb, self.W[p + "o_w"], self.WT.get(p + "o_w"), do)
            qkv = L["qkv"]
            dqkv = self._e(Ml, 3 * d)
            K.attn_bwd(qkv[:, :d], qkv[:, d:2 * d], qkv[:, 2 * d:], L["o"], L["lse"], do, dqkv[:, :d], dqkv[:, d:2 * d],
                       dqkv[:, 2 * d:], ws, rope_cos=cos, rope_sin=sin, B=B, S=S, Hq=Hh, Hkv=Hh, causal=True)
            K.mm(dqkv, L["h"], self.G[p + "qkv_w"], ta=True, tb=False, accumulate=True)
            dh = self._e(Ml, d, dtype=F32)
            self._mm_dx(dqkv, self.W[p + "qkv_w"], self.WT.get(p + "qkv_w"), dh)
            K.norm_bwd(L["n1"], dh, dX, dx_accumulate=True, dgamma=self.G[p + "ln1"], param_accumulate=True,
                       ws=self._ws(K.norm_ws_floats(d)), dx_bf16=dxb)
            del dqkv, dh, dh2, do
            self._group_done(f"llm{i}")
        # ---- assembly backward: queries, speed / target-point encoders ----
        K.call("slx_gather_sum", K.P(dX), d, K.P(pl["qpos"]), B, NQ, d, K.P(self.G["drv.query_route"]), 0,
               K.stream_ptr())
        dpre = self._e(B * Sf, d, dtype=F32)
        K.call("slx_gather_rows", K.P(dX), d, K.P(pl["fixed_pos"]), B * Sf, d, K.P(dpre), d, 0, K.stream_ptr())
        for tag, rows, n in (("spd", pl["spd_rows"], B), ("rte", pl["rte_rows"], B * cfg.n_tp)):
            g_ = self._e(n, d, dtype=F32)
            K.call("slx_gather_rows", K.P(dpre), d, K.P(rows), n, d, K.P(g_), d, 0, K.stream_ptr())
            self._mlp_bwd(g_, sv[tag], need_dx=False)
        self._group_done("inputs")
        # ---- projection + encodings ----
        nv = B * Ti
        dvis = self._e(nv, d, dtype=F32)
        K.call("slx_gather_rows", K.P(dpre), d, K.P(pl["vis_rows"]), nv, d, K.P(dvis), d, 0, K.stream_ptr())
        dvisb = self._e(nv, d)
        K.call("slx_cast_rows", K.P(dvis), d, K.P(dvisb), d, nv, d, K.stream_ptr())
        self._colsum(dvis, self.G["enc.proj.b"], 1)
        self.G["enc.temporal"].copy_(self.G["enc.proj.b"])
        self.G["enc.camera"].copy_(self.G["enc.proj.b"])
        K.mm(dvisb, sv["merged"], self.G["enc.proj.w"], ta=True, tb=False, accumulate=True)
        dmerged = self._e(nv, Pd, dtype=F32)
        self._mm_dx(dvisb, self.W["enc.proj.w"], self.WT.get("enc.proj.w"), dmerged)
        del dvis, dvisb, dpre
        # image_newline: the last column of every pooled row
        r0, hu, c0, wu = cfg.unpad()
        wo = wu // cfg.pool
        K.call("slx_colsum", 1, K.P(dmerged[wo:]), (wo + 1) * Pd, B * (hu // cfg.pool), Pd, K.P(self.G["mm.newline"]), 1,
               K.P(self._ws(1)), K.stream_ptr())
        g = cfg.vit_grid
        dp2 = self._e(Mf, Pd)
        K.call("slx_llava_merge_bwd", K.P(dmerged), Pd, B, cfg.npatch_h, cfg.npatch_w, g, r0, hu, c0, wu, cfg.pool,
               K.P(dp2), K.stream_ptr())
        del dmerged
        K.mm(dp2, sv["p1"], self.G["mm.fc2.w"], ta=True, tb=False, accumulate=True)
        self._colsum(dp2, self.G["mm.fc2.b"], 0)
        dp1 = self._e(Mf, Pd)
        self._mm_dx(dp2, self.W["mm.fc2.w"], self.WT.get("mm.fc2.w"), dp1, epi=K.EPI_GELU_BWD, aux=sv["p1pre"], ldaux=Pd,
             colsum=self.G["mm.fc1.b"])
        del dp2
        K.mm(dp1, sv["feat"], self.G["mm.fc1.w"], ta=True, tb=False, accumulate=True)
        dfeatv = self._e(Mf, D, dtype=F32)
        self._mm_dx(dp1, self.W["mm.fc1.w"], self.WT.get("mm.fc1.w"), dfeatv)
        del dp1
        dxv = self._z(Mv, D)
        K.call("slx_scatter_rows", K.P(dfeatv), D, K.P(pl["nocls"]), Mf, D, K.P(dxv), D, 0, K.stream_ptr())
        del dfeatv
        self._group_done("venc")
        # ---- CLIP layers ----
        F_, H, T = cfg.vit_ffn, cfg.vit_heads, cfg.vit_tokens
        vws = K.attn_ws(N, T, H, H, self.device)
        gb = self._e(Mv, D)
        nws = self._ws(K.norm_ws_floats(D))
        for i in reversed(range(cfg.vit_used)):
            p = f"vit.{i}."
            L = sv["vit"][i]
            # xo = xm + fc2(qgelu(fc1(ln2(xm))))
            K.call("slx_ls_branch_bwd", K.P(dxv), D, K.P(None), K.P(None), D, K.P(gb), D, Mv, D, K.P(None),
                   K.P(self.G[p + "fc2.b"]), 1, K.P(None), K.stream_ptr())
            K.mm(gb, L["hact"], self.G[p + "fc2.w"], ta=True, tb=False, accumulate=True)
            dh = self._e(Mv, F_)
            self._mm_dx(gb, self.W[p + "fc2.w"], self.WT.get(p + "fc2.w"), dh, epi=K.EPI_QGELU_BWD, aux=L["hpre"], ldaux=F_,
                 colsum=self.G[p + "fc1.b"], aux_grad=L["hgrad"])
            K.mm(dh, L["h2"], self.G[p + "fc1.w"], ta=True, tb=False, accumulate=True)
            dh2 = self._e(Mv, D, dtype=F32)
            self._mm_dx(dh, self.W[p + "fc1.w"], self.WT.get(p + "fc1.w"), dh2)
            del dh
            K.norm_bwd(L["n2"], dh2, dxv, dx_accumulate=True, dgamma=self.G[p + "ln2.w"], dbeta=self.G[p + "ln2.b"],
                       ws=nws, param_accumulate=True)
            # xm = x + out_proj(attn(ln1(x)))
            K.call("slx_ls_branch_bwd", K.P(dxv), D, K.P(None), K.P(None), D, K.P(gb), D, Mv, D, K.P(None),
                   K.P(self.G[p + "proj.b"]), 1, K.P(None), K.stream_ptr())
            K.mm(gb, L["o"], self.G[p + "proj.w"], ta=True, tb=False, accumulate=True)
            do = self._e(Mv, D)
            self._mm_dx(gb, self.W[p + "proj.w"], self.WT.get(p + "proj.w"), do)
            qkv = L["qkv"]
            dqkv = self._e(Mv, 3 * D)
            K.attn_bwd(qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:], L["o"], L["lse"], do, dqkv[:, :D],
                       dqkv[:, D:2 * D], dqkv[:, 2 * D:], vws, B=N, S=T, Hq=H, Hkv=H, causal=False)
            del do
            K.mm(dqkv, L["h1"], self.G[p + "qkv.w"], ta=True, tb=False, accumulate=True)
            self._colsum(dqkv, self.G[p + "qkv.b"], 0)
            self._mm_dx(dqkv, self.W[p + "qkv.w"], self.WT.get(p + "qkv.w"), dh2)
            del dqkv
            K.norm_bwd(L["n1"], dh2, dxv, dx_accumulate=True, dgamma=self.G[p + "ln1.w"], dbeta=self.G[p + "ln1.b"],
                       ws=nws, param_accumulate=True)
            del dh2
            self._group_done(f"vit{i}")
        # ---- pre_layrnorm + embeddings ----
        dx0 = self._e(Mv, D, dtype=F32)
        K.norm_bwd(sv["npre"], dxv, dx0, dgamma=self.G["vit.pre_ln.w"], dbeta=self.G["vit.pre_ln.b"], ws=nws,
                   param_accumulate=True)
        del dxv
        dpatch = self._e(N * g * g, D)
        K.call("slx_vit_embed_bwd", K.P(dx0), N, T, D, K.P(self.G["vit.pos"]), K.P(self.G["vit.cls"]), K.P(dpatch),
               K.stream_ptr())
        dwp = self._e(D, cfg.patch_kpad, dtype=F32)
        K.mm(dpatch, sv["col"], dwp, ta=True, tb=False)
        self.G["vit.patch.w"].copy_(dwp[:, :cfg.patch_k])
        self._group_done("vit_embed")
        self._group_done("nodecay")
        self.saved = None

    # ==========================================================================================
    def adamw_step(self, lr, vision_lr, step, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.1, max_norm=1.0):
        """torch AdamW over the four segments of base_params.flat_layout (decay / no decay x rest / vision),
        after one global-norm clip (train.py:189 gradient_clip_val=1.0)."""
        self.wait_grads()
        if not hasattr(self, "m_state"):
            self.m_state = torch.zeros_like(self.master)
            self.v_state = torch.zeros_like(self.master)
            self.sumsq = torch.zeros(1, dtype=F32, device=self.device)
        ws = self._sumsq_ws()  # fixed-order sum: identical clip factor on every data-parallel replica
        K.call("slx_sumsq_ws", K.P(self.grad), self.n_flat, K.P(self.sumsq), 1, K.P(ws), ws.numel(), K.stream_ptr())
        hp = ((lr, weight_decay), (vision_lr, weight_decay), (vision_lr, 0.0), (lr, 0.0))
        for (a, b), (lr_k, wd_k) in zip(self.seg_bounds, hp):
            if b <= a:
                continue
            K.call("slx_adamw", K.P(self.master[a:]), K.P(self.grad[a:]), K.P(self.m_state[a:]), K.P(self.v_state[a:]),
                   K.P(self.wbf[a:]), b - a, float(lr_k), float(betas[0]), float(betas[1]), float(eps), float(wd_k),
                   int(step), K.P(self.sumsq), float(max_norm if max_norm else 0.0), 1.0 / self.world, K.stream_ptr())
        self._refresh_derived()
