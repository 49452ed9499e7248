"""Shared host-side plumbing of the HIP engines (VLAEngine, BaseEngine): device allocation helpers, the
norm / column-sum / small-MLP call patterns, gradient-bucket hooks and HIP-event probes. Every
computation is a libslx_hip.so call; torch only allocates and supplies the stream."""
from __future__ import annotations

import torch

from . import kernels as K

BF16, F32 = torch.bfloat16, torch.float32


class EngineOps:
    """Mixin: expects self.device, self.bucketer (GradBucketer), self.world, self.P / self.G dicts."""

    def _transpose_table(self, pairs):
        """[(w [r][c], wt [c][r]), ...] -> (device table for slx_transpose_bf16, most 64 x 64 tiles of an entry)."""
        rows = [[w.data_ptr(), w.stride(0), wt.data_ptr(), wt.stride(0), w.shape[0], w.shape[1]] for w, wt in pairs]
        tiles = max(((w.shape[0] + 63) // 64) * ((w.shape[1] + 63) // 64) for w, _ in pairs)
        return torch.tensor(rows, dtype=torch.int64, device=self.device), tiles

    def _transposed_copies(self, names):
        """W^T [in][out] for each named bf16 weight W [out][in] (self.WT), the refresh table (self._tr_tab, run by
        _refresh_transposes after every optimizer step) and one refresh now."""
        self.WT = {}
        self._tr_tab = None
        for n in names:
            w = self.W[n]
            self.WT[n] = torch.empty(w.shape[1], w.shape[0], dtype=BF16, device=self.device)
        if names:
            self._tr_tab, self._tr_tiles = self._transpose_table([(self.W[n], self.WT[n]) for n in names])
            self._refresh_transposes()

    def _refresh_transposes(self):
        if getattr(self, "_tr_tab", None) is not None:
            K.call("slx_transpose_bf16", K.P(self._tr_tab), self._tr_tab.shape[0], self._tr_tiles, K.stream_ptr())

    def _mm_dx(self, dy, w, wt, out, **kw):
        """dX = dY W for a Linear weight w [out][in]: NT over its transposed copy wt [in][out] when there is one
        (the NT main loop is 6-21% faster than NN on the steps' shapes: profiles/round3_nn_vs_nt.txt)."""
        if wt is not None:
            return K.mm(dy, wt, out, tb=True, **kw)
        return K.mm(dy, w, out, tb=False, **kw)

    def _probe(self, site):
        """Context manager: HIP events around one call site on the current stream (bench.py). `probe_site` is one
        site name or a set of them; events go to `probe_events` (a list for a single site, else {site: list})."""
        eng = self

        def on():
            ps = eng.probe_site
            return ps == site if isinstance(ps, str) else (ps is not None and site in ps)

        class _P:
            def __enter__(self):
                self.on = on()
                if self.on:
                    self.e0 = torch.cuda.Event(enable_timing=True)
                    self.e0.record()
                return self

            def __exit__(self, *a):
                if self.on:
                    e1 = torch.cuda.Event(enable_timing=True)
                    e1.record()
                    if isinstance(eng.probe_events, dict):
                        eng.probe_events.setdefault(site, []).append((self.e0, e1))
                    else:
                        eng.probe_events.append((self.e0, e1))
                return False
        return _P()

    def set_distributed(self, pg=None, world: int = 1):
        self.world = world
        self.bucketer.set_distributed(pg, world)

    def _group_done(self, g):
        self.bucketer.group_done(g)

    def wait_grads(self):
        self.bucketer.wait()

    def _e(self, *shape, dtype=None):
        """Uninitialised device buffer; default dtype = the engine's activation dtype (bf16, f32 in parity mode)."""
        return torch.empty(*shape, dtype=dtype or getattr(self, "adt", BF16), device=self.device)

    def _swiglu(self, gu, act, M, F):
        name = "slx_swiglu_fwd_f32" if gu.dtype == F32 else "slx_swiglu_fwd"
        K.call(name, K.P(gu), gu.stride(0), K.P(act), act.stride(0), M, F, K.stream_ptr())

    def _gather_feat(self, src, ld, idx, n, D, dst):
        """rows of a norm output (bf16, or f32 in parity mode) -> dst rows (f32 or bf16)."""
        if src.dtype == F32:
            K.call("slx_gather_rows", K.P(src), ld, K.P(idx), n, D, K.P(dst), dst.stride(0), int(dst.dtype == BF16),
                   K.stream_ptr())
        elif dst.dtype == F32:
            K.call("slx_gather_rows_b2f", K.P(src), ld, K.P(idx), n, D, K.P(dst), dst.stride(0), K.stream_ptr())
        else:
            K.call("slx_gather_rows_bf16", K.P(src), ld, K.P(idx), n, D, K.P(dst), dst.stride(0), K.stream_ptr())

    def _z(self, *shape, dtype=F32):
        return torch.zeros(*shape, dtype=dtype, device=self.device)

    def _buf(self, key, *shape, dtype=None, zero=False):
        """Persistent activation buffer (the step's arena): allocated (and zeroed, if asked) once per key and shape,
        then reused every step - buffers whose padding columns must stay zero are not re-filled per step."""
        dtype = dtype or getattr(self, "adt", BF16)
        arena = self.__dict__.setdefault("_arena", {})
        t = arena.get(key)
        if t is None or tuple(t.shape) != tuple(shape) or t.dtype != dtype:
            t = (torch.zeros if zero else torch.empty)(*shape, dtype=dtype, device=self.device)
            arena[key] = t
        return t

    def _norm(self, x, gamma, beta, rows, D, eps, rms=False, ps=0, tpi=0, ldx=None, out=None):
        y = self._e(rows, D) if out is None else out
        mean = None if rms else self._e(rows, dtype=F32)
        rstd = self._e(rows, dtype=F32)
        d = K.norm_desc(x, gamma, beta, y, mean, rstd, rows, D, eps, rms=rms, ps_grid=ps, tok_per_img=tpi, ldx=ldx)
        K.norm_fwd(d)
        return y, d

    def _sumsq_ws(self):
        """Partials of the ordered gradient sum of squares (slx_sumsq_ws, SLX_SUMSQ_PARTS floats)."""
        if getattr(self, "_sumsq_part", None) is None:
            self._sumsq_part = torch.empty(2048, dtype=F32, device=self.device)
        return self._sumsq_part

    def _ws(self, nfloats):
        if getattr(self, "_wsbuf", None) is None or self._wsbuf.numel() < nfloats:
            self._wsbuf = self._e(max(nfloats, 1 << 20), dtype=F32)
        return self._wsbuf

    def _colsum(self, x, out, mode=None):
        """out += column sums of x (mode 0 bf16 rows, 1 f32 rows; inferred from x when None)."""
        M, N = x.shape
        mode = int(x.dtype == F32) if mode is None else mode
        assert mode == int(x.dtype == F32), (mode, x.dtype)
        ws = self._ws(K.lib().slx_colsum_ws_floats(N))
        K.call("slx_colsum", mode, K.P(x), x.stride(0), M, N, K.P(out), 1, K.P(ws), K.stream_ptr())

    def _ls_branch_precise(self, dres, ls, y, g, dls, dbias):
        """fp32 parity mode of slx_ls_branch_bwd (and of the branch fused into slx_norm_bwd): g = dres * ls,
        dls += colsum(dres * y), dbias += colsum(g) - f32 rows throughout."""
        M, N = g.shape
        K.call("slx_mul_f32", 1, K.P(dres), dres.stride(0), K.P(ls), 0, K.P(g), g.stride(0), M, N, K.stream_ptr())
        self._colsum(g, dbias)
        if dls is not None:
            t = self._e(M, N, dtype=F32)
            K.call("slx_mul_f32", 0, K.P(dres), dres.stride(0), K.P(y), y.stride(0), K.P(t), N, M, N, K.stream_ptr())
            self._colsum(t, dls)

    def _mlp_fwd(self, x, layers):
        """driving head: list of (prefix, out_dim, act) -> saved [(out, pre, in)]"""
        saved = []
        h = x
        M = x.shape[0]
        for pre_name, n, act in layers:
            kin = h.shape[1]
            out = self._e(M, n, dtype=F32)
            pre = self._e(M, n, dtype=F32) if act != K.ACT_NONE else None
            bias = self.P.get(pre_name + ".b")
            K.sgemm(h, kin, 1, self.P[pre_name + ".w"], 1, kin, out, n, 1, M, n, kin, bias=bias, act=act, pre=pre,
                    ldpre=n)
            saved.append((out, pre, h, pre_name, act))
            h = out
        saved.reverse()
        return saved

    def _mlp_bwd(self, dout, saved, need_dx=True):
        """saved: [(out, pre, in, prefix, act)] from last layer to first; dout: grad of the last output."""
        g = dout
        for (out, pre, inp, name, act) in saved:
            M, n = g.shape
            kin = inp.shape[1]
            if act != K.ACT_NONE:
                gp = self._e(M, n, dtype=F32)
                K.call("slx_act_bwd", K.P(g), K.P(pre), K.P(gp), M * n, act, K.stream_ptr())
                g = gp
            # dW[n, kin] = g^T inp ; db = colsum(g) ; dinp = g W
            K.sgemm(g, 1, n, inp, kin, 1, self.G[name + ".w"], kin, 1, n, kin, M)
            if name + ".b" in self.G:
                K.sgemm(g, 1, n, self.ones_col(M), 1, 1, self.G[name + ".b"], 1, 1, n, 1, M)
            if inp is saved[-1][2] and not need_dx:
                break
            dinp = self._e(M, kin, dtype=F32)
            K.sgemm(g, n, 1, self.P[name + ".w"], kin, 1, dinp, kin, 1, M, kin, n)
            g = dinp
        return g

    def ones_col(self, M):
        if getattr(self, "_ones", None) is None or self._ones.numel() < M:
            self._ones = torch.ones(max(M, 1024), dtype=F32, device=self.device)
        return self._ones

    def grad_norm(self):
        """L2 norm of the (averaged) gradient the optimizer reads (after wait_grads at N > 1: the summed f32 buffer or
        the bf16 wire buffer) — diagnostic (syncs)."""
        g, _ = self.bucketer.optimizer_grad()
        return float(torch.linalg.vector_norm(g.float()).item()) / self.world
