"""ctypes binding of libslx_hip.so (include/slx.h).

PyTorch supplies device memory and the current HIP stream; every computation happens in the HIP
library. There is deliberately no fallback: if the library is missing or a call fails, a
RuntimeError is raised (a silent eager/CPU path would void every parity claim).
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import torch

# SLX_LIB_PATH: load another build of the library (A/B of two builds in alternating processes); the in-tree build
# is the default and the only one the product path ships
_LIB_PATH = Path(os.environ.get("SLX_LIB_PATH") or Path(__file__).resolve().parent / "csrc" / "libslx_hip.so")
_lib = None

c_int, c_i64, c_u64, c_float, c_vp = ctypes.c_int, ctypes.c_int64, ctypes.c_uint64, ctypes.c_float, ctypes.c_void_p

# ---- enums (mirror include/slx.h) --------------------------------------------------------------
GEMM_NT, GEMM_NN, GEMM_TN, GEMM_TT = 0, 1, 2, 3
GEMM_VARIANT = int(os.environ.get("SLX_GEMM_VARIANT", "0"))  # 0 = automatic (tuning hook)
EPI_STORE, EPI_GELU, EPI_RESID_LS, EPI_GELU_BWD, EPI_SWIGLU_BWD, EPI_DROPMASK, EPI_DROPMASK_SWIGLU = 0, 1, 2, 3, 4, 5, 6
EPI_QGELU, EPI_QGELU_BWD = 7, 8


class GemmDesc(ctypes.Structure):
    _fields_ = [
        ("layout", c_int), ("epilogue", c_int), ("out_f32", c_int),
        ("M", c_int), ("N", c_int), ("K", c_int), ("batch", c_int),
        ("A", c_vp), ("lda", c_i64), ("sA", c_i64),
        ("B", c_vp), ("ldb", c_i64), ("sB", c_i64),
        ("C", c_vp), ("ldc", c_i64), ("sC", c_i64),
        ("alpha", c_float),
        ("bias", c_vp), ("ls", c_vp),
        ("aux", c_vp), ("ldaux", c_i64),
        ("aux_out", c_vp), ("ldaux_out", c_i64),
        ("resid", c_vp), ("ldr", c_i64),
        ("accumulate", c_int),
        ("seed", c_u64), ("drop_p", c_float), ("ldmask", c_i64),
        ("ksplit_max", c_int), ("variant", c_int), ("drop_operand", c_int),
        ("colsum", c_vp), ("colsum_ws", c_vp), ("maskbits", c_vp), ("ldbits", c_i64), ("rem_ws", c_vp),
        ("rem_ws_floats", c_i64), ("resid_bf16", c_int), ("split_ws", c_vp), ("split_ws_floats", c_i64),
        ("rope_cos", c_vp), ("rope_sin", c_vp), ("rope_S", c_int), ("rope_ncols", c_int), ("aux_grad", c_int),
    ]


class GemmLtDesc(ctypes.Structure):  # slx_gemm_lt_desc
    _fields_ = [
        ("M", c_i64), ("N", c_i64), ("K", c_i64),
        ("A", c_vp), ("lda", c_i64), ("B", c_vp), ("ldb", c_i64),
        ("C", c_vp), ("ldc", c_i64), ("D", c_vp), ("ldd", c_i64),
        ("alpha", c_float), ("beta", c_float), ("out_f32", c_int),
        ("ws", c_vp), ("ws_bytes", c_i64),
    ]


# name -> argtypes (restype int unless listed in _RESTYPE)
_SIGS: dict[str, list] = {
    "slx_gemm_lt": [ctypes.POINTER(GemmLtDesc), c_vp],
    "slx_abi_version": [],
    "slx_device_sync": [],
    "slx_gemm_bf16": [ctypes.POINTER(GemmDesc), c_vp],
    "slx_gemm_bf16_pair": [ctypes.POINTER(GemmDesc), ctypes.POINTER(GemmDesc), c_vp],
}
_RESTYPE = {"slx_last_error": ctypes.c_char_p}


def lib():
    global _lib
    if _lib is None:
        if not _LIB_PATH.exists():
            raise RuntimeError(
                f"{_LIB_PATH} is not built: run `python -m simlingo_amd.build` (hipcc, gfx950). "
                "There is no CPU/eager fallback for the SimLingo MI355X kernels.")
        _lib = ctypes.CDLL(str(_LIB_PATH))
        _lib.slx_last_error.restype = ctypes.c_char_p
        _lib.slx_last_error.argtypes = []
        for name, args in _SIGS.items():
            f = getattr(_lib, name)
            f.argtypes = args
            f.restype = _RESTYPE.get(name, c_int)
    return _lib


def register(name: str, argtypes: list, restype=None):
    """Declare a C-ABI entry point (used by modules that add bindings); restype defaults to int."""
    _SIGS[name] = argtypes
    if restype is not None:
        _RESTYPE[name] = restype
    if _lib is not None:
        f = getattr(_lib, name)
        f.argtypes = argtypes
        f.restype = _RESTYPE.get(name, c_int)


def exported_symbols() -> list[str]:
    return ["slx_last_error"] + list(_SIGS)


def check(rc: int, name: str):
    if rc != 0:
        msg = lib().slx_last_error().decode(errors="replace")
        raise RuntimeError(f"{name} failed (rc={rc}): {msg}")


def call(name: str, *args):
    check(getattr(lib(), name)(*args), name)


def stream_ptr() -> c_vp:
    return c_vp(torch.cuda.current_stream().cuda_stream)


def P(t: torch.Tensor | None) -> c_vp:
    """Raw device pointer of a tensor (None -> NULL)."""
    if t is None:
        return c_vp(0)
    return c_vp(t.data_ptr())


def _require_cuda(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("SimLingo MI355X kernels need device tensors (no CPU fallback)")


# ------------------------------------------------------------------------------------------------
# GEMM
# ------------------------------------------------------------------------------------------------
_colsum_ws: dict = {}  # per-device partials workspace of the colsum epilogue (stream-ordered reuse)
_rem_ws: dict = {}     # per-device split-K scratch of the M-remainder rows (stream-ordered reuse)
REM_WS_FLOATS = 16 << 20  # 64 MB: 32 splits x 64 rows x 8192 columns
_split_ws: dict = {}   # per-stream in-launch split-K slabs of the 256x256 kernel (weight gradients)
SPLIT_WS_FLOATS = (32 << 20) + 16384  # 128 MB of slabs (e.g. 128 tiles x 4 splits) + 16384 counter words
SPLIT_WS_ON = os.environ.get("SLX_SPLIT_WS", "1") != "0"  # A/B hook: 0 = split-K partials through f32 atomics


def gemm(A, B, C, M, N, K, layout, lda, ldb, ldc, **kw):
    d = _gemm_desc(A, B, C, M, N, K, layout, lda, ldb, ldc, **kw)
    if A.dtype == torch.float32:  # fp32 parity mode (csrc/precise.hip)
        if B.dtype != torch.float32 or C.dtype != torch.float32:
            raise RuntimeError("fp32 parity-mode GEMM needs f32 A, B and C")
        colsum = kw.get("colsum")
        d.colsum = d.colsum_ws = 0  # the f32 twin has no fused colsum: the output's column sums separately
        check(lib().slx_gemm_f32(ctypes.byref(d), stream_ptr()), "slx_gemm_f32")
        if colsum is not None:
            call("slx_colsum", 1, C.data_ptr(), int(ldc), int(M), int(N), colsum.data_ptr(), 1, 0, stream_ptr())
        rope = kw.get("rope")
        if rope is not None:  # the f32 kernels have no fused RoPE epilogue: the separate rotation
            cos, sin, rs, rn = rope
            rope_rows(C, M, rs, rn // 64, cos, sin)
        return
    check(lib().slx_gemm_bf16(ctypes.byref(d), stream_ptr()), "slx_gemm_bf16")


def _gemm_desc(A, B, C, M, N, K, layout, lda, ldb, ldc, *, epi=EPI_STORE, alpha=1.0, bias=None, ls=None,
               aux=None, ldaux=0, aux_out=None, ldaux_out=0, resid=None, ldr=0, accumulate=False,
               seed=0, drop_p=0.0, ldmask=0, batch=1, sA=0, sB=0, sC=0, ksplit_max=0, variant=None, drop_operand=0,
               colsum=None, maskbits=None, split_ws=True, rope=None, aux_grad=False):
    _require_cuda(A, B, C)
    if aux_grad and A.dtype == torch.float32:
        raise RuntimeError("aux_grad (derivative stored as the GELU aux) is a bf16-path option; the fp32 parity "
                           "kernels store the pre-activation")
    d = GemmDesc()
    d.aux_grad = 1 if aux_grad else 0
    d.layout, d.epilogue = layout, epi
    d.out_f32 = 1 if C.dtype == torch.float32 else 0
    d.M, d.N, d.K, d.batch = int(M), int(N), int(K), int(batch)
    d.A, d.lda, d.sA = A.data_ptr(), int(lda), int(sA)
    d.B, d.ldb, d.sB = B.data_ptr(), int(ldb), int(sB)
    d.C, d.ldc, d.sC = C.data_ptr(), int(ldc), int(sC)
    d.alpha = float(alpha)
    d.bias = bias.data_ptr() if bias is not None else 0
    d.ls = ls.data_ptr() if ls is not None else 0
    d.aux = aux.data_ptr() if aux is not None else 0
    d.ldaux = int(ldaux)
    d.aux_out = aux_out.data_ptr() if aux_out is not None else 0
    d.ldaux_out = int(ldaux_out)
    d.resid = resid.data_ptr() if resid is not None else 0
    d.resid_bf16 = int(resid is not None and resid.dtype == torch.bfloat16)
    d.ldr = int(ldr)
    d.accumulate = 1 if accumulate else 0
    d.seed, d.drop_p, d.ldmask = int(seed) & ((1 << 64) - 1), float(drop_p), int(ldmask)
    d.ksplit_max = int(ksplit_max)
    d.variant = int(GEMM_VARIANT if variant is None else variant)
    d.drop_operand = int(drop_operand)
    d.colsum = colsum.data_ptr() if colsum is not None else 0
    if maskbits is not None:
        d.maskbits, d.ldbits = maskbits.data_ptr(), maskbits.stride(0)
    sk = (C.device, torch.cuda.current_stream(C.device).cuda_stream)  # one workspace per stream (side-stream GEMMs)
    rw = _rem_ws.get(sk)
    if rw is None:
        # zeroed once: the last 4096 words are the folded-remainder arrival counters (reset by every GEMM that uses them)
        rw = _rem_ws[sk] = torch.zeros(REM_WS_FLOATS, dtype=torch.float32, device=C.device)
    d.rem_ws, d.rem_ws_floats = rw.data_ptr(), rw.numel()
    if split_ws and SPLIT_WS_ON and d.out_f32 and d.epilogue == EPI_STORE:
        sw = _split_ws.get(sk)
        if sw is None:
            # zeroed once: the last 16384 words are the in-launch split-K arrival counters (left zero by every call)
            sw = _split_ws[sk] = torch.zeros(SPLIT_WS_FLOATS, dtype=torch.float32, device=C.device)
        d.split_ws, d.split_ws_floats = sw.data_ptr(), sw.numel()
    if rope is not None:  # (cos, sin, S, ncols): RoPE fused into a bf16 STORE epilogue (the Qwen2 q|k columns)
        cos, sin, rs, rn = rope
        _require_cuda(cos, sin)
        d.rope_cos, d.rope_sin, d.rope_S, d.rope_ncols = cos.data_ptr(), sin.data_ptr(), int(rs), int(rn)
    if colsum is not None:
        need = (int(M) + 63) // 64 * int(N)
        ws = _colsum_ws.get(sk)
        if ws is None or ws.numel() < need:
            ws = torch.empty(max(need, 1 << 20), dtype=torch.float32, device=C.device)
            _colsum_ws[sk] = ws
        d.colsum_ws = ws.data_ptr()
    return d


def linear(x: torch.Tensor, w: torch.Tensor, out: torch.Tensor, bias=None, **kw):
    """out[M,N] = x[M,K] @ w[N,K]^T (+bias) — 2-D row-major views with unit inner stride."""
    M, K = x.shape
    N = w.shape[0]
    gemm(x, w, out, M, N, K, GEMM_NT, x.stride(0), w.stride(0), out.stride(0), bias=bias, **kw)
    return out


def dgrad(dy: torch.Tensor, w: torch.Tensor, out: torch.Tensor, **kw):
    """out[M,K] = dy[M,N] @ w[N,K]."""
    M, N = dy.shape
    K = w.shape[1]
    gemm(dy, w, out, M, K, N, GEMM_NN, dy.stride(0), w.stride(0), out.stride(0), **kw)
    return out


def wgrad(dy: torch.Tensor, x: torch.Tensor, out: torch.Tensor, **kw):
    """out[N,K] = dy[M,N]^T @ x[M,K]."""
    M, N = dy.shape
    K = x.shape[1]
    gemm(dy, x, out, N, K, M, GEMM_TN, dy.stride(0), x.stride(0), out.stride(0), **kw)
    return out


# ------------------------------------------------------------------------------------------------
# Attention
# ------------------------------------------------------------------------------------------------
class AttnDesc(ctypes.Structure):
    _fields_ = [
        ("B", c_int), ("S", c_int), ("Hq", c_int), ("Hkv", c_int), ("head_dim", c_int), ("causal", c_int),
        ("q", c_vp), ("ldq", c_i64), ("k", c_vp), ("ldk", c_i64), ("v", c_vp), ("ldv", c_i64),
        ("o", c_vp), ("ldo", c_i64), ("lse", c_vp), ("seqlens", c_vp), ("scale", c_float),
    ]


class AttnBwdDesc(ctypes.Structure):
    _fields_ = [
        ("dout", c_vp), ("lddo", c_i64), ("dq", c_vp), ("lddq", c_i64), ("dk", c_vp), ("lddk", c_i64),
        ("dv", c_vp), ("lddv", c_i64), ("delta_ws", c_vp), ("dq_acc", c_vp), ("dk_acc", c_vp), ("dv_acc", c_vp),
        ("rope_cos", c_vp), ("rope_sin", c_vp), ("dbias_q", c_vp), ("dbias_k", c_vp), ("dbias_v", c_vp),
    ]


class NormDesc(ctypes.Structure):
    _fields_ = [
        ("rms", c_int), ("x", c_vp), ("ldx", c_i64), ("gamma", c_vp), ("beta", c_vp), ("y", c_vp), ("ldy", c_i64),
        ("mean", c_vp), ("rstd", c_vp), ("rows", c_i64), ("D", c_int), ("eps", c_float),
        ("pixel_shuffle_grid", c_int), ("tokens_per_image", c_int), ("y_f32", c_int),
        ("dx_bf16", c_vp), ("lddx_bf16", c_i64),
        ("ls", c_vp), ("ls_y", c_vp), ("ld_ls_y", c_i64), ("ls_g", c_vp), ("ld_ls_g", c_i64), ("ls_dls", c_vp),
        ("ls_dbias", c_vp), ("dy_bf16", c_int),
    ]


ACT_NONE, ACT_RELU, ACT_SILU = 0, 1, 2


class SgemmDesc(ctypes.Structure):
    _fields_ = [
        ("M", c_int), ("N", c_int), ("K", c_int), ("act", c_int), ("accumulate", c_int),
        ("A", c_vp), ("sam", c_i64), ("sak", c_i64), ("B", c_vp), ("sbk", c_i64), ("sbn", c_i64),
        ("C", c_vp), ("scm", c_i64), ("scn", c_i64), ("bias", c_vp), ("pre", c_vp), ("ldpre", c_i64),
        ("alpha", c_float),
    ]


class LoraDownDesc(ctypes.Structure):
    _fields_ = [
        ("x", c_vp), ("ldx", c_i64), ("M", c_i64), ("Kin", c_int), ("r", c_int), ("nsites", c_int),
        ("A", c_vp * 4), ("seed", ctypes.c_uint64 * 4), ("t", c_vp), ("ldt", c_i64), ("p", c_float), ("ldmask", c_i64),
        ("bits", c_vp * 4), ("ldbits", c_i64), ("gen_bits", c_int),
    ]


class DropoutBitsJob(ctypes.Structure):
    _fields_ = [("seed", ctypes.c_uint64), ("bits", c_vp), ("ldbits", c_i64), ("ldmask", c_i64), ("cols", c_int)]


class DropoutBitsDesc(ctypes.Structure):
    _fields_ = [("njobs", c_int), ("p", c_float), ("rows", c_i64), ("job", DropoutBitsJob * 8)]


class LoraBwdDesc(ctypes.Structure):
    _fields_ = [
        ("x", c_vp), ("ldx", c_i64), ("M", c_i64), ("Kin", c_int), ("r", c_int), ("nsites", c_int),
        ("dt", c_vp), ("lddt", c_i64), ("A", c_vp * 4), ("bits", c_vp * 4), ("ldbits", c_i64), ("dA", c_vp * 4),
        ("dx", c_vp), ("lddx", c_i64), ("dx_bf16", c_vp), ("lddx_bf16", c_i64), ("p", c_float), ("dt_bf16", c_int),
        ("dt_bf16_out", c_vp), ("ld_dt_bf16_out", c_i64),
    ]


class LoraGradJob(ctypes.Structure):
    _fields_ = [
        ("x", c_vp), ("ldx", c_i64), ("n", c_int), ("t", c_vp), ("ldt", c_i64), ("t_bf16", c_int), ("nsites", c_int),
        ("bits", c_vp * 3), ("ldbits", c_i64), ("p", c_float), ("alpha", c_float), ("out", c_vp * 3), ("out_nr", c_int),
    ]


_vp, _i, _I, _f = c_vp, c_int, c_i64, c_float
for _n, _a in {
    "slx_attn_fwd": [ctypes.POINTER(AttnDesc), _vp],
    "slx_lora_down": [ctypes.POINTER(LoraDownDesc), _vp],
    "slx_lora_pack_a": [_vp, ctypes.c_int64, ctypes.c_int, ctypes.c_int, _vp, _vp],
    "slx_lora_bwd": [ctypes.POINTER(LoraBwdDesc), _vp],
    "slx_lora_bwd_ws": [ctypes.POINTER(LoraBwdDesc), _vp, _I, _vp],
    "slx_lora_grad": [ctypes.POINTER(LoraGradJob), _i, _I, _vp],
    "slx_dropout_bits": [ctypes.POINTER(DropoutBitsDesc), _vp],
    "slx_attn_bwd": [ctypes.POINTER(AttnDesc), ctypes.POINTER(AttnBwdDesc), _vp],
    "slx_rope": [_vp, _I, _I, _i, _i, _vp, _vp, _i, _vp],
    "slx_norm_fwd": [ctypes.POINTER(NormDesc), _vp],
    "slx_norm_bwd": [ctypes.POINTER(NormDesc), _vp, _I, _vp, _I, _i, _vp, _vp, _i, _vp, _vp],
    "slx_norm_partial_ws_floats": [_i],
    "slx_im2col_patch": [_vp, _i, _i, _i, _i, _i, _vp, _vp],
    "slx_vit_embed_fwd": [_vp, _vp, _vp, _vp, _i, _i, _i, _vp],
    "slx_vit_embed_bwd": [_vp, _i, _i, _i, _vp, _vp, _vp, _vp],
    "slx_swiglu_fwd": [_vp, _I, _vp, _I, _I, _i, _vp],
    "slx_colsum": [_i, _vp, _I, _I, _i, _vp, _i, _vp, _vp],
    "slx_colsum_ws_floats": [_i],
    "slx_ls_branch_bwd": [_vp, _I, _vp, _vp, _I, _vp, _I, _I, _i, _vp, _vp, _i, _vp, _vp],
    "slx_assemble_tokens": [_vp, _I, _i, _vp, _i, _vp, _vp, _vp, _vp, _vp],
    "slx_gather_rows": [_vp, _I, _vp, _I, _i, _vp, _I, _i, _vp],
    "slx_gather_rows_bf16": [_vp, _I, _vp, _I, _i, _vp, _I, _vp],
    "slx_gather_sum": [_vp, _I, _vp, _i, _i, _i, _vp, _i, _vp],
    "slx_dropout": [_vp, _I, _vp, _I, _I, _i, c_u64, _f, _I, _vp],
    "slx_sgemm": [ctypes.POINTER(SgemmDesc), _vp],
    "slx_act_bwd": [_vp, _vp, _vp, _I, _i, _vp],
    "slx_ce_fwd": [_vp, _I, _vp, _I, _i, _vp, _vp, _vp],
    "slx_ce_bwd": [_vp, _I, _vp, _vp, _I, _i, _vp, _vp, _I, _vp],
    "slx_lmhead_ce_ws_floats": [_I, _i],
    "slx_lmhead_ce_fwd": [_vp, _I, _vp, _I, _vp, _I, _i, _i, _vp, _vp, _vp, _I, _vp],
    "slx_lmhead_ce_bwd": [_vp, _I, _vp, _I, _vp, _vp, _I, _i, _i, _vp, _vp, _I, _vp],
    "slx_wp_loss_fwd": [_vp, _vp, _i, _i, _i, _i, _vp, _vp, _vp],
    "slx_wp_loss_bwd": [_vp, _vp, _i, _i, _i, _i, _vp, _vp, _vp],
    "slx_affine": [_vp, _I, _f, _f, _vp, _vp],
    "slx_vec_sum3": [_vp, _vp, _vp, _I, _vp, _vp],
    "slx_llava_merge_tokens": [_i, _i, _i],
    "slx_llava_merge_fwd": [_vp, _i, _I, _i, _i, _i, _i, _i, _i, _i, _i, _vp, _vp, _vp],
    "slx_llava_merge_bwd": [_vp, _i, _I, _i, _i, _i, _i, _i, _i, _i, _i, _vp, _vp],
    "slx_loss_finalize": [_vp, _i, _vp, _i, _vp, _i, _vp, _vp],
    "slx_loss_gscale": [_vp, _i, _i, _i, _vp, _vp],
    "slx_sumsq": [_vp, _I, _vp, _i, _vp],
    "slx_adamw": [_vp, _vp, _vp, _vp, _vp, _I, _f, _f, _f, _f, _f, _i, _vp, _f, _f, _vp],
    "slx_scatter_rows": [_vp, _I, _vp, _I, _i, _vp, _I, _i, _vp],
    "slx_gather_rows_b2f": [_vp, _I, _vp, _I, _i, _vp, _I, _vp],
    "slx_swiglu_bwd": [_vp, _I, _vp, _I, _vp, _I, _I, _i, _vp],
    "slx_cast_rows": [_vp, _I, _vp, _I, _I, _i, _vp],
    "slx_pack_scaled": [_vp, _i, _vp],
    "slx_pack_scaled_flat": [_vp, _i, _vp, _i, _vp],
    "slx_transpose_bf16": [_vp, _i, _I, _vp],
    "slx_cast_f32_bf16": [_vp, _vp, _I, _vp],
    # fp32 parity mode (csrc/precise.hip)
    "slx_gemm_f32": [ctypes.POINTER(GemmDesc), _vp],
    "slx_attn_fwd_f32": [ctypes.POINTER(AttnDesc), _vp],
    "slx_rope_f32": [_vp, _I, _I, _i, _i, _vp, _vp, _i, _vp],
    "slx_swiglu_fwd_f32": [_vp, _I, _vp, _I, _I, _i, _vp],
    "slx_im2col_patch_f32": [_vp, _i, _i, _i, _i, _i, _vp, _vp],
    "slx_assemble_tokens_f32": [_vp, _I, _i, _vp, _i, _vp, _vp, _vp, _vp, _vp],
    "slx_llava_merge_fwd_f32": [_vp, _i, _I, _i, _i, _i, _i, _i, _i, _i, _i, _vp, _vp, _vp],
    "slx_attn_bwd_f32": [ctypes.POINTER(AttnDesc), ctypes.POINTER(AttnBwdDesc), _vp],
    "slx_swiglu_bwd_f32": [_vp, _I, _vp, _I, _vp, _I, _I, _i, _vp],
    "slx_mul_f32": [_i, _vp, _I, _vp, _I, _vp, _I, _I, _i, _vp],
    "slx_ce_bwd_f32": [_vp, _I, _vp, _vp, _I, _i, _vp, _vp, _I, _vp],
    "slx_vit_embed_bwd_f32": [_vp, _i, _i, _i, _vp, _vp, _vp, _vp],
    "slx_set_deterministic": [_i, _vp, _I],
    "slx_sumsq_bf16": [_vp, _I, _vp, _i, _vp],
    "slx_sumsq_ws": [_vp, _I, _vp, _i, _vp, _I, _vp],
    "slx_mfma_peak": [_i, _i, _vp, _vp],
    "slx_sumsq_bf16_ws": [_vp, _I, _vp, _i, _vp, _I, _vp],
    "slx_adamw_bf16g": [_vp, _vp, _vp, _vp, _vp, _I, _f, _f, _f, _f, _f, _i, _vp, _f, _f, _vp],
    "slx_get_deterministic": [],
}.items():
    register(_n, _a)
register("slx_lora_bwd_ws_floats", [_I, _i, _i], restype=c_i64)  # int64_t result (include/slx.h)


def attn_desc(q, k, v, o, lse, *, B, S, Hq, Hkv, causal=False, seqlens=None, scale=0.125):
    d = AttnDesc()
    d._keep = (q, k, v, o, lse, seqlens)
    d.B, d.S, d.Hq, d.Hkv, d.head_dim, d.causal = B, S, Hq, Hkv, 64, int(bool(causal))
    d.q, d.ldq = q.data_ptr(), q.stride(0)
    d.k, d.ldk = k.data_ptr(), k.stride(0)
    d.v, d.ldv = v.data_ptr(), v.stride(0)
    d.o, d.ldo = o.data_ptr(), o.stride(0)
    d.lse = lse.data_ptr() if lse is not None else 0
    d.seqlens = seqlens.data_ptr() if seqlens is not None else 0
    d.scale = float(scale)
    return d


def attn_fwd(q, k, v, o, lse, **kw):
    """q/k/v/o: 2-D token-major views [B*S, >= H*64] (column slices allowed)."""
    _require_cuda(q, k, v, o)
    d = attn_desc(q, k, v, o, lse, **kw)
    name = "slx_attn_fwd_f32" if q.dtype == torch.float32 else "slx_attn_fwd"  # f32: parity mode
    check(getattr(lib(), name)(ctypes.byref(d), stream_ptr()), name)


def attn_bwd(q, k, v, o, lse, dout, dq, dk, dv, ws, *, rope_cos=None, rope_sin=None, dbias=None, **kw):
    """ws: attn_ws(...) f32 buffers (delta, dq_acc, and dk_acc/dv_acc for GQA or RoPE).
    dbias: optional f32 [3 * Hq * 64] (q | k | v bias gradients) += column sums of dq, dk, dv (no GQA, no RoPE)."""
    d = attn_desc(q, k, v, o, lse, **kw)
    g = AttnBwdDesc()
    g.dout, g.lddo = dout.data_ptr(), dout.stride(0)
    g.dq, g.lddq = dq.data_ptr(), dq.stride(0)
    g.dk, g.lddk = dk.data_ptr(), dk.stride(0)
    g.dv, g.lddv = dv.data_ptr(), dv.stride(0)
    g.delta_ws = ws["delta"].data_ptr()
    g.dq_acc = ws["dq_acc"].data_ptr()
    g.dk_acc = ws["dk_acc"].data_ptr() if "dk_acc" in ws else 0
    g.dv_acc = ws["dv_acc"].data_ptr() if "dv_acc" in ws else 0
    g.rope_cos = rope_cos.data_ptr() if rope_cos is not None else 0
    g.rope_sin = rope_sin.data_ptr() if rope_sin is not None else 0
    if dbias is not None:
        n = d.Hq * 64
        assert dbias.dtype == torch.float32 and dbias.is_contiguous() and dbias.numel() == 3 * n
        g.dbias_q, g.dbias_k, g.dbias_v = dbias.data_ptr(), dbias.data_ptr() + 4 * n, dbias.data_ptr() + 8 * n
    if q.dtype == torch.float32:  # fp32 parity mode: the plain restatement, then RoPE^T and the bias column sums
        g.rope_cos = g.rope_sin = g.dbias_q = g.dbias_k = g.dbias_v = 0
        check(lib().slx_attn_bwd_f32(ctypes.byref(d), ctypes.byref(g), stream_ptr()), "slx_attn_bwd_f32")
        ntok = d.B * d.S
        if rope_cos is not None:
            rope(dq, ntok, d.S, d.Hq, rope_cos, rope_sin, inverse=True)
            rope(dk, ntok, d.S, d.Hkv, rope_cos, rope_sin, inverse=True)
        if dbias is not None:
            n = d.Hq * 64
            for j, t in enumerate((dq, dk, dv)):
                call("slx_colsum", 1, P(t), t.stride(0), ntok, n, dbias.data_ptr() + 4 * n * j, 1, 0, stream_ptr())
        return
    if dbias is not None and deterministic():  # the fused bias sums end in f32 atomics: ordered column sums instead
        g.dbias_q = g.dbias_k = g.dbias_v = 0
        check(lib().slx_attn_bwd(ctypes.byref(d), ctypes.byref(g), stream_ptr()), "slx_attn_bwd")
        n = d.Hq * 64
        for j, t in enumerate((dq, dk, dv)):
            call("slx_colsum", int(t.dtype == torch.float32), P(t), t.stride(0), d.B * d.S, n,
                 dbias.data_ptr() + 4 * n * j, 1, 0, stream_ptr())
        return
    check(lib().slx_attn_bwd(ctypes.byref(d), ctypes.byref(g), stream_ptr()), "slx_attn_bwd")


def attn_ws(B, S, Hq, Hkv, device, rope=False):
    """f32 workspaces of slx_attn_bwd: delta, dq_acc; dk_acc/dv_acc [B*S, Hq*64] (head-split partials) for GQA
    or RoPE."""
    ws = {"delta": torch.empty(B * Hq * S, device=device), "dq_acc": torch.empty(B * S * Hq * 64, device=device)}
    if Hq != Hkv or rope:
        ws["dk_acc"] = torch.empty(B * S * Hq * 64, device=device)
        ws["dv_acc"] = torch.empty(B * S * Hq * 64, device=device)
    return ws


_det_ws: dict = {}
DET_WS_FLOATS = 16 << 20  # 64 MB: the largest partial set of the InternVL2-1B step (LoRA MLP half, ~2.2 M floats) x 7


def set_deterministic(on: bool, device=None):
    """Deterministic-reduction mode (slx_set_deterministic, process-wide): every cross-block f32 reduction of the step
    goes through per-block partials and an ordered sum instead of f32 atomics, so two runs on the same inputs give
    bitwise-equal gradients. The workspace is allocated once per device and kept. The library holds ONE workspace
    pointer for the process, so the mode serves one device per process (the one-process-per-GPU model): turning it on
    for a second device while it is on for another raises."""
    if on:
        dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        if dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        other = [d for d in _det_ws if d != dev]
        if other and deterministic():
            raise RuntimeError(f"deterministic mode is already on for {other[0]}; the library's workspace is "
                               f"process-wide (one device per process)")
        ws = _det_ws.get(dev)
        if ws is None:
            ws = _det_ws[dev] = torch.empty(DET_WS_FLOATS, dtype=torch.float32, device=dev)
        check(lib().slx_set_deterministic(1, P(ws), ws.numel()), "slx_set_deterministic")
    else:
        check(lib().slx_set_deterministic(0, None, 0), "slx_set_deterministic")


def deterministic() -> bool:
    return bool(lib().slx_get_deterministic())


def rope_rows(x, ntok, S, nheads, cos, sin):
    rope(x, ntok, S, nheads, cos, sin)


def rope(x, ntok, S, nheads, cos, sin, inverse=False):
    call("slx_rope_f32" if x.dtype == torch.float32 else "slx_rope", P(x), x.stride(0), ntok, S, nheads, P(cos), P(sin),
         int(inverse), stream_ptr())


def rope_tables(S, theta, device, head_dim=64):
    """HF Qwen2RotaryEmbedding: inv_freq[i] = theta^(-2i/d); tables [S, d/2] f32."""
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.int64).float() / head_dim))
    t = torch.arange(S, dtype=torch.int64).float()
    fr = torch.outer(t, inv)
    return fr.cos().to(device).contiguous(), fr.sin().to(device).contiguous()


# ------------------------------------------------------------------------------------------------
# Norms
# ------------------------------------------------------------------------------------------------
def norm_desc(x, gamma, beta, y, mean, rstd, rows, D, eps, rms=False, ps_grid=0, tok_per_img=0, ldx=None):
    """y may be bf16 (GEMM operand) or f32 (a residual stream, e.g. CLIP's pre_layrnorm)."""
    """The descriptor keeps references to every tensor it points to (ctypes holds raw pointers only;
    without this the caching allocator could recycle the saved statistics before the backward)."""
    d = NormDesc()
    d._keep = (x, gamma, beta, y, mean, rstd)
    d.rms = int(rms)
    d.x, d.ldx = x.data_ptr(), ldx if ldx is not None else x.stride(0)
    d.gamma = gamma.data_ptr()
    d.beta = beta.data_ptr() if beta is not None else 0
    d.y, d.ldy = (y.data_ptr(), y.stride(0)) if y is not None else (0, 0)
    d.mean = mean.data_ptr() if mean is not None else 0
    d.rstd = rstd.data_ptr()
    d.rows, d.D, d.eps = int(rows), int(D), float(eps)
    d.pixel_shuffle_grid, d.tokens_per_image = int(ps_grid), int(tok_per_img)
    d.y_f32 = int(y is not None and y.dtype == torch.float32)
    return d


def norm_fwd(d: NormDesc):
    check(lib().slx_norm_fwd(ctypes.byref(d), stream_ptr()), "slx_norm_fwd")


def norm_bwd(d: NormDesc, dy, dx, *, dx_accumulate=False, dgamma=None, dbeta=None, param_accumulate=False, ws=None,
             lddx=None, dx_bf16=None, ls_branch=None):
    """dy: f32 or bf16 rows. dx_bf16: optional bf16 [rows, >= D] view that receives a bf16 copy of the (accumulated) dx
    in the same pass.
    ls_branch = (ls f32 [D], y bf16 [rows, D], g bf16 [rows, D], dls f32 [D], dbias f32 [D]): the layer-scale branch
    backward (slx_ls_branch_bwd, accumulating) fused onto the updated dx rows."""
    d.dx_bf16, d.lddx_bf16 = (dx_bf16.data_ptr(), dx_bf16.stride(0)) if dx_bf16 is not None else (0, 0)
    assert dy.dtype in (torch.float32, torch.bfloat16)
    d.dy_bf16 = int(dy.dtype == torch.bfloat16)
    if ls_branch is not None:
        ls, y, g, dls, dbias = ls_branch
        d.ls, d.ls_y, d.ld_ls_y, d.ls_g, d.ld_ls_g = ls.data_ptr(), y.data_ptr(), y.stride(0), g.data_ptr(), g.stride(0)
        d.ls_dls, d.ls_dbias = dls.data_ptr(), dbias.data_ptr()
    else:
        d.ls = d.ls_y = d.ls_g = d.ls_dls = d.ls_dbias = 0
    check(lib().slx_norm_bwd(ctypes.byref(d), P(dy), dy.stride(0), P(dx), lddx if lddx is not None else dx.stride(0),
                             int(dx_accumulate), P(dgamma), P(dbeta), int(param_accumulate), P(ws), stream_ptr()),
          "slx_norm_bwd")


def norm_ws_floats(D):
    return lib().slx_norm_partial_ws_floats(D)


def sgemm(A, sam, sak, B, sbk, sbn, C, scm, scn, M, N, Kd, *, bias=None, act=ACT_NONE, pre=None, ldpre=0,
          accumulate=False, alpha=1.0):
    d = SgemmDesc()
    d.M, d.N, d.K, d.act, d.accumulate = int(M), int(N), int(Kd), int(act), int(accumulate)
    d.A, d.sam, d.sak = A.data_ptr(), sam, sak
    d.B, d.sbk, d.sbn = B.data_ptr(), sbk, sbn
    d.C, d.scm, d.scn = C.data_ptr(), scm, scn
    d.bias = bias.data_ptr() if bias is not None else 0
    d.pre = pre.data_ptr() if pre is not None else 0
    d.ldpre = ldpre
    d.alpha = alpha
    check(lib().slx_sgemm(ctypes.byref(d), stream_ptr()), "slx_sgemm")


def dropout_bits(jobs, rows, p):
    """Keep masks as bits, one launch for up to 8 (seed, bits int32 [rows, >= cols/32], cols, ldmask) jobs:
    bits[r][w] bit c = keep(seed, r*ldmask + 32w + c) (common.h drop_keep; host mirror simlingo_amd.dropmask)."""
    assert 1 <= len(jobs) <= 8 and p > 0
    d = DropoutBitsDesc()
    d.njobs, d.p, d.rows = len(jobs), float(p), int(rows)
    for j, (seed, bits, cols, ldmask) in enumerate(jobs):
        assert bits.dtype == torch.int32 and bits.shape[0] >= rows and bits.shape[1] * 32 >= cols and bits.is_cuda
        d.job[j].seed = int(seed) & ((1 << 64) - 1)
        d.job[j].bits, d.job[j].ldbits, d.job[j].ldmask, d.job[j].cols = bits.data_ptr(), bits.stride(0), int(ldmask), int(cols)
    check(lib().slx_dropout_bits(ctypes.byref(d), stream_ptr()), "slx_dropout_bits")


def lora_pack_a(a, layout=0, out=None):
    """A [32, kin] bf16 (peft lora_A.weight layout) -> a packed fragment order: layout 0 is read by slx_lora_down,
    layout 1 by slx_lora_bwd's dx term."""
    assert a.dtype == torch.bfloat16 and a.dim() == 2 and a.shape[0] == 32 and a.stride(1) == 1
    out = torch.empty(32 * a.shape[1], device=a.device, dtype=torch.bfloat16) if out is None else out
    assert out.dtype == torch.bfloat16 and out.is_contiguous() and out.numel() == a.numel()
    check(lib().slx_lora_pack_a(P(a), a.stride(0), a.shape[1], int(layout), P(out), stream_ptr()), "slx_lora_pack_a")
    return out


def lora_down(x, As, t, seeds, p=0.0, ldmask=None, bits=None, packed=False, gen=False):
    """t[:, 32j:32j+32] = drop_j(x) As[j]^T for the sites sharing x (one launch); p > 0: bits[j] (int32
    [M, >= kin/32]) holds site j's keep mask (dropout_bits), or with gen=True the kernel generates it from seeds[j]
    (the same drop_keep hash) and writes it there for the backward.
    packed=True: As[j] are already in slx_lora_pack_a's fragment order (flat, 32 * kin elements); else the [32, kin]
    matrices are packed here first (one extra launch per site)."""
    assert x.dtype == torch.bfloat16 and t.dtype == torch.bfloat16 and 1 <= len(As) <= 4
    M, kin = x.shape
    assert t.shape[0] == M and t.shape[1] >= 32 * len(As)
    if not packed:
        for a in As:
            assert a.shape == (32, kin)
        As = [lora_pack_a(a, 0) for a in As]
    d = LoraDownDesc()
    d.x, d.ldx, d.M, d.Kin, d.r, d.nsites = P(x).value, x.stride(0), M, kin, 32, len(As)
    for j, a in enumerate(As):
        assert a.numel() == 32 * kin and a.is_contiguous() and a.dtype == torch.bfloat16
        d.A[j] = a.data_ptr()
        d.seed[j] = int(seeds[j]) & ((1 << 64) - 1)
        if bits is not None and bits[j] is not None:
            assert bits[j].dtype == torch.int32 and bits[j].shape[0] == M and bits[j].shape[1] * 32 >= kin
            d.bits[j] = bits[j].data_ptr()
            d.ldbits = bits[j].stride(0)
    d.t, d.ldt, d.p, d.ldmask = P(t).value, t.stride(0), float(p), kin if ldmask is None else ldmask
    d.gen_bits = int(bool(gen))
    check(lib().slx_lora_down(ctypes.byref(d), stream_ptr()), "slx_lora_down")


_lora_ws: dict = {}  # per-stream dA partials of slx_lora_bwd_ws
# SLX_LORA_DA_SLAB=1: the LoRA A gradients through per-row-chunk partials + an in-order sum (slx_lora_bwd_ws) instead of
# the dA kernel's f32 atomics
LORA_DA_SLAB = os.environ.get("SLX_LORA_DA_SLAB", "0") == "1"


def lora_bwd(x, dt, As, bits, dAs, dx=None, dx_bf16=None, p=0.0, packed=False, dt_out=None):
    """peft LoRA backward of the sites sharing x (one launch): dAs[j] (f32 [32, kin]) += dT_j^T drop_j(x) (dAs=None:
    skipped) and, if dx (f32 [M, kin]) is given, dx += sum_j drop_j'(dT_j As[j]) in place - or written as
    bf16(dx + ...) to dx_bf16.
    dt: f32 or bf16 [M, >= 32 n] (dT_j = columns 32j..); bits[j]: keep bits from lora_down (None when p == 0).
    As: [32, kin] matrices (packed here into slx_lora_pack_a layout 1 when dx is asked for), or with packed=True the
    layout-1 copies themselves (only the dx term reads A)."""
    assert x.dtype == torch.bfloat16 and dt.dtype in (torch.float32, torch.bfloat16) and 1 <= len(As) <= 4
    M, kin = x.shape
    assert dt.shape[0] == M and dt.shape[1] >= 32 * len(As) and dt.stride(1) == 1
    d = LoraBwdDesc()
    d.dt_bf16 = int(dt.dtype == torch.bfloat16)
    d.x, d.ldx, d.M, d.Kin, d.r, d.nsites = P(x).value, x.stride(0), M, kin, 32, len(As)
    d.dt, d.lddt = P(dt).value, dt.stride(0)
    if not packed:
        for a in As:
            assert a.shape == (32, kin) and a.dtype == torch.bfloat16
        As = [lora_pack_a(a, 1) for a in As] if dx is not None else As
    for j, a in enumerate(As):
        assert a.numel() == 32 * kin and a.is_contiguous() and a.dtype == torch.bfloat16
        d.A[j] = a.data_ptr()
        if dAs is not None:  # None: dx only
            g = dAs[j]
            assert g.shape == (32, kin) and g.is_contiguous() and g.dtype == torch.float32
            d.dA[j] = g.data_ptr()
        if p > 0:
            assert bits[j] is not None and bits[j].shape[0] == M
            d.bits[j] = bits[j].data_ptr()
            d.ldbits = bits[j].stride(0)
    if dx is not None:
        assert dx.dtype == torch.float32 and dx.shape[0] == M and dx.shape[1] >= kin
        d.dx, d.lddx = dx.data_ptr(), dx.stride(0)
    if dx_bf16 is not None:
        assert dx_bf16.dtype == torch.bfloat16 and dx_bf16.shape[0] == M
        d.dx_bf16, d.lddx_bf16 = dx_bf16.data_ptr(), dx_bf16.stride(0)
    if dt_out is not None:  # the dx kernel also writes the bf16 dT (slx_lora_grad's operand)
        assert dx is not None and dt_out.dtype == torch.bfloat16 and dt_out.shape[0] == M and dt_out.stride(1) == 1
        assert dt_out.shape[1] >= 32 * len(As)
        d.dt_bf16_out, d.ld_dt_bf16_out = dt_out.data_ptr(), dt_out.stride(0)
    d.p = float(p)
    if LORA_DA_SLAB and dAs is not None:  # dA summed through per-row-chunk partials (no f32 atomics, deterministic)
        need = lib().slx_lora_bwd_ws_floats(M, kin, len(As))
        sk = (x.device, torch.cuda.current_stream(x.device).cuda_stream)
        ws = _lora_ws.get(sk)
        if ws is None or ws.numel() < need:
            ws = _lora_ws[sk] = torch.empty(need, dtype=torch.float32, device=x.device)
        check(lib().slx_lora_bwd_ws(ctypes.byref(d), P(ws), ws.numel(), stream_ptr()), "slx_lora_bwd_ws")
        return
    check(lib().slx_lora_bwd(ctypes.byref(d), stream_ptr()), "slx_lora_bwd")


class LoraSwigluBwdDesc(ctypes.Structure):
    _fields_ = [("dt", c_vp), ("lddt", c_i64), ("at", c_vp), ("ldat", c_i64), ("resid", c_vp), ("ldr", c_i64),
                ("gu", c_vp), ("ldgu", c_i64), ("bits", c_vp), ("ldbits", c_i64), ("p", c_float), ("dgu", c_vp),
                ("lddgu", c_i64), ("M", c_i64), ("F", c_int)]


register("slx_lora_swiglu_bwd", [ctypes.POINTER(LoraSwigluBwdDesc), c_vp])


def lora_swiglu_bwd(dt, at, resid, gu, dgu, bits, p):
    """slx_lora_swiglu_bwd: dgu = SwiGLU'(gu) applied to d = resid + keep * (dT[:, :32] . A) / (1 - p).
    dt bf16 [M, >= 32] view, at bf16 [F, 32] (A^T), resid bf16 [M, F] view, gu bf16 [M, 2F], dgu bf16 [M, 2F],
    bits int32 [M, >= F/32] (p > 0)."""
    M, F = resid.shape
    for t in (dt, at, resid, gu, dgu):
        assert t.dtype == torch.bfloat16 and t.is_cuda and t.stride(1) == 1
    assert at.shape == (F, 32) and gu.shape[0] == M and gu.shape[1] >= 2 * F and dgu.shape[1] >= 2 * F
    assert dt.shape[0] == M and dt.shape[1] >= 32
    d = LoraSwigluBwdDesc()
    d.dt, d.lddt, d.at, d.ldat = dt.data_ptr(), dt.stride(0), at.data_ptr(), at.stride(0)
    d.resid, d.ldr, d.gu, d.ldgu = resid.data_ptr(), resid.stride(0), gu.data_ptr(), gu.stride(0)
    if p > 0:
        assert bits is not None and bits.dtype == torch.int32 and bits.shape[0] == M and bits.shape[1] * 32 >= F
        d.bits, d.ldbits = bits.data_ptr(), bits.stride(0)
    d.p, d.dgu, d.lddgu, d.M, d.F = float(p), dgu.data_ptr(), dgu.stride(0), M, F
    check(lib().slx_lora_swiglu_bwd(ctypes.byref(d), stream_ptr()), "slx_lora_swiglu_bwd")


class LoraSwigluBwdGradsDesc(ctypes.Structure):
    _fields_ = [("sw", LoraSwigluBwdDesc), ("tg", c_vp), ("tu", c_vp), ("ldtg", c_i64), ("dA_down", c_vp),
                ("dB_gate", c_vp), ("dB_up", c_vp), ("alpha_b", c_float), ("ws", c_vp), ("ws_floats", c_i64)]


register("slx_lora_swiglu_bwd_grads_ws_floats", [c_i64, c_int], restype=c_i64)
register("slx_lora_swiglu_bwd_grads", [ctypes.POINTER(LoraSwigluBwdGradsDesc), c_vp])
_lswg_ws = {}


def lora_swiglu_bwd_grads(dt, at, resid, gu, dgu, bits, p, tg, tu, dA_down, dB_gate, dB_up, alpha_b):
    """slx_lora_swiglu_bwd_grads: lora_swiglu_bwd's dgu, and from the same pass dA_down [32, F] += dT^T drop(act),
    dB_gate / dB_up [F, 32] += alpha_b dgu[:, :F]^T tg / dgu[:, F:]^T tu. tg, tu bf16 [M, 32] views (same stride),
    the three outputs f32 contiguous."""
    M, F = resid.shape
    for t in (dt, at, resid, gu, dgu, tg, tu):
        assert t.dtype == torch.bfloat16 and t.is_cuda and t.stride(1) == 1
    assert at.shape == (F, 32) and gu.shape[0] == M and gu.shape[1] >= 2 * F and dgu.shape[1] >= 2 * F
    assert dt.shape[0] == M and dt.shape[1] >= 32
    assert tg.shape == (M, 32) and tu.shape == (M, 32) and tg.stride(0) == tu.stride(0)
    assert dA_down.shape == (32, F) and dB_gate.shape == (F, 32) and dB_up.shape == (F, 32)
    for t in (dA_down, dB_gate, dB_up):
        assert t.dtype == torch.float32 and t.is_contiguous()
    need = int(lib().slx_lora_swiglu_bwd_grads_ws_floats(M, F))
    key = (dt.device, torch.cuda.current_stream(dt.device).cuda_stream)
    ws = _lswg_ws.get(key)
    if ws is None or ws.numel() < need:
        ws = _lswg_ws[key] = torch.empty(need, dtype=torch.float32, device=dt.device)
    s = LoraSwigluBwdDesc()
    s.dt, s.lddt, s.at, s.ldat = dt.data_ptr(), dt.stride(0), at.data_ptr(), at.stride(0)
    s.resid, s.ldr, s.gu, s.ldgu = resid.data_ptr(), resid.stride(0), gu.data_ptr(), gu.stride(0)
    if p > 0:
        assert bits is not None and bits.dtype == torch.int32 and bits.shape[0] == M and bits.shape[1] * 32 >= F
        s.bits, s.ldbits = bits.data_ptr(), bits.stride(0)
    s.p, s.dgu, s.lddgu, s.M, s.F = float(p), dgu.data_ptr(), dgu.stride(0), M, F
    d = LoraSwigluBwdGradsDesc()
    d.sw = s
    d.tg, d.tu, d.ldtg = tg.data_ptr(), tu.data_ptr(), tg.stride(0)
    d.dA_down, d.dB_gate, d.dB_up = dA_down.data_ptr(), dB_gate.data_ptr(), dB_up.data_ptr()
    d.alpha_b, d.ws, d.ws_floats = float(alpha_b), ws.data_ptr(), ws.numel()
    check(lib().slx_lora_swiglu_bwd_grads(ctypes.byref(d), stream_ptr()), "slx_lora_swiglu_bwd_grads")


class SwigluLoraDownDesc(ctypes.Structure):
    _fields_ = [("gu", c_vp), ("ldgu", c_i64), ("act", c_vp), ("ldact", c_i64), ("A", c_vp), ("lda", c_i64),
                ("bits", c_vp), ("ldbits", c_i64), ("p", c_float), ("t", c_vp), ("ldt", c_i64), ("ws", c_vp),
                ("ws_floats", c_i64), ("M", c_i64), ("F", c_int), ("seed", ctypes.c_uint64), ("gen_bits", c_int)]


register("slx_swiglu_lora_down", [ctypes.POINTER(SwigluLoraDownDesc), c_vp])
register("slx_swiglu_lora_down_ws_floats", [c_i64, c_int], restype=c_i64)


def swiglu_lora_down(gu, act, A, t, bits, p, ws, seed=None):
    """slx_swiglu_lora_down: act = bf16(silu(g) u) from gu bf16 [M, 2F], t = drop(act) A^T (bf16 [M, 32] view).
    A bf16 [>= 32, F] rows (lora_A), bits int32 [M, >= F/32] keep bits (p > 0), ws f32 scratch of
    slx_swiglu_lora_down_ws_floats(M, F) floats (engine-owned, reused). seed given (p > 0): the kernel generates the keep
    bits (the site seed's drop_keep hash, mask index m * F + n) and writes them to bits instead of reading them."""
    M, F = act.shape
    for x in (gu, act, A, t):
        assert x.dtype == torch.bfloat16 and x.is_cuda and x.stride(1) == 1
    assert gu.shape[0] == M and gu.shape[1] >= 2 * F and A.shape[1] == F and A.shape[0] >= 32 and t.shape == (M, 32)
    need = lib().slx_swiglu_lora_down_ws_floats(M, F)
    assert ws.dtype == torch.float32 and ws.numel() >= need
    d = SwigluLoraDownDesc()
    d.gu, d.ldgu, d.act, d.ldact = gu.data_ptr(), gu.stride(0), act.data_ptr(), act.stride(0)
    d.A, d.lda = A.data_ptr(), A.stride(0)
    if p > 0:
        assert bits is not None and bits.dtype == torch.int32 and bits.shape[0] == M and bits.shape[1] * 32 >= F
        d.bits, d.ldbits = bits.data_ptr(), bits.stride(0)
    d.p, d.t, d.ldt, d.ws, d.ws_floats, d.M, d.F = float(p), t.data_ptr(), t.stride(0), ws.data_ptr(), ws.numel(), M, F
    if seed is not None:
        d.seed, d.gen_bits = int(seed) & ((1 << 64) - 1), 1
    check(lib().slx_swiglu_lora_down(ctypes.byref(d), stream_ptr()), "slx_swiglu_lora_down")


def lora_grad(jobs, M):
    """The LoRA parameter gradients of one layer group in one launch (slx_lora_grad). jobs: dicts with
    x (bf16 [M, n] view, n % 128 == 0), t (bf16 [M, >= 32 * nsites] view), outs (list of f32 gradients, 1..3 sites),
    out_nr (True: outs are [n, 32] B gradients; False: [32, n] A gradients), alpha, and for A gradients with dropout
    p > 0 the keep bits (list, one int32 [M, >= n/32] per site)."""
    assert 1 <= len(jobs) <= 12
    arr = (LoraGradJob * len(jobs))()
    for i, jb in enumerate(jobs):
        x, t, outs = jb["x"], jb["t"], jb["outs"]
        n = x.shape[1]
        assert x.dtype == torch.bfloat16 and x.shape[0] == M and x.stride(1) == 1 and n % 128 == 0
        assert t.dtype == torch.bfloat16 and t.shape[0] == M and t.stride(1) == 1 and t.shape[1] >= 32 * len(outs)
        d = arr[i]
        d.x, d.ldx, d.n = x.data_ptr(), x.stride(0), n
        d.t, d.ldt, d.t_bf16, d.nsites = t.data_ptr(), t.stride(0), 1, len(outs)
        for j, o in enumerate(outs):
            assert o.dtype == torch.float32 and o.is_contiguous()
            assert o.shape == ((n, 32) if jb["out_nr"] else (32, n)), (o.shape, n)
            d.out[j] = o.data_ptr()
        p = float(jb.get("p", 0.0))
        if p > 0:
            for j, b in enumerate(jb["bits"]):
                assert b.dtype == torch.int32 and b.shape[0] == M and b.shape[1] * 32 >= n
                d.bits[j] = b.data_ptr()
            d.ldbits = jb["bits"][0].stride(0)
        d.p, d.alpha, d.out_nr = p, float(jb.get("alpha", 1.0)), int(bool(jb["out_nr"]))
    check(lib().slx_lora_grad(arr, len(jobs), M, stream_ptr()), "slx_lora_grad")


def _mm_dims(A, B, C, ta, tb):
    if ta:
        Kd, M = A.shape
    else:
        M, Kd = A.shape
    N = B.shape[0] if tb else B.shape[1]
    layout = {(False, True): GEMM_NT, (False, False): GEMM_NN, (True, False): GEMM_TN, (True, True): GEMM_TT}[(ta, tb)]
    assert C.shape[0] >= M and C.shape[1] >= N, (C.shape, M, N)
    return M, N, Kd, layout


LT_WS_BYTES = 32 << 20
_lt_ws: dict = {}


def mm_lt(A, B, D, *, C=None, alpha=1.0, beta=0.0, ws=None):
    """D = alpha * A @ B^T + beta * C through hipBLASLt (slx_gemm_lt): A [M,K] and B [N,K] bf16 row-major views with
    unit inner stride, C / D [M,N] both f32 or both bf16 (C may be D). The plain GEMMs it runs faster than
    slx_gemm_bf16 (csrc/blaslt.hip); ws: a >= LT_WS_BYTES uint8 device buffer (one per device by default)."""
    _require_cuda(A, B, D)
    M, Kd = A.shape
    N = B.shape[0]
    if A.dtype != torch.bfloat16 or B.dtype != torch.bfloat16 or B.shape[1] != Kd:
        raise RuntimeError("slx_gemm_lt: bf16 A [M,K] and B [N,K]")
    if D.dtype not in (torch.float32, torch.bfloat16) or D.shape[0] < M or D.shape[1] < N:
        raise RuntimeError("slx_gemm_lt: D [M,N] f32 or bf16")
    if beta != 0.0 and (C is None or C.dtype != D.dtype):
        raise RuntimeError("slx_gemm_lt: beta != 0 needs C of D's dtype")
    if ws is None:
        ws = _lt_ws.get(D.device)
        if ws is None:
            ws = _lt_ws[D.device] = torch.empty(LT_WS_BYTES, dtype=torch.uint8, device=D.device)
    d = GemmLtDesc()
    d.M, d.N, d.K = int(M), int(N), int(Kd)
    d.A, d.lda, d.B, d.ldb = A.data_ptr(), int(A.stride(0)), B.data_ptr(), int(B.stride(0))
    d.C, d.ldc = (C.data_ptr(), int(C.stride(0))) if C is not None else (0, 0)
    d.D, d.ldd = D.data_ptr(), int(D.stride(0))
    d.alpha, d.beta, d.out_f32 = float(alpha), float(beta), int(D.dtype == torch.float32)
    d.ws, d.ws_bytes = ws.data_ptr(), int(ws.numel())
    check(lib().slx_gemm_lt(ctypes.byref(d), stream_ptr()), "slx_gemm_lt")
    return D


def mm_pair(g1, g2, *, ta=True, tb=False, alpha=1.0, ksplit_max=0, variant=None):
    """Two accumulating f32 GEMMs C_i += op(A_i) @ op(B_i) (g_i = (A_i, B_i, C_i), same layout and K) in one
    launch (slx_gemm_bf16_pair): the InternViT weight-gradient pairs."""
    ds = []
    for A, B, C in (g1, g2):
        M, N, Kd, layout = _mm_dims(A, B, C, ta, tb)
        ds.append(_gemm_desc(A, B, C, M, N, Kd, layout, A.stride(0), B.stride(0), C.stride(0), alpha=alpha,
                             accumulate=True, ksplit_max=ksplit_max, variant=variant))
    check(lib().slx_gemm_bf16_pair(ctypes.byref(ds[0]), ctypes.byref(ds[1]), stream_ptr()), "slx_gemm_bf16_pair")


def mm(A, B, C, *, ta=False, tb=True, **kw):
    """C = op(A) @ op(B). A is stored [M,K] (ta=False) or [K,M] (ta=True); B is stored [K,N] (tb=False)
    or [N,K] (tb=True). All operands are 2-D views with unit inner stride (column slices allowed)."""
    if ta:
        Kd, M = A.shape
    else:
        M, Kd = A.shape
    N = B.shape[0] if tb else B.shape[1]
    layout = {(False, True): GEMM_NT, (False, False): GEMM_NN, (True, False): GEMM_TN, (True, True): GEMM_TT}[(ta, tb)]
    assert C.shape[0] >= M and C.shape[1] >= N, (C.shape, M, N)
    gemm(A, B, C, M, N, Kd, layout, A.stride(0), B.stride(0), C.stride(0), **kw)
    return C
