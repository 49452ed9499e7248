"""KV-cached greedy decode (agent inference, BASELINE configs[4]) vs the CPU fp32 oracle, which restates
LLM.greedy_sample literally (whole sequence re-run per token, llm.py:178-250) and the final driving forward
(driving.py:156-165).

The HIP path runs bf16 weights with LoRA merged, so its logits differ from the fp32 oracle's by bf16
rounding. Token check (teacher forced on the HIP tokens, one oracle pass gives every step's logits): the
chosen token's oracle logit is within 3e-2 x std(logits) of the oracle maximum at every step, and wherever
the oracle's top-2 margin exceeds 0.2 x std the tokens are identical. Driving predictions from the oracle's
final forward over the same prompt + tokens + queries: every per-point head output (the increment the
cumsum adds) within 0.015 m and the cumulated waypoints within 0.1 m of the fp32 oracle (observed 0.074 m: with a
random-init head the 20 increments carry near-identical bf16 errors, so the cumsum's error grows linearly), and
within SURVEY §8d's bf16 gate of 5e-2 m of the oracle evaluated on the decoder's own bf16 operands (every weight
rounded as the engine holds it, the LoRA-merged Qwen2 projections; observed <= 0.018 m). EOS stopping, the
graph-replayed and the eager step, and the single-forward mode are checked for exact agreement.
"""
import pytest
import torch

from golden_util import load_case
from oracle import vla_oracle as O

pytestmark = pytest.mark.gpu


def _setup(dev, case="leftpad"):
    from simlingo_amd.engine import VLAEngine
    cfg, P, ex, _ = load_case(case)
    eng = VLAEngine(cfg, dev, P)
    return cfg, P, ex, eng


def _oracle_teacher(P, cfg, ex, toks_all):
    """Per sample: oracle logits for every decode step given the HIP tokens, and the oracle's drive preds."""
    pix = ex.driving_input.camera_images
    Bn, _, NP, C, H, W = pix.shape
    vit = O.extract_feature(P, cfg, pix.reshape(Bn * NP, C, H, W))
    lang, valid = O.language_inputs(P, cfg, ex, vit, inference=True)
    queries = torch.cat([P["drv.query_route"], P["drv.query_speed"]], 0)
    out = []
    for b, toks in enumerate(toks_all):
        emb = lang[b][valid[b]]
        x = torch.cat([emb, P["llm.embed"][torch.tensor(toks, dtype=torch.long)]], 0)
        _, logits = O.llm_forward(P, cfg, x[None], torch.ones(1, x.shape[0], dtype=torch.bool))
        S0 = emb.shape[0]
        step_logits = logits[0, S0 - 1:S0 - 1 + len(toks)]
        r, s = O.drive_after(P, cfg, x, queries)
        out.append((step_logits, r[0], s[0]))
    return out


def test_greedy_decode_vs_oracle(dev):
    cfg, P, ex, eng = _setup(dev)
    _check_greedy(cfg, P, ex, eng, n_new=12, max_len=512, tag="tiny")


def test_greedy_decode_full_width_vs_oracle(dev):
    """VERDICT r5 missing #4: the agent's greedy loop at the REAL InternVL2-1B widths (InternViT D 1024 / T 1025, Qwen2
    d 896, GQA 14/2, FFN 4864, the V = 151655 argmax; 2 + 2 layers so the oracle's literal re-run per token stays
    cheap), a ~576-token prompt (512 image tokens + 64 text, sample 1 left-padded by 5) and 30 generated tokens,
    teacher-forced against the oracle's logits with the same gates as the tiny case
    (/root/reference/simlingo_training/models/language_model/llm.py:178-250, team_code/agent_simlingo.py:797)."""
    from simlingo_amd.config import full_config
    from simlingo_amd.engine import VLAEngine
    from simlingo_amd.params import init_params
    from simlingo_amd.synthetic import make_batch
    torch.set_num_threads(16)
    cfg = full_config(vit_layers=2, llm_layers=2, lora_dropout=0.0)
    P = init_params(cfg, seed=7, lora_b_std=0.02)
    ex = make_batch(cfg, B=2, s_text=64, n_loss=1, seed=7, pad=[0, 5])
    eng = VLAEngine(cfg, dev, P)
    _check_greedy(cfg, P, ex, eng, n_new=30, max_len=1024, tag="full-width")


def _check_greedy(cfg, P, ex, eng, n_new, max_len, tag):
    from simlingo_amd.decode import GreedyDecoder, infer_example
    dec = GreedyDecoder(eng, max_len=max_len, max_new_tokens=n_new, eos_id=-1)
    sp, rp, toks = infer_example(eng, dec, ex)
    assert all(len(t) == n_new for t in toks)
    ref = _oracle_teacher(P, cfg, ex, toks)
    worst_gap, worst_d, worst_inc = 0.0, 0.0, 0.0
    for b, (lg, r_ref, s_ref) in enumerate(ref):
        std = lg.std(dim=-1)
        top2 = lg.topk(2, dim=-1).values
        for i, t in enumerate(toks[b]):
            gap = (top2[i, 0] - lg[i, t]).item()
            worst_gap = max(worst_gap, gap / std[i].item())
            assert gap <= 3e-2 * std[i].item(), (b, i, t, gap, std[i].item())
            if (top2[i, 0] - top2[i, 1]).item() > 0.2 * std[i].item():
                assert t == int(lg[i].argmax()), (b, i)
        for got, want in ((rp[b].cpu(), r_ref), (sp[b].cpu(), s_ref)):
            diff = (got - want).abs()
            inc = (torch.diff(got, dim=0, prepend=torch.zeros(1, got.shape[1]))
                   - torch.diff(want, dim=0, prepend=torch.zeros(1, want.shape[1]))).abs()
            worst_d, worst_inc = max(worst_d, diff.max().item()), max(worst_inc, inc.max().item())
            assert diff.max().item() <= 0.1 and inc.max().item() <= 0.015, (b, diff.max().item(), inc.max().item())
    print(f"[decode {tag}] worst chosen-token gap {worst_gap:.4g} std, cumulated max |diff| {worst_d:.4g} m, "
          f"per-point increment {worst_inc:.4g} m")
    # SURVEY §8d's bf16 gate (5e-2 m) against the oracle evaluated with the decoder's own bf16 GEMM operands: every
    # engine weight rounded to bf16 as the engine holds it, the Qwen2 projections replaced by the decoder's merged
    # bf16 W + s B A (LoRA B zeroed in the oracle so the merged term is not added twice); what remains is the bf16
    # rounding of activations
    Pq = {k: (v.detach().float().cpu().bfloat16().float() if k in eng.W else v) for k, v in P.items()}
    groups = (("qkv_w", ("q", "k", "v")), ("o_w", ("o",)), ("gate_up_w", ("gate", "up")), ("down_w", ("down",)))
    for i, layer in enumerate(dec.Wm):
        for name, sites in groups:
            Pq[f"llm.{i}.{name}"] = layer[name].float().cpu()
            if cfg.lora:
                for site in sites:
                    Pq[f"llm.{i}.lora.{site}.b"] = torch.zeros_like(P[f"llm.{i}.lora.{site}.b"])
    refq = _oracle_teacher(Pq, cfg, ex, toks)
    for b, (_, r_q, s_q) in enumerate(refq):
        for got, want in ((rp[b].cpu(), r_q), (sp[b].cpu(), s_q)):
            dq = (got - want).abs().max().item()
            print(f"[decode {tag} b={b}] vs the oracle on the decoder's bf16 operands: cumulated max |diff| {dq:.4g} m")
            assert dq <= 5e-2, (b, dq)
    # the oracle's own free-running greedy agrees up to its first near-tie decision
    _, _, toks_o = O.infer(P, cfg, ex, n_new, eos=-1)
    for b in range(len(toks)):
        lg = ref[b][0]
        for i in range(n_new):
            if toks[b][i] != toks_o[b][i]:
                top2 = lg[i].topk(2).values
                assert (top2[0] - top2[1]).item() <= 0.2 * lg[i].std().item(), (b, i)
                break


def test_eos_stop_and_graph_equivalence(dev):
    from simlingo_amd.decode import GreedyDecoder, infer_example
    cfg, P, ex, eng = _setup(dev, "nopad")
    n_new = 10
    dec_g = GreedyDecoder(eng, max_len=512, max_new_tokens=n_new, eos_id=-1, use_graph=True, check_every=3)
    dec_e = GreedyDecoder(eng, max_len=512, max_new_tokens=n_new, eos_id=-1, use_graph=False)
    sp_g, rp_g, toks_g = infer_example(eng, dec_g, ex)
    sp_e, rp_e, toks_e = infer_example(eng, dec_e, ex)
    assert toks_g == toks_e
    assert torch.equal(sp_g, sp_e) and torch.equal(rp_g, rp_e)
    # EOS = the token generated at step 4 of sample 0: decoding stops right after its first occurrence
    eos = toks_g[0][4]
    first = toks_g[0].index(eos)
    dec_s = GreedyDecoder(eng, max_len=512, max_new_tokens=n_new, eos_id=eos)
    _, _, toks_s = infer_example(eng, dec_s, ex)
    assert toks_s[0] == toks_g[0][:first + 1]
    for b in range(1, len(toks_g)):
        stop = toks_g[b].index(eos) + 1 if eos in toks_g[b] else n_new
        assert toks_s[b] == toks_g[b][:stop]


def test_driving_model_forward_surface(dev):
    from simlingo_amd.driving import DrivingModel
    cfg, P, ex, _ = load_case("nopad")
    m = DrivingModel(language_model={"variant": "tiny", "lora_dropout": 0.0}, vision_model={"variant": "tiny"},
                     init_params=P, max_new_tokens=5)
    m.build_engine(dev)
    m.eval()
    sp, rp, lang = m(ex)
    B = ex.driving_input.camera_images.shape[0]
    assert sp.shape == (B, cfg.n_speed, cfg.speed_dims) and rp.shape == (B, cfg.n_route, 2)
    assert len(lang) == B and all(len(t) <= 5 for t in m.sampled_tokens)
    m.predict_language = False
    sp1, rp1, lang1 = m(ex)
    assert lang1 == [] and sp1.shape == sp.shape


def _check_rotated_k(krow, want, orig):
    """The k row written back is rotate_half(k) rounded to bf16: equal to the torch rotation except where the kernel's
    fused multiply-add (x0 c - x1 s in one rounding) lands on the other side of a bf16 rounding boundary, i.e. at most
    one bf16 ulp on a couple of elements (seen on cancelling terms: 2.1839e-4 vs 2.1744e-4)."""
    bad = (krow != want).nonzero().flatten()
    assert bad.numel() <= 2, bad.tolist()
    assert ((krow - want).abs() <= want.abs().clamp_min(krow.abs()) * 2.0 ** -7).all(), \
        (bad.tolist(), krow[bad].tolist(), want[bad].tolist())
    if not torch.equal(want, orig):
        assert not torch.equal(krow, orig)  # rotated, not left as written by the q|k|v GEMV


@pytest.mark.parametrize("pos", [0, 31, 300, 1000])
def test_dec_attn_forms_vs_torch(dev, pos):
    """slx_dec_attn at the agent geometry (14 q / 2 kv heads): the single-workgroup MFMA form (caches <= 1024 rows) and
    the split form with its last-arriver merge, each vs a torch fp32 softmax attention of the same bf16 rows (q and
    row pos's k rotated with the same tables); the k row written back must be the rotated one."""
    import ctypes
    from simlingo_amd import decode  # noqa: F401
    from simlingo_amd import kernels as K
    K.register("slx_dec_attn_force_split", [ctypes.c_int])
    Hq, Hkv, lmax = 14, 2, 1024
    ld = (Hq + 2 * Hkv) * 64
    gen = torch.Generator(device=dev).manual_seed(pos)
    cache0 = torch.randn(lmax, ld, device=dev, generator=gen).bfloat16()
    cos, sin = K.rope_tables(lmax, 1e6, dev)
    st = torch.tensor([pos, 0, 0, 100, -1, 0, 0, 0], dtype=torch.int32, device=dev)

    def rope(x):  # [n, 64] f32 -> rotate_half with row `pos` of the tables, rounded to bf16
        c, s_ = cos[pos], sin[pos]
        x0, x1 = x[:, :32], x[:, 32:]
        return torch.cat([x0 * c - x1 * s_, x1 * c + x0 * s_], 1).bfloat16().float()

    c0 = cache0.float()
    ref = torch.empty(Hq, 64, device=dev)
    G = Hq // Hkv
    for g in range(Hkv):
        k = c0[:pos + 1, Hq * 64 + 64 * g: Hq * 64 + 64 * (g + 1)].clone()
        k[pos] = rope(k[pos:pos + 1])[0]
        v = c0[:pos + 1, (Hq + Hkv) * 64 + 64 * g: (Hq + Hkv) * 64 + 64 * (g + 1)]
        q = rope(c0[pos, 64 * G * g: 64 * G * (g + 1)].reshape(G, 64))
        ref[G * g: G * (g + 1)] = torch.softmax(q @ k.t() * 0.125, -1) @ v
    lib = K.lib()
    for split in (0, 1):
        cache = cache0.clone()
        ws = torch.zeros(lib.slx_dec_attn_ws_floats(Hq, Hkv, lmax), device=dev)
        out = torch.empty(Hq * 64, dtype=torch.bfloat16, device=dev)
        lib.slx_dec_attn_force_split(split)
        try:
            K.check(lib.slx_dec_attn(K.P(cache), ld, Hq, Hkv, K.P(cos), K.P(sin), lmax, K.P(ws), K.P(out), K.P(st),
                                     K.stream_ptr()), "slx_dec_attn")
            torch.cuda.synchronize()
        finally:
            lib.slx_dec_attn_force_split(0)
        err = (out.float().reshape(Hq, 64) - ref).abs().max().item()
        assert err <= 2e-2 * ref.abs().max().item() + 1e-3, (split, err)
        for g in range(Hkv):
            krow = cache[pos, Hq * 64 + 64 * g: Hq * 64 + 64 * (g + 1)].float()
            orig = c0[pos, Hq * 64 + 64 * g: Hq * 64 + 64 * (g + 1)]
            _check_rotated_k(krow, rope(orig[None])[0], orig)


@pytest.mark.parametrize("pos", [0, 31, 32, 300, 1000, 1023])
def test_dec_attn_o_split_vs_torch(dev, pos):
    """slx_dec_attn_o_split (the attention split over 8 workgroups per kv head, partials merged in the O GEMV's
    prologue): the merged attention output vs a torch fp32 softmax attention of the same bf16 rows, the residual row vs
    X + W_o . (that output rounded to bf16) and vs the single-workgroup MFMA form followed by the O GEMV, and the k row
    written back rotated."""
    import ctypes
    from simlingo_amd import decode as D
    from simlingo_amd import kernels as K
    Hq, Hkv, lmax, d = 14, 2, 1024, 896
    ld = (Hq + 2 * Hkv) * 64
    gen = torch.Generator(device=dev).manual_seed(pos + 11)
    cache0 = torch.randn(lmax, ld, device=dev, generator=gen).bfloat16()
    Wo = (torch.randn(d, Hq * 64, device=dev, generator=gen) * 0.03).bfloat16()
    X0 = torch.randn(d, device=dev, generator=gen)
    cos, sin = K.rope_tables(lmax, 1e6, dev)
    st = torch.tensor([pos, 0, 0, 100, -1, 0, 0, 0], dtype=torch.int32, device=dev)

    def rope(x):
        c, s_ = cos[pos], sin[pos]
        x0, x1 = x[:, :32], x[:, 32:]
        return torch.cat([x0 * c - x1 * s_, x1 * c + x0 * s_], 1).bfloat16().float()

    c0 = cache0.float()
    ref = torch.empty(Hq, 64, device=dev)
    G = Hq // Hkv
    for g in range(Hkv):
        k = c0[:pos + 1, Hq * 64 + 64 * g: Hq * 64 + 64 * (g + 1)].clone()
        k[pos] = rope(k[pos:pos + 1])[0]
        v = c0[:pos + 1, (Hq + Hkv) * 64 + 64 * g: (Hq + Hkv) * 64 + 64 * (g + 1)]
        q = rope(c0[pos, 64 * G * g: 64 * G * (g + 1)].reshape(G, 64))
        ref[G * g: G * (g + 1)] = torch.softmax(q @ k.t() * 0.125, -1) @ v
    lib = K.lib()
    ws = torch.zeros(lib.slx_dec_attn_ws_floats(Hq, Hkv, lmax), device=dev)
    for rep in range(2):  # no state carried between calls (no counters)
        cache, X, out = cache0.clone(), X0.clone(), torch.empty(Hq * 64, dtype=torch.bfloat16, device=dev)
        K.check(lib.slx_dec_attn_o_split(K.P(cache), ld, Hq, Hkv, K.P(cos), K.P(sin), lmax, K.P(ws), K.P(out),
                                         K.P(st), K.P(Wo), Wo.stride(0), d, Hq * 64, K.P(X), K.stream_ptr()),
                "slx_dec_attn_o_split")
        torch.cuda.synchronize()
        err = (out.float().reshape(Hq, 64) - ref).abs().max().item()
        assert err <= 2e-2 * ref.abs().max().item() + 1e-3, (rep, err)
        Xref = X0 + Wo.float() @ out.float()
        assert (X - Xref).abs().max().item() <= 1e-4 * Xref.abs().max().item() + 1e-5
        for g in range(Hkv):
            krow = cache[pos, Hq * 64 + 64 * g: Hq * 64 + 64 * (g + 1)].float()
            orig = c0[pos, Hq * 64 + 64 * g: Hq * 64 + 64 * (g + 1)]
            want = rope(orig[None])[0]
            _check_rotated_k(krow, want, orig)
    # against the single-workgroup form + the O GEMV (different summation order: bf16-level agreement)
    c1, X1, o1 = cache0.clone(), X0.clone(), torch.empty(Hq * 64, dtype=torch.bfloat16, device=dev)
    K.check(lib.slx_dec_attn(K.P(c1), ld, Hq, Hkv, K.P(cos), K.P(sin), lmax, K.P(ws), K.P(o1), K.P(st),
                             K.stream_ptr()), "slx_dec_attn")
    desc = D._gemv_desc(D.DEC_RESID, Wo, d, Hq * 64, xb=o1, resid=X1, state=st)
    K.check(lib.slx_dec_gemv(ctypes.byref(desc), K.stream_ptr()), "slx_dec_gemv")
    torch.cuda.synchronize()
    assert torch.equal(c1, cache)
    assert (o1.float() - out.float()).abs().max().item() <= 2e-2 * ref.abs().max().item() + 1e-3
    assert (X1 - X).abs().max().item() <= 2e-2 * (X1 - X0).abs().max().item() + 1e-4


def test_greedy_decode_split_o(dev, monkeypatch):
    """The graph-captured decode with SLX_DEC_SPLIT_O (split attention merged by the O GEMV) against the default path:
    the same tokens up to a near-tie of the oracle's teacher-forced logits, and every token within the greedy gate of
    test_greedy_decode_vs_oracle."""
    from simlingo_amd import decode as D
    cfg, P, ex, eng = _setup(dev)
    n_new = 12
    toks = []
    for split in (False, True):
        monkeypatch.setattr(D, "SPLIT_O", split)
        dec = D.GreedyDecoder(eng, max_len=512, max_new_tokens=n_new, eos_id=-1)
        toks.append(D.infer_example(eng, dec, ex)[2])
    ref = _oracle_teacher(P, cfg, ex, toks[1])
    for b, (lg, _, _) in enumerate(ref):
        std = lg.std(dim=-1)
        top2 = lg.topk(2, dim=-1).values
        for i, t in enumerate(toks[1][b]):
            assert (top2[i, 0] - lg[i, t]).item() <= 3e-2 * std[i].item(), (b, i)
            if toks[0][b][i] != t:  # the two paths may part only at a near-tie
                assert (top2[i, 0] - top2[i, 1]).item() <= 0.2 * std[i].item(), (b, i)
                break
