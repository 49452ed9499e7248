"""Checkpoint compatibility on the CPU: the reference state-dict layout, both directions.

Pins: tests/golden/ckpt_keys.json and vla_tiny_refsd.safetensors were produced by oracle/gen_golden_ckpt.py from the
reference's own adaptor modules + transformers' Qwen2ForCausalLM with the llm.py alias and peft naming (the InternViT
remote code is restated there). The ZeRO-2 directory reader follows deepspeed 0.16.2's zero_to_fp32 file format
(deepspeed is absent: parity unpinned beyond the synthetic directory built here the way DeepSpeed lays it out).
"""
import json
import os
import sys

import pytest
import torch

from golden_util import GOLDEN, load_case
from simlingo_amd.checkpoint import ALIASES, consolidate_zero, from_reference, load_checkpoint, to_reference
from simlingo_amd.config import full_config
from simlingo_amd.params import param_specs

KEYS = json.load(open(os.path.join(GOLDEN, "ckpt_keys.json")))


def _empty(cfg):
    return {s.name: torch.zeros(s.shape) for s in param_specs(cfg)}


def test_key_layout_matches_reference_tree():
    cfg, P, _, _ = load_case("nopad")
    sd = to_reference(P, cfg)
    assert {k: list(v.shape) for k, v in sd.items()} == KEYS["tiny"]
    full = full_config()
    sdf = to_reference(_empty(full), full)
    assert {k: list(v.shape) for k, v in sdf.items()} == KEYS["full"]
    assert len(KEYS["full"]) == 992  # 24 ViT layers x 14 + 4 + 6 mlp1 + 24 x 26 LLM + 3 + 3 aliases + 16 heads/wp


def test_reference_fixture_loads_to_the_golden_parameters():
    from safetensors.torch import load_file
    cfg, P, _, _ = load_case("nopad")
    sd = load_file(os.path.join(GOLDEN, "vla_tiny_refsd.safetensors"))  # aliases stripped by safetensors
    back = from_reference(sd, cfg)
    assert set(back) == set(P)
    for k in P:
        assert torch.equal(back[k], P[k]), k


def test_round_trip_and_wrappers():
    cfg, P, _, _ = load_case("leftpad")
    sd = to_reference(P, cfg)
    for wrapped in ({"state_dict": sd}, {"module": {"module." + k: v for k, v in sd.items()}},
                    {"_forward_module." + k: v for k, v in sd.items()}):
        back = from_reference(wrapped, cfg)
        assert all(torch.equal(back[k], P[k]) for k in P)


def test_strict_errors():
    cfg, P, _, _ = load_case("nopad")
    sd = dict(to_reference(P, cfg))
    bad = dict(sd)
    del bad["adaptors.driving.query_embeds_wps"]
    with pytest.raises(KeyError, match="missing"):
        from_reference(bad, cfg)
    bad = dict(sd, **{"vision_model.extra.weight": torch.zeros(1)})
    with pytest.raises(KeyError, match="unexpected"):
        from_reference(bad, cfg)
    bad = dict(sd)
    k = "language_model.model.base_model.model.model.layers.0.self_attn.q_proj.base_layer.weight"
    bad[k] = torch.zeros(3, 3)
    with pytest.raises(ValueError, match="shape"):
        from_reference(bad, cfg)
    bad = dict(sd)
    a = next(iter(ALIASES))
    bad[a] = bad[a] + 1
    with pytest.raises(ValueError, match="alias"):
        from_reference(bad, cfg)


def test_fusion_layout():
    """q/k/v and gate/up are concatenated along the output rows in that order (the engine's fused operands)."""
    cfg, P, _, _ = load_case("nopad")
    sd = to_reference(P, cfg)
    base = "language_model.model.base_model.model.model.layers.1."
    qkv = torch.cat([sd[base + f"self_attn.{s}_proj.base_layer.weight"] for s in "qkv"])
    assert torch.equal(qkv, P["llm.1.qkv_w"])
    gu = torch.cat([sd[base + "mlp.gate_proj.base_layer.weight"], sd[base + "mlp.up_proj.base_layer.weight"]])
    assert torch.equal(gu, P["llm.1.gate_up_w"])
    pw = sd["vision_model.image_encoder.model.vision_model.embeddings.patch_embedding.weight"]
    assert torch.equal(pw.reshape(pw.shape[0], -1), P["vit.patch.w"])


def _fake_classes():
    """Classes pickled under the module paths DeepSpeed 0.16 / Lightning use (the packages are absent here): registered
    in sys.modules only while the fixture is written, so loading must go through inert stand-ins."""
    import enum
    import types
    made = []

    def mod(name):
        parts = name.split(".")
        for i in range(1, len(parts) + 1):
            n = ".".join(parts[:i])
            if n not in sys.modules:
                sys.modules[n] = types.ModuleType(n)
                made.append(n)
        return sys.modules[name]

    m = mod("deepspeed.runtime.fp16.loss_scaler")

    class LossScaler:
        def __init__(self, scale):
            self.cur_scale, self.cur_iter = scale, 0
    LossScaler.__module__, m.LossScaler = m.__name__, LossScaler
    m = mod("deepspeed.runtime.zero.config")

    class ZeroStageEnum(int, enum.Enum):
        disabled, optimizer_states, gradients = 0, 1, 2
    ZeroStageEnum.__module__, m.ZeroStageEnum = m.__name__, ZeroStageEnum
    m = mod("deepspeed.utils.tensor_fragment")

    class fragment_address:  # noqa: N801 (DeepSpeed's name)
        def __init__(self, numel, start):
            self.numel, self.start = numel, start
    fragment_address.__module__, m.fragment_address = m.__name__, fragment_address
    m = mod("lightning.fabric.utilities.data")

    class AttributeDict(dict):
        pass
    AttributeDict.__module__, m.AttributeDict = m.__name__, AttributeDict

    for c in (LossScaler, ZeroStageEnum, fragment_address, AttributeDict):
        c.__qualname__ = c.__name__  # picklable by module path + name, like the real classes

    def cleanup():
        for n in made:
            sys.modules.pop(n, None)
    return LossScaler, ZeroStageEnum, fragment_address, AttributeDict, cleanup


def _write_zero2_dir(root, sd, world, group_split, ds_objects=False):
    """A ZeRO stage-2 checkpoint as DeepSpeed 0.16 lays it out: <root>/latest -> tag; the tag dir holds
    mp_rank_00_model_states.pt (module = non-trainable state, param_shapes = [OrderedDict] per group) and one
    zero_pp_rank_{r}_mp_rank_00_optim_states.pt per rank with that rank's slice of every flat fp32 group."""
    from collections import OrderedDict
    tag = os.path.join(root, "global_step7")
    os.makedirs(tag)
    open(os.path.join(root, "latest"), "w").write("global_step7")
    names = [k for k in sd if k not in ALIASES]
    trainable = [k for k in names if not k.startswith("language_model.model.base_model.model.model.embed_tokens")
                 and "base_layer" not in k and "lm_head" not in k and "norm.weight" not in k
                 and "layernorm" not in k]
    frozen = [k for k in names if k not in trainable]
    groups = [trainable[:group_split], trainable[group_split:]]
    shapes = [OrderedDict((k, torch.Size(sd[k].shape)) for k in g) for g in groups]
    LossScaler = ZeroStageEnum = fragment_address = AttributeDict = None
    cleanup = lambda: None  # noqa: E731
    if ds_objects:
        LossScaler, ZeroStageEnum, fragment_address, AttributeDict, cleanup = _fake_classes()
    ms = {"module": {k: sd[k].clone() for k in frozen}, "param_shapes": shapes}
    if ds_objects:  # what DeepSpeed + Lightning add next to the tensors
        ms.update(ds_config={"zero_optimization": {"stage": 2}, "fp16": {"loss_scale": 32}}, ds_version="0.16.2",
                  hyper_parameters=AttributeDict(lr=3e-5), global_steps=7)
    torch.save(ms, os.path.join(tag, "mp_rank_00_model_states.pt"))
    flats = []
    for g in groups:
        flat = torch.cat([sd[k].reshape(-1).float() for k in g])
        pad = (-flat.numel()) % (2 * world)  # DeepSpeed aligns each flat group to 2 * world elements
        flats.append(torch.cat([flat, torch.zeros(pad)]))
    for r in range(world):
        parts = [f.chunk(world)[r].clone() for f in flats]
        osd = {"single_partition_of_fp32_groups": parts}
        if ds_objects:
            osd.update(loss_scaler=LossScaler(32.0), dynamic_loss_scale=False, zero_stage=ZeroStageEnum.gradients,
                       param_slice_mappings=[OrderedDict((k, fragment_address(sd[k].numel(), 0)) for k in g[:3])
                                             for g in groups], ds_version="0.16.2")
        torch.save({"optimizer_state_dict": osd, "ds_config": {"train_micro_batch_size_per_gpu": 8}},
                   os.path.join(tag, f"zero_pp_rank_{r}_mp_rank_00_optim_states.pt"))
    cleanup()


@pytest.mark.parametrize("world,ds_objects", [(1, False), (2, True), (8, False), (8, True)])
def test_zero2_directory_consolidation(tmp_path, world, ds_objects):
    """ds_objects: the optimizer / model-state files also pickle DeepSpeed's LossScaler, ZeroStageEnum,
    fragment_address records and Lightning hparams: loaded weights-only through inert stand-ins."""
    cfg, P, _, _ = load_case("nopad")
    sd = to_reference(P, cfg)
    _write_zero2_dir(str(tmp_path), sd, world, group_split=5, ds_objects=ds_objects)
    assert not any(k.startswith("deepspeed") for k in sys.modules)
    got = consolidate_zero(str(tmp_path))
    back = from_reference(got, cfg)
    assert all(torch.equal(back[k], P[k]) for k in P)
    assert set(load_checkpoint(str(tmp_path))) == set(got)


def test_driving_model_state_dict_surface(tmp_path):
    """DrivingModel.state_dict()/load_state_dict() speak the reference layout (no GPU needed before the engine is
    built): load the reference fixture, read it back, save/load a flat file like agent_simlingo.py:223."""
    from safetensors.torch import load_file
    from simlingo_amd.driving import DrivingModel
    cfg, P, _, _ = load_case("nopad")
    m = DrivingModel(vision_model={"variant": "tiny"}, language_model={"variant": "tiny", "lora_dropout": 0.0})
    res = m.load_state_dict(load_file(os.path.join(GOLDEN, "vla_tiny_refsd.safetensors")))
    assert res.missing_keys == [] and res.unexpected_keys == []
    sd = m.state_dict()
    assert list(sd) == list(KEYS["tiny"]) or set(sd) == set(KEYS["tiny"])
    path = str(tmp_path / "model.pt")
    torch.save(sd, path)
    m2 = DrivingModel(vision_model={"variant": "tiny"}, language_model={"variant": "tiny", "lora_dropout": 0.0})
    m2.load_state_dict(torch.load(path, weights_only=True))
    got = m2.vla_params()
    assert all(torch.equal(got[k], P[k]) for k in P)
    part = {k: v for k, v in sd.items() if k.startswith("adaptors.driving.")}
    res = m2.load_state_dict(part, strict=False)
    assert len(res.missing_keys) > 0 and res.unexpected_keys == []


def test_safe_load_names_unknown_globals(tmp_path):
    """A global outside the DeepSpeed / Lightning / OmegaConf packages is never stood in for: the weights-only
    error names it, and a stand-in never runs the original constructor."""
    import pickle
    import types
    from simlingo_amd.checkpoint import safe_load
    mod = types.ModuleType("evilpkg")

    class Payload:
        def __init__(self):
            self.x = 1
    Payload.__module__, Payload.__qualname__, mod.Payload = "evilpkg", "Payload", Payload
    sys.modules["evilpkg"] = mod
    try:
        torch.save({"p": Payload(), "t": torch.ones(1)}, str(tmp_path / "x.pt"))
    finally:
        sys.modules.pop("evilpkg")
    with pytest.raises(pickle.UnpicklingError, match="evilpkg.Payload"):
        safe_load(str(tmp_path / "x.pt"))
    LossScaler, _, _, _, cleanup = _fake_classes()
    torch.save({"ls": LossScaler(32.0)}, str(tmp_path / "y.pt"))
    cleanup()
    got = safe_load(str(tmp_path / "y.pt"))["ls"]
    assert type(got).__module__ == "simlingo_amd.checkpoint" and got._state == {"cur_scale": 32.0, "cur_iter": 0}


@pytest.mark.parametrize("prefix", ["omegaconf.listconfig", "lightning.fabric.utilities.data"])
def test_safe_load_list_subclass_becomes_plain_list(tmp_path, prefix):
    """A list subclass under a stand-in prefix (OmegaConf's ListConfig, a Lightning container) fills itself with
    APPEND / APPENDS; torch 2.10's weights-only unpickler words that error 'Can only append to lists' / 'Can only
    extend lists'. safe_load replaces the subclass by a plain list instead of re-raising."""
    import types
    from simlingo_amd.checkpoint import safe_load
    made = []
    parts = prefix.split(".")
    for i in range(1, len(parts) + 1):
        n = ".".join(parts[:i])
        if n not in sys.modules:
            sys.modules[n] = types.ModuleType(n)
            made.append(n)
    m = sys.modules[prefix]

    class ListConfig(list):
        pass
    ListConfig.__module__, ListConfig.__qualname__, m.ListConfig = prefix, "ListConfig", ListConfig
    try:
        torch.save({"hp": ListConfig([1, 2, 3]), "one": ListConfig([7]), "t": torch.ones(2)}, str(tmp_path / "l.pt"))
    finally:
        for n in made:
            sys.modules.pop(n, None)
    got = safe_load(str(tmp_path / "l.pt"))
    assert type(got["hp"]) is list and got["hp"] == [1, 2, 3] and got["one"] == [7]
    assert torch.equal(got["t"], torch.ones(2))


def test_trainable_ref_keys_match_to_reference():
    """The optimizer-state keys (FusedAdamW.state_dict) are exactly the reference state-dict keys and shapes of the
    trainable tensors (tiny case: the real tensors, so identity is checked; full geometry: keys and shapes)."""
    from simlingo_amd.checkpoint import trainable_ref_keys
    cfg, P, _, _ = load_case("nopad")
    sd = to_reference(P, cfg, aliases=False)
    names = trainable_ref_keys(cfg)
    assert len(names) == sum(1 for s in param_specs(cfg) if s.trainable)
    for n, (key, shape) in names.items():
        assert tuple(sd[key].shape) == shape, key
        assert sd[key].data_ptr() == P[n].data_ptr(), (n, key)
    full = full_config()
    keys = KEYS["full"]
    for n, (key, shape) in trainable_ref_keys(full).items():
        assert keys[key] == list(shape), key


def test_optimizer_state_round_trip_cpu():
    """simlingo_amd.optstate on a stand-in engine (flat m / v buffers + offsets, as VLAEngine holds them): export cuts the
    moments per reference key, import writes them back bit-exactly together with the step count, the param groups and
    the dropout counter; mismatched keys are refused."""
    import io
    import math
    from types import SimpleNamespace

    from simlingo_amd.checkpoint import trainable_ref_keys
    from simlingo_amd.optstate import export_state, import_state
    cfg, _, _, _ = load_case("nopad")
    names = trainable_ref_keys(cfg)
    offs, o = {}, 0
    for n, (_, shape) in names.items():
        offs[n] = o
        o += (math.prod(shape) + 63) // 64 * 64
    g = torch.Generator().manual_seed(0)
    eng = SimpleNamespace(device=torch.device("cpu"), offsets=offs, master=torch.zeros(o), step_seed=17,
                          m_state=torch.randn(o, generator=g), v_state=torch.rand(o, generator=g))
    p = torch.nn.Parameter(torch.zeros(()))
    opt = torch.optim.SGD([p], lr=3e-5)
    opt.step_count, opt.max_norm = 7, 0.3
    opt.param_groups[0]["betas"] = (0.87, 0.999)
    import torch.cuda as tc
    orig = tc.current_stream
    tc.current_stream = lambda *_: SimpleNamespace(synchronize=lambda: None)
    try:
        sd = export_state(opt, eng, names)
    finally:
        tc.current_stream = orig
    buf = io.BytesIO()
    torch.save(sd, buf)
    buf.seek(0)
    sd2 = torch.load(buf, weights_only=True)
    assert set(sd2["state"]) == {k for k, _ in names.values()}
    eng2 = SimpleNamespace(device=torch.device("cpu"), offsets=offs, master=torch.zeros(o), step_seed=0)
    opt2 = torch.optim.SGD([torch.nn.Parameter(torch.zeros(()))], lr=1.0)
    opt2.step_count, opt2.max_norm = 0, 0.3
    import_state(opt2, eng2, names, sd2)
    assert opt2.step_count == 7 and eng2.step_seed == 17 and opt2.param_groups[0]["betas"] == (0.87, 0.999)
    for n, (_, shape) in names.items():
        a, k = offs[n], math.prod(shape)
        assert torch.equal(eng2.m_state[a:a + k], eng.m_state[a:a + k])
        assert torch.equal(eng2.v_state[a:a + k], eng.v_state[a:a + k])
    bad = dict(sd2, state=dict(list(sd2["state"].items())[1:]))
    with pytest.raises(KeyError):
        import_state(opt2, eng2, names, bad)
