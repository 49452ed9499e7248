"""The reference's encoder / language-model modules as inner seams of the MI355X DrivingModel.

Hydra instantiates VLMEncoderConfig._target_ (simlingo_training/config.py:46) and LanguageModelConfig._target_
(:71) inside DrivingModel.__init__ (driving.py:62-74). Here the classes keep those constructor signatures and config
keys, and - once bound to a DrivingModel (which owns the VLAEngine and its parameters) - serve the calls other
reference code makes on them, on the same HIP kernels as the training step:

  vision_model.image_encoder.extract_feature(pixel_values)            internvl2_model.py:114 (InternViT + mlp1)
  vision_model.image_encoder.replace_placeholder_tokens(adaptor_dict, pixel_values, placeholder_values, wp_encoder)
                                                                      internvl2_model.py:17-144 (mutates the dict)
  language_model.model(attention_mask, position_ids, inputs_embeds, output_hidden_states, return_dict)
                                                                      driving.py:217-225 -> [0] logits, .hidden_states
  language_model.forward(embeddings, attention_mask, return_dict, position_ids) -> (features, logits)  llm.py:126-143
  language_model.sample_categorical / greedy_sample                   llm.py:145-250

They run in eval mode (LoRA dropout off), reuse the step's activation arena (call them between training steps, as
the reference's VisualiseCallback does, callbacks/visualise.py:205-208), and need the HIP library like everything else.
Key-padding masks must be valid-first (the layout AdaptorList.forward produces); other masks raise.
"""
from __future__ import annotations

import weakref

import torch
from torch import nn

from . import kernels as K

F32 = torch.float32


class _Bound:
    """Weak back-reference to the owning DrivingModel (a strong one would make the module tree cyclic)."""

    def _bind(self, owner):
        object.__setattr__(self, "_owner_ref", weakref.ref(owner))
        return self

    @property
    def owner(self):
        ref = getattr(self, "_owner_ref", None)
        m = ref() if ref is not None else None
        if m is None:
            raise RuntimeError(f"{type(self).__name__} is not bound to a DrivingModel (build it through DrivingModel)")
        return m

    @property
    def engine(self):
        return self.owner.build_engine()


class ModelOutput:
    """Minimal CausalLMOutputWithPast stand-in: out[0] = logits, out.hidden_states[-1] = post-norm features."""

    def __init__(self, logits, features):
        self.logits = logits
        self.hidden_states = (features,)

    def __getitem__(self, i):
        return (self.logits,)[i]


def _valid_lengths(mask: torch.Tensor | None, B: int, S: int, device) -> torch.Tensor:
    """[B] int32 valid-row counts of a valid-first key-padding mask (None = all valid)."""
    if mask is None:
        return torch.full((B,), S, dtype=torch.int32, device=device)
    m = mask.to(device).bool()
    n = m.sum(1)
    ar = torch.arange(S, device=device)[None]
    if not torch.equal(m, ar < n[:, None]):
        raise NotImplementedError("the MI355X kernels take valid-first key-padding masks (AdaptorList.forward's layout)")
    return n.to(torch.int32)


class LingoInternVLModel(_Bound):
    """internvl2_model.py:6-144 surface over the engine's InternViT + mlp1 + token assembly."""

    def extract_feature(self, pixel_values: torch.Tensor) -> torch.Tensor:
        """[N, 3, 448, 448] (or [B, T, tiles, 3, 448, 448]) normalised tiles -> vit_embeds [N, 256, d] f32."""
        eng = self.engine
        cfg = eng.cfg
        pix = pixel_values.reshape(-1, 3, cfg.img_size, cfg.img_size).to(eng.device)
        img = eng.vit_features(pix)
        return img.float().view(pix.shape[0], cfg.img_tokens_per_tile, cfg.llm_dim)

    @torch.no_grad()
    def replace_placeholder_tokens(self, adaptor_dict: dict, pixel_values, placeholder_values, wp_encoder=None) -> dict:
        """Writes the vision features, the wp_encoder rows of the <TARGET_POINT> placeholders and the image merge into
        adaptor_dict['language_inputs'] and ['inputs'] in place (internvl2_model.py:44-142) and returns the dict.

        placeholder_values: the caller's coordinates are used (the reference reads them here, :80-81); when they
        differ from those of the example the dict was built from, the token plan is rebuilt from the dict's ids and
        masks with the caller's values. wp_encoder: a caller-supplied module (WaypointInputAdaptor, called on
        [1, n, 2] in its own dtype as :80-82 does) produces the placeholder rows; None uses the engine's own
        wp_encoder weights (the DrivingModel's, which is what the reference's forward_model passes)."""
        import numpy as np
        from .plan import build_plan
        eng = self.engine
        cfg = eng.cfg
        plan, dplan = adaptor_dict["_plan"], adaptor_dict["_dplan"]
        if placeholder_values is not None:
            p2 = build_plan(cfg, adaptor_dict["language__ids"], adaptor_dict["language_inputs_mask"],
                            adaptor_dict["language__ids_mask"], placeholder_values, plan.n_img)
            if not (np.array_equal(p2.wp_coords, plan.wp_coords) and np.array_equal(p2.code, plan.code)):
                plan, dplan = p2, p2.to_device(eng.device)
                adaptor_dict["_plan"], adaptor_dict["_dplan"] = plan, dplan
        X = eng.encode_inputs(pixel_values.to(eng.device), plan, dplan, {})  # [B*S, d] f32, permuted layout
        B, S, L, d = plan.B, plan.S, plan.L, cfg.llm_dim
        nwp = plan.wp_coords.shape[0]
        if wp_encoder is not None and nwp:
            w0 = wp_encoder.mlp[0].weight if hasattr(wp_encoder, "mlp") else next(wp_encoder.parameters())
            coords = torch.from_numpy(plan.wp_coords).to(w0.device, w0.dtype)
            rows = wp_encoder(coords.unsqueeze(0)).squeeze(0).to(eng.device, F32)
            pos = torch.from_numpy(plan.wp_pos.astype(np.int64)).to(eng.device)
            keep = pos < B * S  # rows the permuted layout does not reference stay out (plan.py wp_pos)
            X[pos[keep]] = rows[keep]
        adaptor_dict["inputs"].copy_(X.view(B, S, d))
        # language positions p >= perm[b, 0] sit at final position p - perm[b, 0] (internvl2_model.py:139-142)
        lang = adaptor_dict["language_inputs"]
        for b in range(B):
            i0 = int(plan.perm[b, 0])
            lang[b, i0:].copy_(X.view(B, S, d)[b, : L - i0])
        return adaptor_dict


class VLMEncoderModel(nn.Module, _Bound):
    """simlingo_training/models/encoder/vlm.py:6-44 signature: (cfg_data_module, processor, cache_dir, **cfg)."""

    def __init__(self, cfg_data_module=None, processor=None, cache_dir=None, **cfg):
        super().__init__()
        for key, value in cfg.items():
            setattr(self, key, value)
        self.variant = cfg.get("variant", "OpenGVLab/InternVL2-1B")
        self.embed_dim = cfg.get("embed_dim", 512)
        self.freeze = cfg.get("freeze", False)
        self.token_size = self.embed_dim  # vlm.py:20
        if "internvl2" not in self.variant.lower() and self.variant != "tiny":
            raise ValueError(f"Unknown variant {self.variant}")
        self.image_encoder = LingoInternVLModel()

    def _bind(self, owner):
        _Bound._bind(self, owner)
        self.image_encoder._bind(owner)
        return self


class _CausalLM(_Bound):
    """language_model.model: peft(Qwen2ForCausalLM) call surface (driving.py:217-223)."""

    @torch.no_grad()
    def __call__(self, attention_mask=None, position_ids=None, inputs_embeds=None, output_hidden_states=True,
                 return_dict=True, **_):
        if position_ids is not None:
            raise NotImplementedError("position_ids other than arange (driving.py:207 passes None)")
        eng = self.engine
        emb = inputs_embeds.to(eng.device)
        B, S, d = emb.shape
        feat, logits = eng.llm_features(emb.float().reshape(B * S, d).contiguous(), B, S,
                                        _valid_lengths(attention_mask, B, S, eng.device), logits=True)
        return ModelOutput(logits.view(B, S, -1), feat.view(B, S, d))


class LLM(nn.Module, _Bound):
    """simlingo_training/models/language_model/llm.py:49-250: (**cfg) constructor, forward, sample_categorical,
    greedy_sample."""

    def __init__(self, **cfg):
        super().__init__()
        for key, value in cfg.items():
            setattr(self, key, value)
        self.variant = cfg.get("variant", "OpenGVLab/InternVL2-1B")
        if "internvl" not in self.variant.lower() and self.variant != "tiny":
            raise ValueError(f"Carefull: Variant {self.variant} not tested.")
        self.lora = cfg.get("lora", True)
        self.lora_alpha = cfg.get("lora_alpha", 64)
        self.lora_r = cfg.get("lora_r", 32)
        self.lora_dropout = cfg.get("lora_dropout", 0.1)
        self.model = _CausalLM()

    def _bind(self, owner):
        _Bound._bind(self, owner)
        self.model._bind(owner)
        cfg = owner.vla_cfg
        self.vocab_size, self.hidden_size = cfg.vocab, cfg.llm_dim  # llm.py:120-121
        return self

    def forward(self, embeddings, attention_mask=None, return_dict: bool = True, position_ids=None):
        """llm.py:126-143 -> (features = hidden_states[-1] post-norm [B,S,d], logits [B,S,V])."""
        out = self.model(attention_mask=attention_mask, position_ids=position_ids, inputs_embeds=embeddings)
        return out.hidden_states[-1], out[0]

    def sample_categorical(self, logits, temperature: float = 0.0, top_k=None, top_p=None, restrict_tokens=None):
        """llm.py:145-176. Greedy (temperature <= 0) is the argmax the agent uses; stochastic sampling is not on the
        MI355X path."""
        if restrict_tokens is not None:
            logits = logits.clone()
            logits[..., : restrict_tokens[0]] = -float("inf")
            logits[..., restrict_tokens[0] + restrict_tokens[1]:] = -float("inf")
        if temperature <= 0.0:
            return logits.argmax(dim=-1, keepdim=False)
        raise NotImplementedError("temperature > 0 sampling (the agent decodes greedily, driving.py:147)")

    @torch.no_grad()
    def greedy_sample(self, input_embeds, inputs_mask=None, max_new_tokens: int = 100, temperature: float = 0.0,
                      top_k=None, top_p=None, eos_token_id=None, cache_offset: int = 0, input_embed_matrix=None,
                      logit_matrix=None, restrict_tokens=None, attention_mask=None, position_ids=None):
        """llm.py:178-250 -> (sampled_tokens [B, n] int64, input_embeds [B, S0 + n, d]) on the KV-cached decoder
        (simlingo_amd.decode): every sample decodes its valid prompt rows; finished samples are padded with EOS as
        the reference's fill does."""
        if temperature > 0.0 or restrict_tokens is not None or input_embed_matrix is not None or logit_matrix is not None:
            raise NotImplementedError("greedy_sample on MI355X: temperature 0, the model's own embed / lm_head")
        owner = self.owner
        eng = self.engine
        dec = owner.decoder()
        emb = input_embeds.to(eng.device).float()
        B, S0, d = emb.shape
        n_valid = _valid_lengths(attention_mask if attention_mask is not None else inputs_mask, B, S0, eng.device)
        eos = eos_token_id if eos_token_id is not None else -1  # None: no early stop (llm.py:241)
        saved, dec.eos = dec.eos, int(eos)
        try:
            toks = [dec.generate(emb[b, : int(n_valid[b])].contiguous(), max_new_tokens) for b in range(B)]
        finally:
            dec.eos = saved
        n = max((t.numel() for t in toks), default=0)
        out = torch.full((B, n), eos if eos_token_id is not None else 0, dtype=torch.long)
        for b, t in enumerate(toks):
            out[b, : t.numel()] = t
        idx = out.to(eng.device).to(torch.int32).reshape(-1)
        new = torch.empty(B * n, d, dtype=F32, device=eng.device)
        if n:
            K.call("slx_gather_rows_b2f", K.P(eng.W["llm.embed"]), d, K.P(idx), B * n, d, K.P(new), d, K.stream_ptr())
        return out.to(eng.device), torch.cat([emb, new.view(B, n, d)], 1)
