"""AdaptorList seam of the MI355X DrivingModel (simlingo_training/models/adaptors/adaptors.py:281-370).

`DrivingModel.adaptors(example)` returns the reference's dict (keys inputs, inputs_mask, perm, split_sizes,
language_inputs, language_inputs_mask, language__ids, language__ids_mask, driving_inputs, driving_inputs_mask) built
from the host token plan (plan.py: the same valid-first permutation) and the engine's embedding / query tables;
`compute_loss(features, logits, input_dict, example)` returns {key: (values, counts)} plus the route / speed
predictions, running the driving heads and the smooth-L1 / cross-entropy on the HIP kernels (sgemm, slx_wp_loss_fwd,
slx_ce_fwd). The training step does not go through here (VLAEngine fuses all of it); these serve the reference's
other callers (VisualiseCallback, predict_step, the agent's forward_model path).
"""
from __future__ import annotations

import torch

from . import kernels as K
from .plan import plan_from_example
from .vlm import _Bound

F32 = torch.float32


class AdaptorList(_Bound):
    def __call__(self, example, inference: bool = False, **kwargs):
        return self.forward(example, inference=inference, **kwargs)

    @torch.no_grad()
    def forward(self, example, inference: bool = False, **kwargs) -> dict:
        """adaptors.py:301-331 (LanguageAdaptor.forward :238-257, DrivingAdaptor.forward :139-161)."""
        eng = self.engine
        cfg = eng.cfg
        di = example.driving_input if hasattr(example, "driving_input") else example
        lab = di.prompt_inference if inference else di.prompt
        plan = plan_from_example(cfg, example, inference=inference)
        dplan = plan.to_device(eng.device)
        B, L, S, d, NQ = plan.B, plan.L, plan.S, cfg.llm_dim, cfg.n_queries
        dev = eng.device
        ids = lab.phrase_ids.long().to(dev)
        valid = lab.phrase_valid.bool().to(dev)
        lang = torch.empty(B * L, d, dtype=F32, device=dev)
        idx = ids.clamp(0, cfg.vocab - 1).to(torch.int32).reshape(-1)  # embed_tokens(ids.clamp(0, V-1)), :256
        K.call("slx_gather_rows_b2f", K.P(eng.W["llm.embed"]), d, K.P(idx), B * L, d, K.P(lang), d, K.stream_ptr())
        lang = lang.view(B, L, d)
        qrows = torch.cat([eng.P["drv.query_route"], eng.P["drv.query_speed"]], 0)  # [30, d] (adjacent params)
        driving = qrows[None].expand(B, NQ, d)
        inputs = torch.cat([lang, driving], 1)
        mask = torch.cat([valid, torch.ones(B, NQ, dtype=torch.bool, device=dev)], 1)
        perm = torch.from_numpy(plan.perm).to(dev)
        ar = torch.arange(B, device=dev)[:, None]
        return {"language_inputs": lang, "language_inputs_mask": valid, "language__ids": ids,
                "language__ids_mask": lab.loss_masking.bool().to(dev),
                "driving_inputs": driving, "driving_inputs_mask": torch.ones(B, NQ, dtype=torch.bool, device=dev),
                "inputs": inputs[ar, perm].contiguous(), "inputs_mask": mask[ar, perm], "perm": perm,
                "split_sizes": torch.as_tensor([L, NQ]), "_plan": plan, "_dplan": dplan}

    def split_outputs_by_adaptor(self, input_dict: dict, outputs: torch.Tensor) -> dict:
        """adaptors.py:357-370: undo the permutation, split [language | driving]."""
        inv = input_dict["perm"].argsort(-1)
        ar = torch.arange(inv.size(0), device=inv.device)[:, None]
        out = outputs[ar, inv]
        sizes = [int(x) for x in input_dict["split_sizes"]]
        lang, drv = out.split(sizes, dim=1)
        return {"language": lang, "driving": drv}

    @torch.no_grad()
    def compute_loss(self, features: torch.Tensor, logits: torch.Tensor, input_dict: dict, example) -> dict:
        """adaptors.py:333-355 (+ DrivingAdaptor.compute_loss :183-221, LanguageAdaptor.compute_loss :259-274):
        {"language_loss": (CE [B, L-1], mask), "route_loss": ([B, 20], ones), "speed_wps_loss": ([B, 10], ones),
        "route_prediction": [B, 20, 2], "speed_wps_prediction": [B, 10, 2]}."""
        eng = self.engine
        cfg = eng.cfg
        dev = eng.device
        feats = self.split_outputs_by_adaptor(input_dict, features.to(dev).float())
        out = {}
        if logits is not None:
            lg = self.split_outputs_by_adaptor(input_dict, logits.to(dev).float())["language"][:, :-1]
            labels = torch.where(input_dict["language__ids_mask"], input_dict["language__ids"], -1)[:, 1:]
            B, Lm1, V = lg.shape
            rows = lg.reshape(B * Lm1, V).contiguous()
            lab = labels.reshape(-1).to(torch.int32).contiguous()
            loss = torch.empty(B * Lm1, dtype=F32, device=dev)
            lse = torch.empty(B * Lm1, dtype=F32, device=dev)
            K.call("slx_ce_fwd", K.P(rows), V, K.P(lab), B * Lm1, V, K.P(loss), K.P(lse), K.stream_ptr())
            loss = loss.view(B, Lm1)  # ignore_index rows come out 0 (slx_ce_fwd)
            out["language_loss"] = (loss, labels.ne(-1))
        dfeat = feats["driving"]  # [B, 30, d]
        B = dfeat.shape[0]
        nr, ns, m = cfg.n_route, cfg.n_speed, cfg.head_mlp
        fr = dfeat[:, :nr].reshape(B * nr, -1).contiguous()
        fs = dfeat[:, nr:].reshape(B * ns, -1).contiguous()
        hd = eng._mlp_fwd(fr, [("route.0", 2 * m, K.ACT_SILU), ("route.1", m, K.ACT_SILU), ("route.2", 2, K.ACT_NONE)])
        sd = eng._mlp_fwd(fs, [("speed.0", m, K.ACT_SILU), ("speed.1", cfg.speed_dims, K.ACT_NONE)])
        lab = example.driving_label
        route_pred = torch.empty(B, nr, 2, dtype=F32, device=dev)
        route_loss = torch.empty(B * nr, dtype=F32, device=dev)
        K.call("slx_wp_loss_fwd", K.P(hd[0][0]), K.P(lab.path.float().to(dev).contiguous()), B, nr, 2, 0,
               K.P(route_pred), K.P(route_loss), K.stream_ptr())
        speed_pred = torch.empty(B, ns, cfg.speed_dims, dtype=F32, device=dev)
        speed_loss = torch.empty(B * ns, dtype=F32, device=dev)
        K.call("slx_wp_loss_fwd", K.P(sd[0][0]), K.P(lab.waypoints[:, : nr + 1].float().to(dev).contiguous()), B, ns,
               cfg.speed_dims, 0, K.P(speed_pred), K.P(speed_loss), K.stream_ptr())
        out["route_loss"] = (route_loss.view(B, nr), torch.ones(B, nr, device=dev))
        out["speed_wps_loss"] = (speed_loss.view(B, ns), torch.ones(B, ns, device=dev))
        out["route_prediction"] = route_pred
        out["speed_wps_prediction"] = speed_pred
        return out
