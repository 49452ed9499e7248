"""Golden fixture for the collate's chat tokens and loss masks (tests/golden/chat_tokens.npz).

Test infrastructure only. The reference's `get_chat_tokens` / `get_assistant_loss_mask`
(simlingo_training/utils/internvl2_utils.py:29-91) are pure torch, but their module imports torchvision (absent), so
the two function definitions are read from the reference file with `ast` and executed on their own, unmodified
(nothing is copied into this repository). Inputs: the prompts of tests/chat_util.CONVERSATIONS built by
simlingo_amd.collate.custom_chat_prompts (the internlm2-chat template restatement; InternVL's conversation.py itself
is a hub download absent from /root/reference, so the prompt strings are pinned only by the structure tests in
tests/test_collate_cpu.py) and a multi-round case for the loss mask. Outputs: token ids, valid masks and loss masks of
the conversation and question prompts, and the multi-round mask.

    python oracle/gen_golden_chat.py
"""
import ast
import os
import sys
from typing import Dict, List

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
REF = "/root/reference/simlingo_training/utils/internvl2_utils.py"


def reference_functions():
    tree = ast.parse(open(REF).read())
    keep = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name in ("get_assistant_loss_mask",
                                                                                   "get_chat_tokens")]
    ns = {"torch": torch, "Dict": Dict, "List": List}
    exec(compile(ast.Module(body=keep, type_ignores=[]), REF, "exec"), ns)
    return ns["get_chat_tokens"], ns["get_assistant_loss_mask"]


def main():
    from chat_util import CONVERSATIONS, build_tokenizer, conversation
    from simlingo_amd.collate import ROLES, custom_chat_prompts
    get_chat_tokens, get_assistant_loss_mask = reference_functions()
    tok = build_tokenizer()
    convs, questions = custom_chat_prompts([conversation(q, a) for q, a in CONVERSATIONS], 8)
    out = {}
    for tag, prompts in (("conv", convs), ("question", questions)):
        d = get_chat_tokens(tok, prompts, ROLES[0], ROLES[1])
        out[f"{tag}.prompts"] = np.asarray(prompts)
        for k in ("phrase_ids", "phrase_valid", "phrase_mask", "loss_masking"):
            out[f"{tag}.{k}"] = d[k].numpy()
    ids = torch.zeros(2, 30, dtype=torch.long)
    us, as_ = [[0, 10, 20], [3, 15]], [[5, 12, 25], [8, 29]]
    out["multi.user_starts"] = np.asarray([0, 10, 20, 3, 15])
    out["multi.assistant_starts"] = np.asarray([5, 12, 25, 8, 29])
    out["multi.loss_mask"] = get_assistant_loss_mask(us, as_, ids).numpy()
    path = os.path.join(ROOT, "tests", "golden", "chat_tokens.npz")
    np.savez(path, **out)
    print("wrote", path, {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
