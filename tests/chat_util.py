"""Synthetic HF tokenizer for the collate / chat-template tests: a word-level `tokenizers` model wrapped in
transformers' PreTrainedTokenizerFast (left padding, as datamodule.py:138 sets it), whose special-token ids match the
tiny VLA geometry (simlingo_amd.config.tiny_config): <|im_end|> = eos 248, <pad> 249, <img> 250, </img> 251,
<IMG_CONTEXT> 252, placeholders 256..263 (>= vocab, clamped by the embedding lookup like the reference's added
tokens). The InternVL2 Qwen2 tokenizer itself is not available offline; the chat-template / loss-mask logic only
needs a tokenizer with the same call surface."""
from tokenizers import Regex, Tokenizer, models, normalizers, pre_tokenizers
from transformers import PreTrainedTokenizerFast

WORDS = ("user assistant system what should the ego vehicle do next drive slow down stop turn left right go straight "
         "follow lane because there is a red light pedestrian car ahead keep speed accelerate brake at target point "
         "route waypoints are commentary question answer and to of in on it this that with for near far green yellow "
         "intersection crossing bicycle truck bus parked construction zone merge change overtake wait yield").split()
PUNCT = list(".,?!:;'-()") + [str(d) for d in range(10)] + [" ", "\n"]


def build_tokenizer():
    vocab = {}
    for w in WORDS + PUNCT:
        vocab.setdefault(w, len(vocab))
    assert len(vocab) < 248
    for i in range(len(vocab), 248):  # no holes in the id space
        vocab[f"<w{i}>"] = i
    vocab.update({"<|im_end|>": 248, "<pad>": 249, "<img>": 250, "</img>": 251, "<IMG_CONTEXT>": 252,
                  "<|im_start|>": 253, "<unk>": 254})
    tk = Tokenizer(models.WordLevel(vocab=vocab, unk_token="<unk>"))
    tk.normalizer = normalizers.Lowercase()
    tk.pre_tokenizer = pre_tokenizers.Split(Regex(r"\n| |[A-Za-z]+|[0-9]|[^\sA-Za-z0-9]"), behavior="isolated")
    specials = ["<|im_end|>", "<pad>", "<img>", "</img>", "<IMG_CONTEXT>", "<|im_start|>", "<unk>"]
    tok = PreTrainedTokenizerFast(tokenizer_object=tk, pad_token="<pad>", unk_token="<unk>", eos_token="<|im_end|>",
                                  additional_special_tokens=specials[2:])
    # the SimLingo placeholders (datamodule.py:130-137), appended at ids 255.. in order
    from simlingo_amd.collate import PLACEHOLDER_TOKENS
    tok.add_special_tokens({"additional_special_tokens": specials[2:] + ["<spare>"] + PLACEHOLDER_TOKENS})
    tok.padding_side = "left"
    assert tok.convert_tokens_to_ids("<WAYPOINTS>") == 256 and tok.convert_tokens_to_ids("<TARGET_POINT>") == 263
    return tok


CONVERSATIONS = [
    ("What should the ego vehicle do next?", "Slow down because there is a pedestrian ahead."),
    ("<image>\nWhat should the ego vehicle do next? Target point <TARGET_POINT> .",
     "Turn left at the intersection and follow the route."),
    ("Drive.", "Stop."),
    ("What should the ego vehicle do next? The route is <ROUTE> and waypoints are <WAYPOINTS> .",
     "Keep speed, go straight, the light is green and there is no car ahead; follow lane to the target point."),
]


def conversation(q, a):
    return [{"role": "user", "content": [{"type": "text", "text": q}]},
            {"role": "assistant", "content": [{"type": "text", "text": a}]}]
