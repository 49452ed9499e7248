"""Collate: per-sample dataset outputs -> one DrivingExample (§8c (iii)).

Host half of `DataModule.dl_collate_fn` (simlingo_training/dataloader/datamodule.py:310-443) and the chat-template /
loss-mask helpers it calls (simlingo_training/utils/internvl2_utils.py:29-175). The image half is the HIP frame kernel
(`simlingo_amd.frames.preprocess_image_batch`, bit-exact Pillow bicubic tiling); everything here is string and index
work on the host, exactly as the reference's DataLoader workers do it.

Chat template. `get_custom_chat_template` builds its prompts with InternVL's `conversation.py`
(`get_conv_template('internlm2-chat')`), which the reference downloads from the hub at run time
(internvl2_utils.py:107-114) - a third-party file absent from /root/reference. Its published definition is restated
here: system template `<|im_start|>system\\n{system_message}`, roles `<|im_start|>user\\n` / `<|im_start|>assistant\\n`,
separator `<|im_end|>`, MPT separator style (`system + sep`, then `role + message + sep` per turn, a bare `role` for an
empty turn). The reference strips the system block again (internvl2_utils.py:156-159), so the system message text never
reaches the tokens. Tokenization uses the caller's tokenizer (the InternVL2-1B Qwen2 tokenizer in the reference, left
padding, datamodule.py:125-138); the user/assistant span search and the loss mask are restated from
`get_chat_tokens` / `get_assistant_loss_mask` and pinned against the reference's own functions
(tests/golden/chat_tokens.npz, oracle/gen_golden_chat.py).
"""
from __future__ import annotations

from typing import Callable, Dict, List, NamedTuple, Optional

import numpy as np
import torch

from .types import DrivingExample, DrivingInput, DrivingLabel, LanguageLabel

IMG_START_TOKEN, IMG_END_TOKEN, IMG_CONTEXT_TOKEN, IMG_TOKEN = "<img>", "</img>", "<IMG_CONTEXT>", "<image>"
# datamodule.py:130-137: placeholder tokens added to the tokenizer
PLACEHOLDER_TOKENS = ["<WAYPOINTS>", "<WAYPOINTS_DIFF>", "<ORG_WAYPOINTS_DIFF>", "<ORG_WAYPOINTS>", "<WAYPOINT_LAST>",
                      "<ROUTE>", "<ROUTE_DIFF>", "<TARGET_POINT>"]
# InternVL conversation.py 'internlm2-chat' [third-party, restated]
SYSTEM_TEMPLATE = "<|im_start|>system\n{system_message}"
ROLES = ("<|im_start|>user\n", "<|im_start|>assistant\n")
SEP = "<|im_end|>"


def mpt_prompt(messages: List[tuple], system_message: str = "") -> str:
    """Conversation.get_prompt for SeparatorStyle.MPT: system + sep, then role + message + sep per non-empty message,
    the bare role for an empty one (the generation prompt)."""
    ret = SYSTEM_TEMPLATE.format(system_message=system_message) + SEP
    for role, message in messages:
        ret += role + message + SEP if message else role
    return ret


def custom_chat_prompts(conversations: List[List[Dict]], num_image_tokens_total: int, system_message: str = ""):
    """internvl2_utils.py:94-162: per conversation [user, assistant] -> (full conversation prompt, question prompt),
    system block removed, the first '<image>' replaced by <img> + <IMG_CONTEXT> x N + </img>."""
    image_tokens = IMG_START_TOKEN + IMG_CONTEXT_TOKEN * num_image_tokens_total + IMG_END_TOKEN
    system = SYSTEM_TEMPLATE.format(system_message=system_message) + SEP
    convs, questions = [], []
    for conv in conversations:
        assert len(conv) == 2, "For question and answer templates only two turn conversation (user + assistant) is supported"
        msgs = []
        for i, part in enumerate(conv):
            text = part["content"][0]["text"]
            if part["role"] == "assistant":
                msgs.append((ROLES[1], text))
            elif part["role"] == "user":
                if i == 0 and IMG_TOKEN not in text:
                    text = f"{IMG_TOKEN}\n" + text
                msgs.append((ROLES[0], text))
            else:
                raise ValueError(f"Role {part['role']} not supported")
        assert conv[0]["role"] == "user", "First turn should be user as this should be the question."
        q = conv[0]["content"][0]["text"]
        if IMG_TOKEN not in q:
            q = f"{IMG_TOKEN}\n" + q
        pc = mpt_prompt(msgs, system_message).replace(system, "")
        pq = mpt_prompt([(ROLES[0], q), (ROLES[1], None)], system_message).replace(system, "")
        convs.append(pc.replace(IMG_TOKEN, image_tokens, 1))
        questions.append(pq.replace(IMG_TOKEN, image_tokens, 1))
    return convs, questions


def assistant_loss_mask(user_starts: List[List[int]], assistant_starts: List[List[int]], ids: torch.Tensor) -> torch.Tensor:
    """get_assistant_loss_mask (internvl2_utils.py:29-47): True from each assistant start to the token before the
    next user start (or to the end of the row)."""
    seq_len = ids.shape[1]
    mask = torch.zeros(ids.shape, dtype=torch.bool)
    for b, (us, as_) in enumerate(zip(user_starts, assistant_starts)):
        assert us[0] < as_[0], "First user start should be before first assistant start"
        assert len(us) == len(as_), "Number of user and assistant starts should be the same"
        for i, start in enumerate(as_):
            end = us[i + 1] - 1 if i < len(us) - 1 else seq_len - 1
            mask[b, start:end + 1] = True
    return mask


def _starts(ids: torch.Tensor, pattern: torch.Tensor) -> List[List[int]]:
    """Start positions of every occurrence of `pattern` in each row (the unfold/all match of get_chat_tokens), as the
    reference collects them: one list per match slot, filled by batch id (internvl2_utils.py:72-83)."""
    n = pattern.shape[0]
    hits = (ids.unfold(1, n, 1) == pattern).all(dim=2)
    rows, cols = torch.nonzero(hits, as_tuple=True)
    out = [[] for _ in range(len(rows))]
    for r, c in zip(rows.tolist(), cols.tolist()):
        out[r].append(c)
    return out


def chat_tokens(tokenizer, prompts: List[str], user_start: str = ROLES[0], assistant_start: str = ROLES[1]) -> Dict:
    """get_chat_tokens (internvl2_utils.py:50-91): tokenize with padding (no special tokens), valid = id != pad,
    loss mask over the assistant spans."""
    tok = tokenizer(prompts, padding=True, return_tensors="pt", add_special_tokens=False)
    ids = tok["input_ids"]
    valid = ids != tokenizer.pad_token_id
    us = _starts(ids, torch.tensor(tokenizer(user_start)["input_ids"]))
    as_ = _starts(ids, torch.tensor(tokenizer(assistant_start)["input_ids"]))
    return {"phrase_ids": ids, "phrase_valid": valid, "phrase_mask": valid, "language_string": prompts,
            "loss_masking": assistant_loss_mask(us, as_, ids)}


def get_custom_chat_template(conversations, tokenizer, num_image_tokens_total: int):
    """(conversation dict, question dict) as internvl2_utils.py:94-175 returns them."""
    convs, questions = custom_chat_prompts(conversations, num_image_tokens_total)
    return chat_tokens(tokenizer, convs), chat_tokens(tokenizer, questions)


def encode_uint8(strings: List[str], common_length: int) -> torch.Tensor:
    """datamodule.py:40-58: null-padded uint8 rows."""
    assert max(len(s) for s in strings) <= common_length, "String is too long"
    return torch.tensor([bytearray(s.ljust(common_length, "\0"), "utf-8") for s in strings], dtype=torch.uint8)


def camera_intrinsics(w: int, h: int, fov: float) -> torch.Tensor:
    """utils/projection.py:24-41."""
    k = np.identity(3)
    k[0, 0] = k[1, 1] = w / (2.0 * np.tan(fov * np.pi / 360.0))
    k[0, 2], k[1, 2] = w / 2.0, h / 2.0
    return torch.tensor(k, dtype=torch.float32)


def camera_extrinsics() -> torch.Tensor:
    """utils/projection.py:43-61: identity rotation, camera at (-1.5, 0, 2)."""
    e = np.zeros((4, 4), dtype=np.float32)
    e[3, 3] = 1.0
    e[:3, :3] = np.eye(3)
    e[:3, 3] = [-1.5, 0.0, 2.0]
    return torch.tensor(e, dtype=torch.float32)


class DatasetOutput(NamedTuple):
    """The fields of the reference's per-sample DatasetOutput that dl_collate_fn reads (custom_types.py,
    dataset_base.py)."""
    image_ff: np.ndarray                 # [T=1, C, H, W] uint8 camera frame (bottom crop already applied)
    image_ff_org_size: tuple
    conversation: List[Dict]             # [user, assistant] turns in the HF chat format
    answer: List[Dict]
    placeholder_values: Dict[str, np.ndarray]
    waypoints: np.ndarray                # [F, 2]
    path: np.ndarray                     # [20, 2]
    speed: np.ndarray
    target_points: np.ndarray
    measurement_path: str
    qa_templates: Optional[list] = None
    eval_infos: Optional[dict] = None


class Collate:
    """dl_collate_fn (datamodule.py:310-443) for the VLA: frames -> HIP tiles (`pixel_fn`, default the frame kernel
    of simlingo_amd.frames on `device`), conversations -> chat-template token ids and loss masks, labels -> tensors.
    `tokenizer` must already carry the placeholder special tokens and left padding (datamodule.py:130-138).

    The work splits at the host/device line so the host half can run where the reference runs its whole collate, in
    the DataLoader workers (datamodule.py:275-284, num_workers = 10): `host(data)` is CPU-only and picklable (token
    ids, masks, labels, the stacked uint8 frames as `camera_images`), `device(example)` uploads the frames through a
    pinned ring and tiles them with the HIP kernel in the training process. `__call__` = device(host(data))."""

    def __init__(self, tokenizer, num_image_tokens_per_patch: int = 256, num_image_patches: int = 2,
                 device=None, pixel_fn: Optional[Callable] = None, predict: bool = False, input_size: int = 448):
        self.tokenizer = tokenizer
        self.num_image_patches = num_image_patches
        self.num_image_tokens_total = num_image_tokens_per_patch * num_image_patches
        self.predict = predict
        self.device_ = device
        self.input_size = input_size
        self.pixel_fn = pixel_fn
        self._pres = {}
        self._uploader = None

    def __getstate__(self):  # DataLoader workers get the host half only
        st = dict(self.__dict__)
        st["_pres"], st["_uploader"] = {}, None
        return st

    def _default_pixels(self, frames_u8, max_num_grid):
        """preprocess_image_batch on the device: pinned-ring upload (no pageable H2D, no host sync) + frame kernel,
        one cached geometry per frame size."""
        from .frames import FramePreprocessor, FrameUploader
        dev = torch.device(self.device_) if self.device_ is not None else torch.device("cuda")
        B, _, H, W = frames_u8.shape
        key = (H, W, max_num_grid)
        if key not in self._pres:
            self._pres[key] = FramePreprocessor(H, W, dev, self.input_size, max_num_grid, False, cut_bottom=False)
        pre = self._pres[key]
        if not frames_u8.is_cuda:
            if self._uploader is None:
                self._uploader = FrameUploader(dev)
            frames_u8 = self._uploader(frames_u8)
        out = {"pixel_values": pre(frames_u8, channels_first=True), "image_sizes": pre.image_sizes(B)}
        if self._uploader is not None:
            self._uploader.release()
        return out

    def host(self, data: List[DatasetOutput]) -> DrivingExample:
        B = len(data)
        img = data[0].image_ff
        T, C, H, W = img.shape
        assert T == 1, "Only one timestep as input supported"
        frames = torch.from_numpy(np.stack([(d.image_ff if d.image_ff is not None else np.zeros_like(img)).reshape(C, H, W)
                                            for d in data]))
        conv_d, q_d = get_custom_chat_template([d.conversation for d in data], self.tokenizer,
                                               self.num_image_tokens_total)
        placeholders = [{self.tokenizer.convert_tokens_to_ids(k): v for k, v in d.placeholder_values.items()}
                        for d in data]
        prompt = LanguageLabel(conv_d["phrase_ids"], conv_d["phrase_valid"], conv_d["phrase_mask"], placeholders,
                               conv_d["language_string"], conv_d["loss_masking"])
        prompt_q = LanguageLabel(q_d["phrase_ids"], q_d["phrase_valid"], q_d["phrase_mask"], placeholders,
                                 q_d["language_string"], q_d["loss_masking"])
        answer = LanguageLabel(None, None, None, None, [d.answer[0]["content"][0]["text"] for d in data], None)
        f32 = torch.float32
        di = DrivingInput(
            camera_images=frames, image_sizes=None,
            camera_intrinsics=camera_intrinsics(W, H, 110).unsqueeze(0).repeat(B, 1, 1),
            camera_extrinsics=camera_extrinsics().unsqueeze(0).repeat(B, 1, 1),
            vehicle_speed=torch.tensor(np.asarray([d.speed for d in data]), dtype=f32),
            target_point=torch.tensor(np.asarray([d.target_points for d in data]), dtype=f32),
            prompt=prompt, prompt_inference=prompt_q)
        dl = DrivingLabel(
            waypoints=torch.tensor(np.asarray([d.waypoints for d in data]), dtype=f32),
            path=torch.tensor(np.asarray([d.path for d in data]), dtype=f32), answer=answer,
            image_ff_org=torch.tensor(np.asarray([d.image_ff_org_size for d in data])),
            eval_infos=[d.eval_infos for d in data] if self.predict else None)
        qa = [d.qa_templates[0] if d.qa_templates is not None else None for d in data] if self.predict else None
        return DrivingExample(driving_input=di, driving_label=dl,
                              run_id=encode_uint8([d.measurement_path for d in data], 1000), qa_templates=qa)

    def device(self, ex: DrivingExample) -> DrivingExample:
        """uint8 frames [B, C, H, W] of a host() batch -> pixel tiles [B, T=1, tiles, C, s, s] (device)."""
        di = ex.driving_input
        frames = di.camera_images
        B, C = frames.shape[:2]
        fn = self.pixel_fn if self.pixel_fn is not None else self._default_pixels
        processed = fn(frames, self.num_image_patches)
        pix = processed["pixel_values"]
        pix = pix.view(B, 1, pix.shape[1], C, pix.shape[-2], pix.shape[-1])
        return ex._replace(driving_input=di._replace(camera_images=pix, image_sizes=processed["image_sizes"]))

    def __call__(self, data: List[DatasetOutput]) -> DrivingExample:
        return self.device(self.host(data))
