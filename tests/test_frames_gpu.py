"""Collate image path on the MI355X (csrc/frames.hip via slx_frames_to_tiles) vs the CPU oracle (real Pillow
resize + torchvision's ToTensor/Normalize ops) and the golden vectors: bit-exact (uint8 resample, f32 tiles
compared with torch.equal)."""
import numpy as np
import pytest
import torch

from frames_util import CASES, frame, golden, sha
from oracle import frames_oracle as O

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", sorted(CASES))
def test_tiles_bit_exact_vs_oracle_and_golden(dev, name):
    from simlingo_amd.frames import FramePreprocessor
    z = golden()
    W, H, cut, mx, seed = CASES[name]
    f = frame(W, H, seed)
    pre = FramePreprocessor(H, W, dev, max_num_grid=mx, cut_bottom=cut)
    got = pre(torch.from_numpy(f)[None].to(dev))
    torch.cuda.synchronize()
    got = got[0].cpu()
    want = O.preprocess_image_batch([f], 448, mx, cut)["pixel_values"][0]
    assert got.shape == want.shape
    assert torch.equal(got, want), (got - want).abs().max().item()
    assert sha(got.numpy()) == str(z[f"{name}.pixel_sha"])
    np.testing.assert_array_equal(pre.image_sizes(1).numpy(), z[f"{name}.image_sizes"])


def test_batch_channels_first_strided(dev):
    """The reference hands preprocess_image_batch [3, H, W] frames (datamodule.py:343-349): a channels-first,
    non-contiguous batch of distinct frames through the drop-in function."""
    from simlingo_amd.frames import preprocess_image_batch
    fr = np.stack([frame(1024, 512, 10 + i) for i in range(5)])              # [5, H, W, 3]
    chw = torch.from_numpy(fr).to(dev).permute(0, 3, 1, 2)                   # strided [5, 3, H, W] view
    r = preprocess_image_batch(chw, cut_bottom=True, channels_first=True)
    torch.cuda.synchronize()
    want = O.preprocess_image_batch(list(fr), 448, 2, True)
    assert torch.equal(r["pixel_values"].cpu(), want["pixel_values"])
    assert torch.equal(r["image_sizes"], want["image_sizes"])


def test_pipeline_double_buffered(dev):
    from simlingo_amd.frames import FramePipeline
    B = 4
    pipe = FramePipeline(B, 512, 1024, dev, depth=2)
    batches = [np.stack([frame(1024, 512, 100 * j + i) for i in range(B)]) for j in range(3)]
    outs = []
    pipe.put(batches[0])
    pipe.put(batches[1])
    with pytest.raises(RuntimeError):
        pipe.put(batches[2])                                                  # both slots in flight
    pv, sizes = pipe.get()
    outs.append(pv.cpu().clone())
    pipe.put(batches[2])                                                      # reuses slot 0 after its kernel
    for _ in range(2):
        pv, sizes = pipe.get()
        outs.append(pv.cpu().clone())
    with pytest.raises(RuntimeError):
        pipe.get()
    torch.cuda.synchronize()
    for j in range(3):
        want = O.preprocess_image_batch(list(batches[j]), 448, 2, True)["pixel_values"]
        assert torch.equal(outs[j][:, 0], want), j
    assert sizes.tolist() == [[359, 1024]] * B


def test_rejects_bad_inputs(dev):
    from simlingo_amd.frames import FramePreprocessor
    pre = FramePreprocessor(512, 1024, dev)
    with pytest.raises(RuntimeError):
        pre(torch.zeros(1, 512, 1024, 3, device=dev))                         # float frames
    with pytest.raises(ValueError):
        pre(torch.zeros(1, 500, 1024, 3, dtype=torch.uint8, device=dev))     # wrong geometry
    with pytest.raises(RuntimeError):
        pre(torch.zeros(1, 512, 1024, 3, dtype=torch.uint8))                  # host memory
