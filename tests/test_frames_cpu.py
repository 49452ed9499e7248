"""Collate image path, CPU side: the oracle against Pillow and the golden vectors, the
C-ABI host coefficient builder against the oracle, and the host grid logic. No GPU calls."""
import numpy as np
import pytest
from PIL import Image

from frames_util import CASES, frame, golden, sha
from oracle import frames_oracle as O
from simlingo_amd import frames as F


@pytest.mark.parametrize("name", sorted(CASES))
def test_oracle_matches_golden(name):
    z = golden()
    W, H, cut, mx, seed = CASES[name]
    f = frame(W, H, seed)
    assert sha(f) == str(z[f"{name}.input_sha"]), "seeded input frame drifted"
    r = O.preprocess_image_batch([f], 448, mx, cut)
    pv = r["pixel_values"][0].numpy()
    assert sha(r["resized"][0]) == str(z[f"{name}.resized_sha"])
    assert sha(pv) == str(z[f"{name}.pixel_sha"])
    np.testing.assert_array_equal(pv.reshape(-1)[z[f"{name}.sample_idx"]], z[f"{name}.sample_val"])
    np.testing.assert_array_equal(r["image_sizes"].numpy(), z[f"{name}.image_sizes"])


@pytest.mark.parametrize("geom", [(1024, 359, 896, 448), (300, 200, 448, 448), (2000, 900, 896, 448),
                                  (37, 23, 448, 896), (1024, 512, 896, 448), (5, 3, 448, 448)])
def test_resample_restatement_bit_exact_vs_pillow(geom):
    W, H, tw, th = geom
    img = np.random.default_rng(W * 7 + H).integers(0, 256, (H, W, 3), dtype=np.uint8)
    np.testing.assert_array_equal(O.pil_resize_bicubic(img, tw, th), np.asarray(Image.fromarray(img).resize((tw, th))))


@pytest.mark.parametrize("ax", [(1024, 896), (359, 448), (2000, 896), (900, 448), (23, 448), (448, 448), (1, 7)])
def test_capi_coeffs_match_oracle(ax):
    b1, k1 = O.pil_resample_coeffs(*ax)
    b2, k2 = F.resample_coeffs(*ax)
    np.testing.assert_array_equal(b1, b2)
    np.testing.assert_array_equal(k1, k2)


def test_capi_coeffs_match_golden():
    z = golden()
    for a, b in ((1024, 896), (359, 448)):
        bd, kk = F.resample_coeffs(a, b)
        np.testing.assert_array_equal(bd, z[f"coeffs_{a}_{b}.bounds"])
        np.testing.assert_array_equal(kk, z[f"coeffs_{a}_{b}.kk"])


def test_capi_coeffs_errors():
    from simlingo_amd import kernels as K
    bd = np.zeros((4, 2), np.int32)
    kk = np.zeros((4, 2), np.int32)
    rc = K.lib().slx_resample_coeffs(8, 4, 2, bd.ctypes.data_as(F._i32p), kk.ctypes.data_as(F._i32p))
    assert rc < 0 and b"kmax" in K.lib().slx_last_error()
    assert K.lib().slx_resample_ksize(0, 4) < 0


def test_grid_and_crop_host_logic():
    assert F.bottom_crop_rows(512) == 359
    assert F.bottom_crop_rows(1024) == 717
    for W, H in [(1024, 359), (1024, 512), (300, 200), (23, 37), (448, 448), (1000, 1000), (100, 10)]:
        for mx in (1, 2, 4, 6, 12):
            assert F.closest_grid(W, H, 1, mx) == O.closest_grid(W, H, 1, mx), (W, H, mx)
    assert F.closest_grid(1024, 359, 1, 2) == (2, 1)


def test_capi_frames_rejects_undersized_lds_window():
    """a C-ABI caller that passes an LDS window smaller than the blocks' Pillow source span is rejected
    before any launch (no GPU needed: the argument check runs on the host)."""
    import ctypes
    from simlingo_amd import kernels as K
    d = F.FrameDesc()
    d.src, d.out, d.hbounds, d.hcoeffs, d.vbounds, d.vcoeffs = 16, 16, 16, 16, 16, 16  # never dereferenced
    d.B, d.H, d.W, d.tw, d.th, d.tile = 1, 359, 1024, 896, 448, 448
    d.sb, d.sy, d.sx, d.sc = 359 * 1024 * 3, 1024 * 3, 3, 1
    d.hksize, d.vksize = 5, 7
    d.need_h, d.need_v = 1, 1
    d.rows_per_block, d.cols_per_block = 16, 128
    d.lds_rows, d.lds_cols = 4, 40   # far below the real span (about 15 rows x 147 columns)
    rc = K.lib().slx_frames_to_tiles(ctypes.byref(d), None)
    assert rc != 0
    assert b"LDS window" in K.lib().slx_last_error()
