"""Post-process and output: the reference's display
median filter (kernelMedianFilter, cu:773-842), Scotty3D's tonemap
(image.h:168-185 + update_pixel image.h:49-58) and the PNG / PFM writers."""
import struct
import zlib

import numpy as np
import pytest

import ptrace
import pyoracle
from conftest import load_fixture


def _frame(rng, h, w, nan=False):
    img = rng.random((h, w, 4), dtype=np.float32) * 2.0
    img[..., 3] = 1.0
    img[rng.random((h, w)) < 0.1] = 0.5  # ties
    if nan:
        img[rng.random((h, w)) < 0.05, 0] = np.nan
    return img


def test_oracle_median_is_fourth_largest():
    rng = np.random.default_rng(3)
    img = _frame(rng, 9, 13)
    out = pyoracle.median(img)
    pad = np.pad(img[..., :3], ((1, 1), (1, 1), (0, 0)), constant_values=1.0)
    for r in range(9):
        for c in range(13):
            win = pad[r:r + 3, c:c + 3].reshape(9, 3)
            assert np.array_equal(out[r, c, :3], np.sort(win, axis=0)[::-1][3])
            assert out[r, c, 3] == 1.0


def test_tonemap_matches_scotty_formula():
    rng = np.random.default_rng(4)
    img = _frame(rng, 7, 5) * 3.0
    got = ptrace.tonemap(img, 2.2, 1.0)
    e = np.float32(np.sqrt(np.float32(2.0)))
    want = np.clip(np.power(img[..., :3] * e, np.float32(1.0 / 2.2)), 0, 1) * 255
    assert np.abs(got[..., :3].astype(int) - np.floor(want).astype(int)).max() <= 1
    assert (got[..., 3] == 255).all()


def _read_png(path):
    data = open(path, "rb").read()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat, w, h = 8, b"", None, None
    while pos < len(data):
        n, t = struct.unpack(">I4s", data[pos:pos + 8])
        body = data[pos + 8:pos + 8 + n]
        assert zlib.crc32(t + body) == struct.unpack(">I", data[pos + 8 + n:pos + 12 + n])[0]
        if t == b"IHDR":
            w, h = struct.unpack(">II", body[:8])
            assert body[8:10] == bytes([8, 6])
        elif t == b"IDAT":
            idat += body
        pos += 12 + n
    raw = zlib.decompress(idat)
    rows = [raw[i * (w * 4 + 1):(i + 1) * (w * 4 + 1)] for i in range(h)]
    assert all(r[0] == 0 for r in rows)
    return np.frombuffer(b"".join(r[1:] for r in rows), dtype=np.uint8).reshape(h, w, 4)


def test_png_and_pfm_round_trip(tmp_path):
    rng = np.random.default_rng(5)
    img = _frame(rng, 300, 260)  # > 65535 raw bytes: several stored blocks
    rgba8 = ptrace.tonemap(img)
    ptrace.write_png(tmp_path / "a.png", rgba8)
    back = _read_png(tmp_path / "a.png")
    assert np.array_equal(back[::-1], rgba8)  # PNG rows top-down, frame rows bottom-up
    ptrace.write_pfm(tmp_path / "a.pfm", img)
    raw = open(tmp_path / "a.pfm", "rb").read()
    head = b"PF\n260 300\n-1.0\n"
    assert raw.startswith(head)
    assert np.array_equal(np.frombuffer(raw[len(head):], dtype="<f4").reshape(300, 260, 3), img[..., :3])


@pytest.mark.gpu
def test_gpu_median_bit_exact(gpu_ctx):
    rng = np.random.default_rng(6)
    for h, w, nan in [(1, 1, False), (2, 3, False), (37, 53, True), (128, 96, True)]:
        img = _frame(rng, h, w, nan)
        g = gpu_ctx.median_filter(img)
        o = pyoracle.median(img)
        assert np.array_equal(g.view(np.uint32), o.view(np.uint32)), (h, w)


@pytest.mark.gpu
def test_display_image_threshold(gpu_ctx):
    sc = load_fixture("CBgems")
    gpu_ctx.load_scene(sc)
    gpu_ctx.clear()
    gpu_ctx.render(40, 24, 16, max_bounces=3)
    acc = gpu_ctx.get_image()
    disp = gpu_ctx.get_display_image()
    assert np.array_equal(disp, pyoracle.median(acc))  # < 32 spp: filtered
    gpu_ctx.render(40, 24, 16, max_bounces=3, sample_offset=16)
    assert np.array_equal(gpu_ctx.get_display_image(), gpu_ctx.get_image())  # 32 spp: accumulated image
