"""TPZ1 byte-plane codec: host C++ encoder/decoder vs the numpy spec decoder; checkpoints."""
import numpy as np
import pytest
import torch

from terraform_provider_iterative_amd.ops import codec
from reference_impls import tpz_decode_tile_py


def _float_streams():
    g = torch.Generator().manual_seed(0)
    return {
        "bf16_weights": torch.randn(200000, generator=g).mul(0.02).to(torch.bfloat16),
        "fp32_moment": torch.randn(100000, generator=g).mul(1e-3),
        "fp32_sq": torch.randn(100000, generator=g).mul(1e-3).pow(2),
        "zeros": torch.zeros(30000),
        "random": torch.randint(0, 256, (123456,), dtype=torch.uint8, generator=g),
        "few_values": torch.randint(0, 3, (50000,), dtype=torch.int32, generator=g),
    }


@pytest.mark.parametrize("tile", [4096, 8192, 1 << 20])
@pytest.mark.parametrize("name", list(_float_streams()))
def test_roundtrip_and_spec_decoder(name, tile):
    raw = _float_streams()[name].contiguous().view(-1).view(torch.uint8).numpy()
    raw = raw[:len(raw) // 16 * 16]
    enc, sizes = codec.encode(raw, tile)
    assert len(sizes) == -(-len(raw) // tile) and int(sizes.sum()) == len(enc)
    assert all(s % 16 == 0 for s in sizes)
    dec, first = codec.decode(enc, sizes, len(raw), tile)
    assert first == -1 and np.array_equal(dec, raw)
    offs = codec.offsets(sizes)
    for t in range(len(sizes)):
        blob = enc[int(offs[t]):int(offs[t + 1])].tobytes()
        lo = t * tile
        want = raw[lo:lo + tile]
        assert np.array_equal(tpz_decode_tile_py(blob, len(want)), want), t


def test_ratios_reflect_float_structure():
    s = _float_streams()
    ratio = {}
    for k in ("bf16_weights", "fp32_moment", "zeros", "random"):
        raw = s[k].view(torch.uint8).numpy()
        raw = raw[:len(raw) // 16 * 16]
        enc, _ = codec.encode(raw, 1 << 20)
        ratio[k] = len(enc) / len(raw)
    assert ratio["bf16_weights"] < 0.8
    assert ratio["fp32_moment"] < 0.9
    assert ratio["zeros"] < 0.01
    assert ratio["random"] < 1.01  # incompressible data costs only the 96-byte headers


def _modes(blob) -> list:
    return [int(blob[24 * p]) for p in range(4)]


def test_huffman_planes_code_float_exponents():
    # the sign/exponent byte of N(0, s) values carries ~2.6 bits: HUF (k=9) beats DICT(3)
    s = _float_streams()
    for name, limit in (("bf16_weights", 0.69), ("fp32_moment", 0.85), ("fp32_sq", 0.85)):
        raw = s[name].contiguous().view(-1).view(torch.uint8).numpy()
        raw = raw[:len(raw) // 16 * 16]
        enc, _ = codec.encode(raw, 1 << 20)
        assert len(enc) / len(raw) < limit, name
        assert 9 in _modes(enc), name


def test_huffman_escapes_roundtrip():
    # plane 3: geometric over ~40 values (dictionary misses -> inline escapes), plane 2: three
    # skewed values, planes 0-1: noise
    g = np.random.default_rng(5)
    n = 300000
    words = g.integers(0, 1 << 16, n, dtype=np.uint32)
    words |= np.minimum(g.geometric(0.25, n) - 1, 255).astype(np.uint32) << 24
    words |= g.choice(np.array([3, 7, 9], np.uint32), n, p=[0.7, 0.2, 0.1]) << 16
    raw = words.view(np.uint8)
    for tile in (4096, 65536, 1 << 18, 1 << 20):
        enc, sizes = codec.encode(raw, tile)
        dec, first = codec.decode(enc, sizes, len(raw), tile)
        assert first == -1 and np.array_equal(dec, raw), tile
        if tile >= 1 << 18:  # (small tiles may prefer DICT: substream index + word padding)
            assert _modes(enc)[3] == 9 and _modes(enc)[2] == 9, tile
        if tile == 1 << 18:
            blob = enc[:int(sizes[0])].tobytes()
            assert np.array_equal(tpz_decode_tile_py(blob, tile), raw[:tile])


def test_huffman_stream_overrun_is_reported():
    raw = _float_streams()["bf16_weights"].view(torch.uint8).numpy()
    enc, sizes = codec.encode(raw, 1 << 20)
    assert _modes(enc)[1] == 9
    bad = enc.copy()
    bad[24 + 4:24 + 8] = np.frombuffer(np.uint32(1).tobytes(), np.uint8)  # plane 1: 1 word
    _, first = codec.decode(bad, sizes, len(raw), 1 << 20)
    assert first == 0
    bad = enc.copy()
    sec1 = 96 + (len(raw) // 4 + 31) // 32 * 32  # plane 0 is RAW
    bad[sec1 + 16 + 4 * 200] ^= 0x04  # plane 1: a substream end offset moves
    _, first = codec.decode(bad, sizes, len(raw), 1 << 20)
    assert first == 0


def test_corrupt_blob_is_reported():
    raw = _float_streams()["bf16_weights"].view(torch.uint8).numpy()[:65536]
    enc, sizes = codec.encode(raw, 16384)
    bad = enc.copy()
    off = int(codec.offsets(sizes)[2])
    bad[off] = 7  # plane 0 mode byte of tile 2 -> invalid mode
    _, first = codec.decode(bad, sizes, len(raw), 16384)
    assert first == 2


def test_checkpointer_codec_roundtrip_host(tmp_path):
    from terraform_provider_iterative_amd.checkpoint import Checkpointer, describe_checkpoint

    src = {k: v.clone() for k, v in _float_streams().items()}
    ref = {k: v.clone() for k, v in src.items()}
    with Checkpointer(src, tile_bytes=8192, codec="tpz1") as ck:
        res = ck.save({"step": 1})
        assert ck.header()["codec"] == "tpz1"
        assert res.wire_bytes < res.bytes
        for v in src.values():
            v.zero_()
        ck.restore()
        path = ck.persist(str(tmp_path / "z.tpi"))
    assert all(torch.equal(src[k], ref[k]) for k in ref)
    info = describe_checkpoint(path)
    assert info["codec"] == "tpz1" and info["stream_bytes"] < info["total"]
    dst = {k: torch.zeros_like(v) for k, v in ref.items()}
    with Checkpointer(dst, tile_bytes=8192) as ck:  # a raw-configured reader loads it too
        ck.load(path)
    assert all(torch.equal(dst[k], ref[k]) for k in ref)


def test_leo_checkpoint_verify(tmp_path):
    import json
    import os
    import subprocess
    import sys

    from terraform_provider_iterative_amd.checkpoint import (Checkpointer, describe_checkpoint,
                                                             verify_checkpoint)

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    src = {k: v.clone() for k, v in _float_streams().items()}
    with Checkpointer(src, tile_bytes=8192, codec="tpz1") as ck:
        ck.save({"step": 4})
        path = ck.persist(str(tmp_path / "z.tpi"))
    assert verify_checkpoint(path)["bad_tiles"] == 0
    leo = [sys.executable, os.path.join(root, "bin", "leo")]
    out = subprocess.run(leo + ["checkpoint", "--verify", path], capture_output=True, text=True)
    assert out.returncode == 0, out.stderr
    info = json.loads(out.stdout)
    assert info["codec"] == "tpz1" and info["metadata"] == {"step": 4} and info["ratio"] < 1
    # flip a byte in the encoded stream -> the verifier names the tile
    off = describe_checkpoint(path)["stream_offset"] + 5000
    with open(path, "r+b") as f:
        f.seek(off)
        b = f.read(1)
        f.seek(off)
        f.write(bytes([b[0] ^ 0x40]))
    bad = verify_checkpoint(path)
    assert bad["bad_tiles"] >= 1 and bad["first_bad"] == 0
    out = subprocess.run(leo + ["checkpoint", "--verify", path], capture_output=True, text=True)
    assert out.returncode == 1
