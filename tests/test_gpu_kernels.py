"""HIP kernels vs host references (run on an MI355X: ``pytest -m gpu``)."""
import os
import numpy as np
import pytest
import torch

from terraform_provider_iterative_amd import ops
from terraform_provider_iterative_amd.ops.packing import PackPlan, crc_array, pack, unpack
from reference_impls import crc32c_py, shard_hash_py

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _require_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU visible")
    # The HIP library must load: a missing extension is a failure, not a skip.
    ops.hip(required=True)


def _rand_bytes(n, seed):
    return np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8)


@pytest.mark.parametrize("n,tile", [(16, 4096), (4096, 4096), (4096 * 5 + 48, 4096),
                                    (3 * (1 << 20), 1 << 20), ((1 << 20) + 4096 * 3 + 32, 1 << 20),
                                    (8192 * 7, 8192),
                                    # > 2 workgroups per CU of tile pairs: the grid-stride loop
                                    (4096 * 2101 + 16, 4096)])
def test_crc32c_tiles_device_matches_host(n, tile):
    data = _rand_bytes(n, n)
    dev = torch.from_numpy(data).cuda()
    got = crc_array(ops.crc32c_tiles(dev, tile_bytes=tile))
    want = ops.crc32c_tiles(data, tile_bytes=tile)
    assert got.tolist() == want.tolist()
    if n <= 3 * 4096:
        assert int(got[0]) == crc32c_py(data[:tile].tobytes())


@pytest.mark.parametrize("n,shard", [(100, 4096), (4096, 4096), (70000, 8192),
                                     ((1 << 20) * 3 + 77, 1 << 20), (5 * 8192 + 31, 8192)])
def test_shard_hash_device_matches_host(n, shard):
    data = _rand_bytes(n, n + 1)
    dev = torch.from_numpy(data).cuda()
    got = ops.shard_hash(dev, shard_bytes=shard, seed=11).cpu().numpy().view(np.uint64)
    host = ops.shard_hash(data, shard_bytes=shard, seed=11)
    assert got.tolist() == host.tolist()
    if n < 100000:
        assert host.tolist() == shard_hash_py(data.tobytes(), shard, seed=11).tolist()


def _tensors(device):
    g = torch.Generator().manual_seed(0)
    base = torch.randn(33, 17, generator=g)
    t = {
        "w": torch.randn(640, 480, generator=g).to(torch.bfloat16),
        "scalar": torch.tensor(3.5),
        "odd": torch.randint(0, 255, (100001,), dtype=torch.uint8, generator=g),
        "transposed": base.t(),
        "sliced": torch.randn(10, 20, 6, generator=g)[:, 3:17:2, 1:5],
        "empty": torch.zeros(0),
        "i64": torch.arange(-50, 77, dtype=torch.int64),
        "big": torch.randn(3 << 18, generator=g),  # 3 MiB
    }
    out = {}
    for k, v in t.items():
        if k == "transposed":
            out[k] = v.t().contiguous().to(device).t()
        elif k == "sliced":
            full = torch.zeros(10, 20, 6, device=device)
            full[:, 3:17:2, 1:5] = v.to(device)
            out[k] = full[:, 3:17:2, 1:5]
        else:
            out[k] = v.to(device)
    return out


def test_pack_device_matches_host_stream():
    dev = _tensors("cuda")
    host = {k: v.cpu() for k, v in dev.items()}
    pd = PackPlan.from_tensors(dev, tile_bytes=1 << 20)
    ph = PackPlan.from_tensors(host, tile_bytes=1 << 20)
    sd, cd = pack(pd)
    sh, ch = pack(ph)
    assert np.array_equal(sd.cpu().numpy(), sh)
    assert crc_array(cd).tolist() == ch.tolist()


def test_unpack_device_roundtrip_and_corruption():
    src = _tensors("cuda")
    plan = PackPlan.from_tensors(src, tile_bytes=1 << 20)
    stream, crcs = pack(plan)
    dst = {k: torch.zeros_like(v) for k, v in src.items()}
    dst["transposed"] = torch.zeros(33, 17, device="cuda").t()
    dst["sliced"] = torch.zeros(10, 20, 6, device="cuda")[:, 3:17:2, 1:5]
    plan.bind(dst)
    assert unpack(plan, stream, crcs) == (0, -1)
    for k in src:
        assert torch.equal(src[k], dst[k]), k
    stream[(1 << 20) + 12345] ^= 1
    bad, first = unpack(plan, stream, crcs)
    assert bad == 1 and first == 1


def test_incremental_sync_moves_only_dirty_tiles():
    from terraform_provider_iterative_amd.checkpoint import Checkpointer

    src = _tensors("cuda")
    tile = 1 << 20
    with Checkpointer(src, tile_bytes=tile, chunk_bytes=2 << 20, nbuf=2) as ck:
        first = ck.sync({"n": 1})
        assert first.dirty_tiles == ck.plan.ntiles
        again = ck.sync({"n": 2})
        assert again.dirty_tiles == 0 and again.bytes == 0
        # touch one element of "big" (3 MiB) -> exactly the tile holding it is dirty
        big = [e for e in ck.plan.entries if e.name == "big"][0]
        src["big"][100000] += 1.0
        touched_tile = (big.offset + 100000 * 4) // tile
        third = ck.sync({"n": 3})
        assert third.dirty_tiles == 1
        # the host region now equals a full pack of the current tensors
        hplan = PackPlan.from_tensors({k: v.cpu() for k, v in src.items()}, tile_bytes=tile)
        hs, hc = pack(hplan)
        assert np.array_equal(ck.region.array(ck.stream_offset, ck.plan.total), hs)
        assert ck.crcs.tolist() == hc.tolist()
        assert 0 <= touched_tile < ck.plan.ntiles
        # strided tensor change is detected too
        src["sliced"][0, 0, 0] = 42.0
        assert ck.sync().dirty_tiles == 1
        # restore round trip after syncs: the slot still holds what the tensors now hold, so
        # the next sync moves nothing; a full save rewrites the slot -> the sync after is full
        ref = {k: v.clone() for k, v in src.items()}
        for v in src.values():
            v.zero_()
        ck.restore()
        torch.cuda.synchronize()
        assert all(torch.equal(src[k], ref[k]) for k in ref)
        assert ck.sync().dirty_tiles == 0
        ck.save()
        assert ck.sync().dirty_tiles == ck.plan.ntiles


@pytest.mark.parametrize("mode", ["sdma", "direct"])
def test_checkpointer_device_roundtrip(mode, tmp_path):
    from terraform_provider_iterative_amd.checkpoint import Checkpointer

    src = _tensors("cuda")
    ref = {k: v.clone() for k, v in src.items()}
    with Checkpointer(src, tile_bytes=1 << 20, chunk_bytes=2 << 20, nbuf=2, mode=mode) as ck:
        res = ck.save({"step": 5})
        assert res.bytes == ck.plan.total
        # host copy matches a host-side pack of the same tensors
        hplan = PackPlan.from_tensors({k: v.cpu() for k, v in ref.items()}, tile_bytes=1 << 20)
        hs, hc = pack(hplan)
        assert np.array_equal(ck.region.array(ck.stream_offset, ck.plan.total), hs)
        assert ck.crcs.tolist() == hc.tolist()
        for v in src.values():
            v.zero_()
        out = ck.restore()
        assert out.bad_tiles == 0
        torch.cuda.synchronize()
        for k in ref:
            assert torch.equal(src[k], ref[k]), k
        path = ck.persist(str(tmp_path / "c.tpi"))
    dst = {k: torch.zeros_like(v) for k, v in ref.items()}
    with Checkpointer(dst, tile_bytes=1 << 20, chunk_bytes=2 << 20, mode=mode) as ck2:
        ck2.load(path)
        torch.cuda.synchronize()
    for k in ref:
        assert torch.equal(dst[k], ref[k]), k


@pytest.mark.parametrize("d2h", ["sdma", "blit"])
def test_d2h_engines_give_identical_checkpoints(d2h, monkeypatch):
    """Every D2H leg (save raw + TPZ1, incremental sync, async spill) through an SDMA engine
    (default) and through HIP's blit kernels (TPI_D2H_ENGINE=blit) lands the same bytes."""
    from terraform_provider_iterative_amd.checkpoint import Checkpointer

    if d2h == "blit":
        monkeypatch.setenv("TPI_D2H_ENGINE", "blit")
    else:
        monkeypatch.delenv("TPI_D2H_ENGINE", raising=False)
    src = _tensors("cuda")
    ref = {k: v.clone() for k, v in src.items()}
    hplan = PackPlan.from_tensors({k: v.cpu() for k, v in ref.items()}, tile_bytes=1 << 20)
    hs, hc = pack(hplan)
    # 1 MiB chunks, 2 buffers: staging buffers are reused several times per call
    with Checkpointer(src, tile_bytes=1 << 20, chunk_bytes=1 << 20, nbuf=2) as ck:
        assert ck.engine.d2h_engine.startswith(d2h)
        ck.save()
        assert np.array_equal(ck.region.array(ck.stream_offset, ck.plan.total), hs)
        assert ck.crcs.tolist() == hc.tolist()
        ck.sync()  # after a full save the slot's digests are unknown: a full sync
        assert ck.sync().dirty_tiles == 0
        keep = src["big"][300000].item()
        src["big"][300000] = keep + 1.0
        assert ck.sync().dirty_tiles == 1
        src["big"][300000] = keep
        assert ck.sync().dirty_tiles == 1
        assert np.array_equal(ck.region.array(ck.stream_offset, ck.plan.total), hs)
        ck.codec = "tpz1"
        ck.save()
        for v in src.values():
            v.zero_()
        assert ck.restore().bad_tiles == 0
        torch.cuda.synchronize()
        assert all(torch.equal(src[k], ref[k]) for k in ref)
        for codec in ("tpz1", "none"):
            ck.codec = codec
            ck.save_async().result()
            for v in src.values():
                v.zero_()
            assert ck.restore().bad_tiles == 0
            torch.cuda.synchronize()
            assert all(torch.equal(src[k], ref[k]) for k in ref), codec


def _geometric_exponents(n, g):
    """u32 words: noise low bytes, a 3-value byte 2 and a geometric byte 3 over ~40 values
    (Huffman planes with dictionary misses, i.e. inline escapes)."""
    words = torch.randint(0, 1 << 16, (n,), dtype=torch.int64, generator=g)
    u = torch.rand(n, generator=g, dtype=torch.float64)
    geo = torch.clamp((torch.log1p(-u) / np.log(0.75)).floor(), max=255).to(torch.int64)
    few = torch.tensor([3, 7, 9])[torch.multinomial(torch.tensor([0.7, 0.2, 0.1]), n, True,
                                                     generator=g)]
    return (words | (few << 16) | (geo << 24)).to(torch.int32).view(torch.uint8)


def _codec_inputs():
    g = torch.Generator().manual_seed(7)
    parts = [
        torch.randn(1 << 19, generator=g).mul(0.02).to(torch.bfloat16).view(torch.uint8),
        torch.randn(1 << 18, generator=g).mul(1e-3).view(torch.uint8),
        torch.randn(1 << 18, generator=g).mul(1e-3).pow(2).view(torch.uint8),
        torch.zeros(200000, dtype=torch.uint8),
        torch.randint(0, 256, (300016,), dtype=torch.uint8, generator=g),
        torch.randint(0, 5, (100000,), dtype=torch.int32, generator=g).view(torch.uint8),
        _geometric_exponents(1 << 18, g),
    ]
    raw = torch.cat([p.reshape(-1) for p in parts])
    return raw[:raw.numel() // 16 * 16 - 48]  # short final tile, length % 128 != 0


@pytest.mark.parametrize("tile", [4096, 65536, 1 << 20])
def test_tpz_device_encoder_is_bit_identical_to_host(tile):
    from terraform_provider_iterative_amd.ops import codec

    raw = _codec_inputs()
    host_blobs, host_sizes = codec.encode(raw.numpy(), tile)
    dev_blobs, dev_sizes = codec.encode(raw.cuda(), tile)
    assert dev_sizes.cpu().numpy().astype(np.uint32).tolist() == host_sizes.tolist()
    assert np.array_equal(dev_blobs.cpu().numpy(), host_blobs)
    # device decode of host blobs (and so of its own) restores the raw stream
    out, _ = codec.decode(torch.from_numpy(host_blobs).cuda(), host_sizes, raw.numel(), tile)
    assert torch.equal(out.cpu(), raw)


def test_tpz_device_decode_corrupt_blob_fails_crc():
    from terraform_provider_iterative_amd.ops import codec

    raw = _codec_inputs()[:1 << 20]
    blobs, sizes = codec.encode(raw.numpy(), 65536)
    bad = blobs.copy()
    bad[int(codec.offsets(sizes)[3])] = 7  # invalid plane mode in tile 3
    out, _ = codec.decode(torch.from_numpy(bad).cuda(), sizes, raw.numel(), 65536)
    got = crc_array(ops.crc32c_tiles(out, tile_bytes=65536)).tolist()
    want = ops.crc32c_tiles(raw.numpy(), tile_bytes=65536).tolist()
    assert [i for i, (a, b) in enumerate(zip(got, want)) if a != b] == [3]


def test_checkpointer_codec_device_roundtrip(tmp_path):
    from terraform_provider_iterative_amd.checkpoint import Checkpointer

    g = torch.Generator().manual_seed(3)
    src = {
        "w": torch.randn(3000, 1000, generator=g).mul(0.02).to(torch.bfloat16).cuda(),
        "m": torch.randn(1500, 1000, generator=g).mul(1e-3).cuda(),
        "v": torch.randn(1500, 1000, generator=g).mul(1e-3).pow(2).cuda(),
        "sliced": torch.randn(64, 96, generator=g).cuda()[:, 5:77:3],
        "odd": torch.randint(0, 255, (100001,), dtype=torch.uint8, generator=g).cuda(),
    }
    ref = {k: v.clone() for k, v in src.items()}
    with Checkpointer(src, tile_bytes=1 << 20, chunk_bytes=4 << 20, nbuf=2, codec="tpz1") as ck:
        res = ck.save({"step": 9})
        assert res.wire_bytes < 0.9 * res.bytes
        # host view of the region = host encoding of a host pack of the same tensors
        hplan = PackPlan.from_tensors({k: v.cpu() for k, v in ref.items()}, tile_bytes=1 << 20)
        hs, hc = pack(hplan)
        assert ck.crcs.tolist() == hc.tolist()
        from terraform_provider_iterative_amd.ops import codec

        hb, hsz = codec.encode(hs, 1 << 20)
        assert ck.csizes.tolist() == hsz.tolist()
        assert np.array_equal(ck.region.array(ck.stream_offset, len(hb)), hb)
        for v in src.values():
            v.zero_()
        out = ck.restore()
        torch.cuda.synchronize()
        assert out.bad_tiles == 0 and out.wire_bytes == res.wire_bytes
        assert all(torch.equal(src[k], ref[k]) for k in ref)
        path = ck.persist(str(tmp_path / "z.tpi"))
        # corrupt one escape/code byte in the region -> strict restore refuses
        ck.region.array(ck.stream_offset + 5000, 1)[0] ^= 0x5A
        with pytest.raises(Exception, match="corrupt"):
            ck.restore()
    dst = {k: torch.zeros_like(v) for k, v in ref.items()}
    dst["sliced"] = torch.zeros(64, 96, device="cuda")[:, 5:77:3]
    with Checkpointer(dst, tile_bytes=1 << 20, chunk_bytes=4 << 20) as ck2:  # codec-agnostic
        ck2.load(path)
        torch.cuda.synchronize()
    assert all(torch.equal(dst[k], ref[k]) for k in ref)


def _views(device):
    """Non-contiguous views of every kernel path (kind in the comment)."""
    g = torch.Generator().manual_seed(11)

    def r(*shape, dtype=torch.float32):
        return torch.randn(*shape, generator=g).to(dtype).to(device)

    return {
        "t_f32": r(300, 257).t(),                                   # TRANSPOSE 2-D
        "t_bf16": r(129, 1000, dtype=torch.bfloat16).t(),           # TRANSPOSE 2-D
        "t_u8": torch.randint(0, 255, (77, 333), dtype=torch.uint8, generator=g).to(device).t(),
        "t_f64": r(65, 70, dtype=torch.float64).t(),                # TRANSPOSE 2-D, 8-byte
        "batched": r(5, 40, 70).transpose(1, 2),                    # TRANSPOSE 3-D
        "channels_last": r(4, 16, 9, 9, dtype=torch.bfloat16)
        .contiguous(memory_format=torch.channels_last),             # TRANSPOSE 3-D (merged)
        "rows": r(100, 300)[:, 7:290],                              # ROWS, unaligned rows
        "rows_aligned": r(64, 512)[:, 64:448],                      # ROWS, vector path
        "stride2": r(100001)[::2],                                  # STRIDED
        "expanded": r(1, 50).expand(30, 50),                        # STRIDED (stride 0)
        "contig": r(1000),
    }


@pytest.mark.parametrize("tile", [4096, 1 << 20])
def test_view_kinds_pack_unpack_match_host(tile):
    dev = _views("cuda")
    host = {k: v.cpu() for k, v in dev.items()}
    pd = PackPlan.from_tensors(dev, tile_bytes=tile)
    ph = PackPlan.from_tensors(host, tile_bytes=tile)
    sd, cd = pack(pd)
    sh, ch = pack(ph)
    assert np.array_equal(sd.cpu().numpy(), sh)
    assert crc_array(cd).tolist() == ch.tolist()
    dst = {k: torch.empty_strided(v.shape, v.stride(), dtype=v.dtype, device=v.device).zero_()
           for k, v in dev.items()}  # same view structure (strides) as the sources
    pd.bind(dst)
    assert unpack(pd, sd, cd) == (0, -1)
    torch.cuda.synchronize()
    for k in dev:
        assert torch.equal(dst[k], dev[k]), k


@pytest.mark.parametrize("codec,mode", [("none", "sdma"), ("tpz1", "sdma"), ("none", "direct")])
def test_view_kinds_through_checkpointer_chunks(codec, mode):
    """Small chunks split the transposed views over many chunk windows (partial ranges)."""
    from terraform_provider_iterative_amd.checkpoint import Checkpointer

    src = _views("cuda")
    ref = {k: v.clone() for k, v in src.items()}
    with Checkpointer(src, tile_bytes=4096, chunk_bytes=16384, nbuf=2, mode=mode,
                      codec=codec) as ck:
        ck.save()
        hplan = PackPlan.from_tensors({k: v.cpu() for k, v in ref.items()}, tile_bytes=4096)
        hs, hc = pack(hplan)
        assert ck.crcs.tolist() == hc.tolist()
        for v in src.values():
            v.zero_()
        assert ck.restore().bad_tiles == 0
        torch.cuda.synchronize()
        for k in ref:
            assert torch.equal(src[k], ref[k]), k
        # incremental sync reads the views through the element path (no staging)
        src["t_f32"][3, 5] += 1
        assert ck.sync().dirty_tiles == ck.plan.ntiles
        src["batched"][1, 2, 3] += 1
        assert ck.sync().dirty_tiles == 1


@pytest.mark.parametrize("codec", ["none", "tpz1"])
def test_save_async_snapshots_before_later_updates(codec, tmp_path):
    """Tensors updated on the current stream right after save_async returns must not leak
    into the checkpoint: the snapshot is ordered before them on the device."""
    from terraform_provider_iterative_amd.checkpoint import Checkpointer

    src = _tensors("cuda")
    src.update({k: v for k, v in _views("cuda").items() if k.startswith("t_")})
    ref = {k: v.clone() for k, v in src.items()}
    kw = dict(tile_bytes=1 << 20, chunk_bytes=2 << 20, nbuf=2)
    with Checkpointer(src, codec=codec, **kw) as ck:
        pending = ck.save_async({"step": 11})
        for v in src.values():  # queued immediately on the same (current) stream
            v.add_(1) if v.dtype.is_floating_point else v.fill_(3)
        res = pending.result(timeout=120)
        assert res.bytes == ck.plan.total and ck.header()["metadata"] == {"step": 11}
        assert ck.header()["codec"] == codec
        path = ck.persist(str(tmp_path / "first.tpi"))
        # a second async save reuses the snapshot buffer (waits for the first spill)
        ck.save_async({"step": 12}).result(timeout=120)
        assert ck.header()["metadata"] == {"step": 12}
    dst = {k: torch.empty_strided(v.shape, v.stride(), dtype=v.dtype, device="cuda").zero_()
           for k, v in ref.items()}
    with Checkpointer(dst, **kw) as ck2:
        ck2.load(path)
        torch.cuda.synchronize()
    for k in ref:
        assert torch.equal(dst[k], ref[k]), k


def test_rollback_from_hbm_snapshot():
    from terraform_provider_iterative_amd.checkpoint import Checkpointer

    src = _tensors("cuda")
    src.update({k: v for k, v in _views("cuda").items() if k.startswith("t_")})
    ref = {k: v.clone() for k, v in src.items()}
    with Checkpointer(src, tile_bytes=1 << 20, chunk_bytes=2 << 20, codec="tpz1") as ck:
        ck.save_async().result(timeout=120)
        for v in src.values():
            v.zero_()
        res = ck.rollback()
        assert res.bad_tiles == 0 and res.wire_bytes == 0
        for k in ref:
            assert torch.equal(src[k], ref[k]), k


@pytest.mark.parametrize("codec", ["none", "tpz1"])
def test_streamed_restore_follows_the_writers_progress(codec, tmp_path):
    """Preemption hand-off on the device path: a successor restores a checkpoint that is
    still being published, chunk by chunk, and finishes only after the last chunk."""
    import threading
    import time

    from terraform_provider_iterative_amd.checkpoint import Checkpointer
    from terraform_provider_iterative_amd.checkpoint import checkpointer as ckmod

    g = torch.Generator().manual_seed(5)
    src = {"a": torch.randn(3 << 20, generator=g).to(torch.bfloat16).cuda(),
           "b": torch.randn(1 << 20, generator=g).mul(1e-3).cuda(),
           "t": torch.randn(640, 1000, generator=g).cuda().t()}
    path = str(tmp_path / "spill")
    kw = dict(tile_bytes=1 << 20, chunk_bytes=2 << 20, nbuf=2, codec=codec)
    writer = Checkpointer(src, path=path, **kw)
    words = np.zeros(2, dtype=np.uint64)  # the engine publishes here during this save
    writer.engine.set_progress(words.ctypes.data)
    res = writer.save({"step": 3})
    writer.engine.set_progress(0)
    assert int(words[0]) == writer.plan.ntiles and int(words[1]) == res.wire_bytes
    # turn the complete checkpoint back into one "being streamed": header + progress block
    slot = writer.slots[0]
    header = writer.header()
    header.update(complete=False, streaming=True)
    writer._write_header(slot, header)
    prog = slot.progress
    prog[1], prog[2], prog[3], prog[4] = header["generation"], 0, 0, ckmod.STREAM_RUNNING
    prog[5] = os.getpid()  # a live writer
    prog[0] = ckmod.PROGRESS_MAGIC
    dst = {k: torch.zeros_like(v) for k, v in src.items()}
    dst["t"] = torch.zeros(640, 1000, device="cuda").t()
    reader = Checkpointer(dst, path=path, **kw)
    assert reader.latest()["streaming"]
    out = {}

    def successor():
        t0 = time.perf_counter()
        out["res"] = reader.restore(stream_timeout=20)
        out["s"] = time.perf_counter() - t0

    th = threading.Thread(target=successor)
    th.start()
    per = writer.engine.chunk_bytes // writer.plan.tile_bytes
    steps = 0
    for tiles in range(per, writer.plan.ntiles + per, per):  # one chunk every 50 ms
        time.sleep(0.05)
        prog[2] = min(tiles, writer.plan.ntiles)
        steps += 1
    prog[4] = ckmod.STREAM_COMPLETE
    th.join(60)
    assert out["res"].bad_tiles == 0 and out["s"] >= 0.05 * (steps - 1)
    torch.cuda.synchronize()
    for k in src:
        assert torch.equal(dst[k], src[k]), k
    reader.close()
    writer.close()


@pytest.mark.parametrize("codec,split", [("none", "2"), ("tpz1", "2"), ("none", "0"),
                                         ("tpz1", "0")])
def test_restore_streams_behind_a_concurrent_save(codec, split, tmp_path, monkeypatch):
    """What bench.py's headline step does: a save streams into the host region while a
    restore in another thread copies each published chunk back into other tensors (the
    per-chunk CRC / blob-offset uploads on their own stream, staging slots reused).
    ``split`` = TPI_H2D_SPLIT_LEAD: 0 sends every chunk's H2D as two halves on two copy
    streams (the duplex-link balancing a trailing restore gets)."""
    import threading

    from terraform_provider_iterative_amd.checkpoint import Checkpointer

    monkeypatch.setenv("TPI_H2D_SPLIT_LEAD", split)
    g = torch.Generator().manual_seed(11)
    src = {"a": torch.randn(3 << 20, generator=g).to(torch.bfloat16).cuda(),
           "b": torch.randn(5 << 20, generator=g).mul(1e-3).cuda(),
           "t": torch.randn(640, 1000, generator=g).cuda().t()}
    dst = {k: torch.zeros_like(v) for k, v in src.items()}
    dst["t"] = torch.zeros(640, 1000, device="cuda").t()
    path = str(tmp_path / "spill")
    kw = dict(tile_bytes=1 << 16, chunk_bytes=1 << 20, nbuf=2, codec=codec)
    writer = Checkpointer(src, path=path, **kw)
    reader = Checkpointer(dst, path=path, **kw)
    for step in (1, 2):  # the second pass reuses every buffer of the first
        box = {}

        def restore():
            try:
                box["res"] = reader.restore(stream_timeout=20)
            except BaseException as error:  # surfaced below
                box["err"] = error

        th = threading.Thread(target=restore)
        writer.save({"step": step}, on_stream=th.start)
        th.join(60)
        assert "err" not in box, box.get("err")
        assert box["res"].bad_tiles == 0
        if split == "0":  # every chunk of at least 128 KiB on the wire went as two halves
            assert reader.engine.split_chunks > 0
        torch.cuda.synchronize()
        for k in src:
            assert torch.equal(dst[k], src[k]), (step, k)
        for v in src.values():
            v.mul_(-1)
        for v in dst.values():
            v.zero_()
    reader.close()
    writer.close()


def test_streamed_restore_gives_up_on_a_stalled_writer(tmp_path):
    from terraform_provider_iterative_amd.checkpoint import CheckpointError, Checkpointer
    from terraform_provider_iterative_amd.checkpoint import checkpointer as ckmod

    src = {"a": torch.randn(1 << 20, device="cuda")}
    path = str(tmp_path / "spill")
    writer = Checkpointer(src, path=path, tile_bytes=1 << 20, chunk_bytes=1 << 20)
    writer.save()
    slot = writer.slots[0]
    header = writer.header()
    header.update(complete=False, streaming=True)
    writer._write_header(slot, header)
    prog = slot.progress
    prog[1], prog[2], prog[4] = header["generation"], 0, ckmod.STREAM_RUNNING
    prog[5] = os.getpid()  # alive, but never makes progress
    prog[0] = ckmod.PROGRESS_MAGIC
    reader = Checkpointer({"a": torch.zeros(1 << 20, device="cuda")}, path=path,
                          tile_bytes=1 << 20, chunk_bytes=1 << 20)
    with pytest.raises(CheckpointError, match="stalled"):
        reader.restore(stream_timeout=0.3)
    prog[4] = ckmod.STREAM_FAILED
    with pytest.raises(CheckpointError):
        reader.restore(stream_timeout=5)
    # the writer dies while the successor waits for its chunks: the native wait notices the
    # exit within ~20 ms instead of sitting out the timeout
    import subprocess
    import sys
    import threading
    import time

    child = subprocess.Popen([sys.executable, "-c", "import time; time.sleep(0.5)"])
    prog[4], prog[5] = ckmod.STREAM_RUNNING, child.pid
    threading.Thread(target=child.wait, daemon=True).start()  # reaped: no zombie
    t0 = time.monotonic()
    with pytest.raises(CheckpointError, match="exited"):
        reader._restore_streaming(reader.slots[0], header, strict=True, timeout=30)
    assert time.monotonic() - t0 < 5
    reader.close()
    writer.close()


@pytest.mark.parametrize("digest,verify", [("xxh", "readback"), ("crc32c", "readback"),
                                           ("xxh", "inline")])
def test_handoff_copy_verify_catches_a_bad_destination(digest, verify, monkeypatch):
    """The hand-off's fused copy records a digest per tile of what it read; the read-back pass
    must flag tiles whose destination differs.  Two destination segments aliasing the same
    memory make the copy overwrite one tensor with another, as a wrong mapping would.  With
    TPI_HANDOFF_VERIFY=inline the copy reads every stored word back itself; aliasing
    destinations -- which an immediate read-back could miss -- fall back to the read-back
    pass, so the fault is still caught."""
    from terraform_provider_iterative_amd.checkpoint import Checkpointer
    from terraform_provider_iterative_amd.ops.packing import PackPlan

    monkeypatch.setenv("TPI_HANDOFF_HASH", digest)  # read by every tpi_copy_segments call
    monkeypatch.setenv("TPI_HANDOFF_VERIFY", verify)
    g = torch.Generator(device="cuda").manual_seed(5)
    src = {"a": torch.randn(1 << 20, device="cuda", generator=g),
           "b": torch.randn(1 << 20, device="cuda", generator=g).to(torch.bfloat16),
           "c": torch.randn(300, 1000, device="cuda", generator=g).t()}  # strided view
    dst = {"a": torch.zeros(1 << 20, device="cuda"),
           "b": torch.zeros(1 << 20, device="cuda", dtype=torch.bfloat16),
           "c": torch.zeros(300, 1000, device="cuda").t()}
    ck = Checkpointer(dst, tile_bytes=1 << 16, chunk_bytes=1 << 20, populate=False)
    src_segs = PackPlan.from_tensors(src, ck.plan.tile_bytes).segs.copy()
    stream = torch.cuda.current_stream().cuda_stream
    res = ck.engine.copy_segments(src_segs, ck.plan, stream)
    torch.cuda.synchronize()
    assert res.bad_tiles == 0
    for k in src:
        assert torch.equal(dst[k], src[k]), k
    ptr = ck.plan.segs["ptr"].copy()
    try:
        ck.plan.segs["ptr"][1] = ptr[0]  # "b" lands on top of "a"
        res = ck.engine.copy_segments(src_segs, ck.plan, stream)
        torch.cuda.synchronize()
    finally:
        ck.plan.segs["ptr"][:] = ptr
    assert res.bad_tiles > 0
    ck.close()


HBM_EXPORTER = r'''
import sys, torch
sys.path.insert(0, %(root)r)
from terraform_provider_iterative_amd.checkpoint import Checkpointer
g = torch.Generator(device="cuda").manual_seed(11)
t = {"a": torch.randn(5 << 20, device="cuda", generator=g).to(torch.bfloat16),
     "m": torch.randn(700, 900, device="cuda", generator=g).t(),
     "s": torch.randn(3000, device="cuda", generator=g)[::3]}
ck = Checkpointer(t, path=%(path)r, tile_bytes=1 << 20, chunk_bytes=4 << 20)
print("exported", ck.export_hbm(), flush=True)
sys.stdin.readline()  # hold the memory until the successor is done
'''


@pytest.mark.parametrize("route,hbm_route", [("fused", "auto"), ("staged", "auto"),
                                             ("fused", "ipc")])
def test_hbm_handoff_copies_a_live_predecessors_tensors(tmp_path, monkeypatch, route, hbm_route):
    """Same-GPU hand-off: the predecessor exports its tensors' allocations as HIP IPC handles
    (TPI_HBM_ROUTE auto or ipc); the
    successor copies them device to device, digest-verified, with no host copy.  The default
    copy is the fused tensor-to-tensor copy plus a read-back verify; TPI_HANDOFF_COPY=staged
    selects pack + unpack through a staging buffer.  Transposed and strided views take the
    element-wise path."""
    import subprocess
    import sys

    if route == "staged":
        monkeypatch.setenv("TPI_HANDOFF_COPY", "staged")
    monkeypatch.setenv("TPI_HBM_ROUTE", hbm_route)

    root = __import__("os").path.dirname(__import__("os").path.dirname(__file__))
    path = str(tmp_path / "spill")
    child = subprocess.Popen([sys.executable, "-c", HBM_EXPORTER % {"root": root, "path": path}],
                             stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
    try:
        line = child.stdout.readline()
        assert line.startswith("exported"), line
        g = torch.Generator(device="cuda").manual_seed(11)
        want = {"a": torch.randn(5 << 20, device="cuda", generator=g).to(torch.bfloat16),
                "m": torch.randn(700, 900, device="cuda", generator=g).t(),
                "s": torch.randn(3000, device="cuda", generator=g)[::3]}
        dst = {"a": torch.zeros(5 << 20, device="cuda", dtype=torch.bfloat16),
               "m": torch.zeros(700, 900, device="cuda").t(),
               "s": torch.zeros(3000, device="cuda")[::3]}
        from terraform_provider_iterative_amd.checkpoint import Checkpointer

        ck = Checkpointer(dst, path=path, tile_bytes=1 << 20, chunk_bytes=4 << 20)
        assert ck.hbm_ready()
        res = ck.restore_hbm()
        torch.cuda.synchronize()
        assert res.bad_tiles == 0
        for k in want:
            assert torch.equal(dst[k], want[k]), k
        assert not ck.hbm_ready()  # consumed
        ck.close()
    finally:
        child.stdin.write("\n")
        child.stdin.flush()
        child.wait(60)


BIG_EXPORTER = r'''
import sys, torch
sys.path.insert(0, %(root)r)
from terraform_provider_iterative_amd.checkpoint import Checkpointer
g = torch.Generator(device="cuda").manual_seed(5)
t = {"emb": torch.empty(int(4.2 * 2 ** 30) // 4, device="cuda"),
     "w": torch.empty(int(2.5 * 2 ** 30) // 2, device="cuda", dtype=torch.bfloat16),
     "n": torch.randn(4096, device="cuda", generator=g)}
t["emb"].normal_(generator=g)
t["w"].normal_(generator=g)
ck = Checkpointer(t, path=%(path)r, tile_bytes=1 << 20, chunk_bytes=256 << 20)
print("exported", ck.export_hbm(), flush=True)
sys.stdin.readline()  # hold the memory until the successor is done
'''


def test_hbm_handoff_of_allocations_beyond_the_ipc_limit(tmp_path, monkeypatch):
    """a state holding 4.2 GiB and 2.5 GiB tensors -- the fp32 embedding / Adam
    moments of a large vocabulary -- hands off device to device, bit-exact: HIP IPC imports of
    such allocations never return (profiles/round5/ipc_cause.md), so the exporter relocates
    those tensors into 1 GiB blocks that travel over HIP IPC (TPI_HBM_ROUTE=auto)."""
    import os
    import subprocess
    import sys

    monkeypatch.setenv("TPI_HBM_ROUTE", "auto")
    monkeypatch.setenv("TPI_IPC_OPEN_TIMEOUT", "30")
    root = os.path.dirname(os.path.dirname(__file__))
    path = str(tmp_path / "spill")
    child = subprocess.Popen([sys.executable, "-c", BIG_EXPORTER % {"root": root, "path": path}],
                             stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
    try:
        line = child.stdout.readline()
        assert line.startswith("exported"), line
        with open(path + ".hbm") as f:
            doc = __import__("json").load(f)
        # auto route: the two big tensors relocated into <= 1 GiB blocks, all over HIP IPC
        assert sorted(len(p) for p in doc["pieces"].values()) == [3, 5], doc["pieces"]
        assert max(doc["allocations"]) <= 1 << 30 and "socket" not in doc
        dst = {"emb": torch.zeros(int(4.2 * 2 ** 30) // 4, device="cuda"),
               "w": torch.zeros(int(2.5 * 2 ** 30) // 2, device="cuda", dtype=torch.bfloat16),
               "n": torch.zeros(4096, device="cuda")}
        from terraform_provider_iterative_amd.checkpoint import Checkpointer

        ck = Checkpointer(dst, path=path, tile_bytes=1 << 20, chunk_bytes=256 << 20)
        assert ck.hbm_ready()
        res = ck.restore_hbm()
        torch.cuda.synchronize()
        assert res.bad_tiles == 0
        ck.wait_hbm_close()
        g = torch.Generator(device="cuda").manual_seed(5)  # the exporter's draw order
        assert torch.equal(dst["n"], torch.randn(4096, device="cuda", generator=g))
        want = torch.empty(int(4.2 * 2 ** 30) // 4, device="cuda")
        want.normal_(generator=g)
        assert torch.equal(dst["emb"], want)
        del want
        w = torch.empty(int(2.5 * 2 ** 30) // 2, device="cuda", dtype=torch.bfloat16)
        w.normal_(generator=g)
        assert torch.equal(dst["w"], w)
        del w
        ck.close()
    finally:
        child.stdin.write("\n")
        child.stdin.flush()
        child.wait(60)


def test_hbm_export_refuses_allocations_at_the_ipc_limit(tmp_path, monkeypatch):
    """The IPC route (TPI_HBM_ROUTE=ipc): imports of allocations of 2 GiB or more never return
    in hipIpcOpenMemHandle (profiles/round5/ipc_cause.md), so export_hbm refuses a state holding
    one before it publishes anything: the successor sees no hand-off and restores from the host
    copy.  The limit is lowered here so that small tensors exercise it."""
    from terraform_provider_iterative_amd.checkpoint import CheckpointError, Checkpointer
    from terraform_provider_iterative_amd.checkpoint import checkpointer as ckmod

    import ctypes

    from terraform_provider_iterative_amd.ops import hip

    monkeypatch.setenv("TPI_HBM_ROUTE", "ipc")
    assert ckmod.IPC_MAX_ALLOC == 2 << 30
    t = {"a": torch.randn(1 << 18, device="cuda"), "b": torch.randn(4 << 20, device="cuda")}
    base, size = ctypes.c_uint64(0), ctypes.c_uint64(0)
    largest = 0  # the caching allocator decides which allocations hold them
    for v in t.values():
        hip().check(hip().tpi_mem_range(ctypes.c_void_p(v.data_ptr()), ctypes.byref(base),
                                        ctypes.byref(size)), "tpi_mem_range")
        largest = max(largest, int(size.value))
    ck = Checkpointer(t, path=str(tmp_path / "spill"), tile_bytes=1 << 20, chunk_bytes=4 << 20)
    monkeypatch.setenv("TPI_IPC_MAX_ALLOC", str(largest))
    with pytest.raises(CheckpointError, match="no HBM hand-off"):
        ck.export_hbm()
    assert not __import__("os").path.exists(str(tmp_path / "spill") + ".hbm")
    monkeypatch.setenv("TPI_IPC_MAX_ALLOC", str(largest + 1))
    assert ck.export_hbm()
    ck.close()


def test_prewarmed_engine_is_taken_by_the_next_checkpointer():
    """A warm standby pre-creates the device engine (preemption.standby -> prewarm_engine);
    the Checkpointer built after activation takes it instead of creating one."""
    from terraform_provider_iterative_amd.checkpoint import Checkpointer, prewarm_engine
    from terraform_provider_iterative_amd.checkpoint import engine as engmod

    assert prewarm_engine(torch.cuda.current_device(), chunk_bytes=4 << 20, nbuf=2,
                          tile_bytes=1 << 20)
    key = (torch.cuda.current_device(), 4 << 20, 2, 1 << 20)
    pooled = engmod._engine_pool[key][-1]
    t = {"a": torch.randn(3 << 20, device="cuda")}
    ck = Checkpointer(t, chunk_bytes=4 << 20, nbuf=2)
    assert ck.engine is pooled and not engmod._engine_pool.get(key)
    want = t["a"].clone()
    ck.save()
    t["a"].zero_()
    ck.restore()
    assert torch.equal(t["a"], want)
    ck.close()


@pytest.mark.parametrize("codec", ["none", "tpz1"])
def test_materialize_streams_groups_behind_a_writer(codec, tmp_path):
    """Checkpointer.materialize() on the GPU: while the writer publishes its stream chunk by
    chunk, a successor thread allocates and restores the state group by group
    (tpi_restore_stream_at: each group waits for its own tiles of the whole stream); then
    once more from the complete copy, one tensor per group."""
    import threading
    import time

    from terraform_provider_iterative_amd.checkpoint import Checkpointer
    from terraform_provider_iterative_amd.checkpoint import checkpointer as ckmod

    g = torch.Generator().manual_seed(12)
    src = {"a": torch.randn(3 << 20, generator=g).to(torch.bfloat16).cuda(),
           "b": torch.randn(5 << 20, generator=g).mul(1e-3).cuda(),
           "t": torch.randn(640, 1000, generator=g).cuda().t(),
           "c": torch.randn(777_777, generator=g).cuda(),
           "d": torch.randint(0, 1 << 30, (2 << 20,), generator=g).cuda()}
    path = str(tmp_path / "spill")
    kw = dict(tile_bytes=1 << 16, chunk_bytes=1 << 20, nbuf=2, codec=codec)
    writer = Checkpointer(src, path=path, **kw)
    writer.save({"step": 2})
    # turn the complete checkpoint back into one "being streamed" (as in
    # test_streamed_restore_follows_the_writers_progress), published below chunk by chunk
    slot = writer.slots[0]
    header = writer.header()
    header.update(complete=False, streaming=True)
    writer._write_header(slot, header)
    prog = slot.progress
    prog[1], prog[2], prog[3], prog[4] = header["generation"], 0, 0, ckmod.STREAM_RUNNING
    prog[5] = os.getpid()
    prog[0] = ckmod.PROGRESS_MAGIC
    box = {}

    def successor():
        try:
            box["out"] = Checkpointer.materialize(path, "cuda", group_bytes=6 << 20,
                                                  stream_timeout=20, chunk_bytes=1 << 20, nbuf=2)
        except BaseException as error:  # surfaced below
            box["err"] = error

    th = threading.Thread(target=successor)
    th.start()
    per = 16  # tiles (1 MiB) per publication, every 20 ms
    for tiles in range(per, writer.plan.ntiles + per, per):
        time.sleep(0.02)
        prog[2] = min(tiles, writer.plan.ntiles)
    header.update(complete=True, streaming=False)
    writer._write_header(slot, header)
    prog[4] = ckmod.STREAM_COMPLETE
    th.join(60)
    assert "err" not in box, box.get("err")
    ck, tensors, res = box["out"]
    assert res.bad_tiles == 0 and ck.materialize_stats["streamed"]
    assert ck.materialize_stats["groups"] >= 3 and ck.materialized_metadata["step"] == 2
    torch.cuda.synchronize()
    for k in src:
        assert tensors[k].is_cuda and torch.equal(tensors[k], src[k]), k
    ck.close()
    ck2, tensors2, _ = Checkpointer.materialize(path, "cuda", group_bytes=1,
                                                chunk_bytes=1 << 20, nbuf=2)
    assert not ck2.materialize_stats["streamed"] and ck2.materialize_stats["groups"] == len(src)
    for k in src:
        assert torch.equal(tensors2[k], src[k]), k
    ck2.close()
    writer.close()


def test_direct_metadata_modes_give_identical_checkpoints(tmp_path):
    """TPI_DIRECT_META (read once per process): the streamed save's kernels store tile CRCs
    and blob sizes straight in the host region, the streamed restore's kernels read CRCs and
    blob offsets from host memory -- or both sides use per-chunk copies.  Every mode must write
    the same region and restore the same bytes."""
    import hashlib
    import subprocess
    import sys

    script = r'''
import hashlib, json, sys, threading, torch
sys.path.insert(0, %r)
from terraform_provider_iterative_amd.checkpoint import Checkpointer
g = torch.Generator().manual_seed(21)
src = {"a": torch.randn(3 << 20, generator=g).to(torch.bfloat16).cuda(),
       "b": torch.randn(5 << 20, generator=g).mul(1e-3).cuda(),
       "t": torch.randn(640, 1000, generator=g).cuda().t()}
dst = {k: torch.zeros_like(v) for k, v in src.items()}
dst["t"] = torch.zeros(640, 1000, device="cuda").t()
out = {}
for codec in ("none", "tpz1"):
    path = sys.argv[1] + "." + codec
    kw = dict(tile_bytes=1 << 16, chunk_bytes=1 << 20, nbuf=2, codec=codec)
    writer, reader = Checkpointer(src, path=path, **kw), Checkpointer(dst, path=path, **kw)
    box = {}
    th = threading.Thread(target=lambda: box.update(res=reader.restore(stream_timeout=20)))
    writer.save({"step": 1}, on_stream=th.start)
    th.join(60)
    torch.cuda.synchronize()
    assert box["res"].bad_tiles == 0
    assert all(torch.equal(dst[k], src[k]) for k in src)
    slot = writer.slots[0]
    out[codec] = hashlib.sha256(slot.crcs.tobytes() + slot.csizes.tobytes()).hexdigest()
    for v in dst.values():
        v.zero_()
    reader.close()
    writer.close()
print(json.dumps(out))
''' % os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    seen = {}
    for mode in ("0", "save", "restore", "1"):
        env = dict(os.environ, TPI_DIRECT_META=mode)
        proc = subprocess.run([sys.executable, "-c", script, str(tmp_path / ("r" + mode))],
                              env=env, capture_output=True, text=True, timeout=180)
        assert proc.returncode == 0, (mode, proc.stderr[-2000:])
        seen[mode] = proc.stdout.strip().splitlines()[-1]
    assert len(set(seen.values())) == 1, seen


def test_materialize_falls_back_when_the_writers_stream_fails(tmp_path):
    """Device path: the predecessor's streamed save of generation 2 fails after publishing
    some tiles; materialize() re-restores every group from generation 1, the complete copy a
    two-slot region still holds, so the state is one generation throughout."""
    import threading
    import time

    from terraform_provider_iterative_amd.checkpoint import Checkpointer
    from terraform_provider_iterative_amd.checkpoint import checkpointer as ckmod

    g = torch.Generator().manual_seed(13)
    src = {"a": torch.randn(3 << 20, generator=g).cuda(),
           "b": torch.randn(5 << 20, generator=g).to(torch.bfloat16).cuda()}
    ref = {k: v.clone() for k, v in src.items()}
    path = str(tmp_path / "spill")
    kw = dict(tile_bytes=1 << 16, chunk_bytes=1 << 20, nbuf=2, codec="tpz1", slots=2)
    writer = Checkpointer(src, path=path, **kw)
    writer.save({"step": 1})  # generation 1, complete
    for v in src.values():
        v.mul_(-1)
    writer.save({"step": 2})  # generation 2 ...
    slot, header = writer._active()
    header.update(complete=False, streaming=True)  # ... turned back into a stream
    writer._write_header(slot, header)
    prog = slot.progress
    prog[1], prog[2], prog[3], prog[4] = header["generation"], 0, 0, ckmod.STREAM_RUNNING
    prog[5] = os.getpid()
    prog[0] = ckmod.PROGRESS_MAGIC
    box = {}

    def successor():
        try:
            box["out"] = Checkpointer.materialize(path, "cuda", group_bytes=4 << 20,
                                                  stream_timeout=20, chunk_bytes=1 << 20, nbuf=2)
        except BaseException as error:  # surfaced below
            box["err"] = error

    th = threading.Thread(target=successor)
    th.start()
    time.sleep(0.2)
    prog[2] = 40  # some tiles of generation 2 arrive, then the writer fails
    time.sleep(0.2)
    prog[4] = ckmod.STREAM_FAILED
    th.join(60)
    assert "err" not in box, box.get("err")
    ck, tensors, res = box["out"]
    assert res.bad_tiles == 0 and ck.materialized_metadata["step"] == 1
    assert ck.materialize_stats["fallback"]
    torch.cuda.synchronize()
    for k in ref:
        assert torch.equal(tensors[k], ref[k]), k
    ck.close()
    writer.close()


@pytest.mark.parametrize("codec", ["none", "tpz1"])
def test_streamed_restore_on_its_own_sdma_engine(codec, tmp_path):
    """tpi_engine_set_h2d_sdma: a restore streaming behind a concurrent save copies host ->
    device on an SDMA engine of its own (host-driven lanes, kernels queued per landed chunk),
    for every staging buffer reused twice; the bytes match."""
    import threading

    from terraform_provider_iterative_amd.checkpoint import Checkpointer

    g = torch.Generator().manual_seed(14)
    src = {"a": torch.randn(3 << 20, generator=g).to(torch.bfloat16).cuda(),
           "b": torch.randn(5 << 20, generator=g).mul(1e-3).cuda(),
           "t": torch.randn(640, 1000, generator=g).cuda().t()}
    dst = {k: torch.zeros_like(v) for k, v in src.items()}
    dst["t"] = torch.zeros(640, 1000, device="cuda").t()
    path = str(tmp_path / "spill")
    kw = dict(tile_bytes=1 << 16, chunk_bytes=1 << 20, nbuf=2, codec=codec)
    writer = Checkpointer(src, path=path, **kw)
    reader = Checkpointer(dst, path=path, **kw)
    engine = reader.engine.set_h2d_sdma(True)
    if engine < 0:
        pytest.skip("no free SDMA engine for host-to-device lanes on this device")
    box = {}

    def restore():
        try:
            box["res"] = reader.restore(stream_timeout=20)
        except BaseException as error:  # surfaced below
            box["err"] = error

    th = threading.Thread(target=restore)
    writer.save({"step": 1}, on_stream=th.start)
    th.join(60)
    assert "err" not in box, box.get("err")
    assert box["res"].bad_tiles == 0
    torch.cuda.synchronize()
    for k in src:
        assert torch.equal(dst[k], src[k]), k
    assert reader.engine.set_h2d_sdma(False) == 0
    reader.close()
    writer.close()


STUCK_EXPORTER = r'''
import sys, torch
sys.path.insert(0, %(root)r)
from terraform_provider_iterative_amd.checkpoint import Checkpointer
g = torch.Generator(device="cuda").manual_seed(23)
t = {"big": torch.empty(int(2.1 * 2 ** 30) // 4, device="cuda"),
     "n": torch.randn(4096, device="cuda", generator=g)}
t["big"].normal_(generator=g)
ck = Checkpointer(t, path=%(path)r, tile_bytes=1 << 20, chunk_bytes=256 << 20)
ck.save({"step": 7})  # the host copy the successor falls back to
print("exported", ck.export_hbm({"step": 7}), flush=True)
sys.stdin.readline()  # hold the memory (and the offer) until the successor is done
'''

STUCK_SUCCESSOR = r'''
import os, sys, threading, time, torch
sys.path.insert(0, %(root)r)
from terraform_provider_iterative_amd.checkpoint import Checkpointer, preemption
g = torch.Generator(device="cuda").manual_seed(23)  # the exporter's draw order: n, then big
want_n = torch.randn(4096, device="cuda", generator=g)
want_big = torch.empty(int(2.1 * 2 ** 30) // 4, device="cuda")
want_big.normal_(generator=g)
dst = {"big": torch.zeros_like(want_big), "n": torch.zeros(4096, device="cuda")}
ck = Checkpointer(dst, path=%(path)r, tile_bytes=1 << 20, chunk_bytes=256 << 20)
assert ck.hbm_ready()
t0 = time.monotonic()
meta = preemption.resume(ck)
took = time.monotonic() - t0
torch.cuda.synchronize()
ok = torch.equal(dst["big"], want_big) and torch.equal(dst["n"], want_n)
stuck = [t.name for t in threading.enumerate() if t.name == "tpi-ipc-open" and t.is_alive()]
print("resumed", meta.get("step"), "took %%.2f" %% took, "bitexact", ok, "stuck", len(stuck),
      flush=True)
ck.close()
sys.exit(0 if ok else 3)
'''


def test_a_stuck_ipc_import_falls_back_to_the_host_copy_on_hardware(tmp_path):
    """VERDICT r5 #6, on the real driver: an IPC import that never returns (a 2.1 GiB
    allocation offered over HIP IPC with the size guard lifted, TPI_HBM_ROUTE=ipc and
    TPI_IPC_MAX_ALLOC=3 GiB) makes the successor give up after TPI_IPC_OPEN_TIMEOUT, restore
    bit-exactly from the host copy, and exit normally with the opener thread still stuck in
    the driver.  The successor is a child process, so a stuck runtime cannot take the test
    runner with it."""
    import os
    import subprocess
    import sys
    import time

    root = os.path.dirname(os.path.dirname(__file__))
    path = str(tmp_path / "spill")
    env = dict(os.environ, TPI_HBM_ROUTE="ipc", TPI_IPC_MAX_ALLOC=str(3 << 30),
               TPI_IPC_OPEN_TIMEOUT="4", TPI_EVENTS_FILE=str(tmp_path / "events.jsonl"))
    child = subprocess.Popen([sys.executable, "-c", STUCK_EXPORTER % {"root": root, "path": path}],
                             stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True, env=env)
    try:
        line = child.stdout.readline()
        assert line.startswith("exported"), line
        t0 = time.monotonic()
        succ = subprocess.run([sys.executable, "-c", STUCK_SUCCESSOR % {"root": root,
                                                                        "path": path}],
                              env=env, capture_output=True, text=True, timeout=100)
        wall = time.monotonic() - t0
    finally:
        child.stdin.write("\n")
        child.stdin.flush()
        child.wait(60)
    out = succ.stdout + succ.stderr
    assert succ.returncode == 0, out[-3000:]
    assert "resumed 7" in out and "bitexact True" in out, out[-3000:]
    took = float(out.split("took ")[1].split()[0])
    assert 3.5 <= took < 30, out[-2000:]  # gave up at the timeout, then the host restore
    events = open(tmp_path / "events.jsonl").read()
    assert "checkpoint-hbm-failed" in events and "TPI_IPC_OPEN_TIMEOUT" in events
    assert '"checkpoint-restored", "description": ["rank 0", "host region"' in events
    print("stuck-import fallback: resume %.2f s, successor wall %.2f s, %s" % (
        took, wall, out.split("stuck ")[1].split()[0] + " opener(s) still stuck at exit"))


def test_a_lite_engine_holds_no_staging_until_a_pipeline_needs_it(tmp_path):
    """A parked successor's prewarmed engine (``DeviceEngine(lite=True)``, the default
    preload's warm-up) leaves its HBM staging ring to the first pipeline that moves data
    through it: the hand-off copy runs without it, a host save allocates it then and is exact."""
    import numpy as np

    from terraform_provider_iterative_amd.checkpoint import Checkpointer
    from terraform_provider_iterative_amd.checkpoint.engine import MODES, DeviceEngine
    from terraform_provider_iterative_amd.checkpoint.host import HostRegion
    from terraform_provider_iterative_amd.ops.packing import PackPlan

    torch.cuda.synchronize()
    chunk, nbuf = 256 << 20, 3
    free0 = torch.cuda.mem_get_info()[0]
    full = DeviceEngine(0, chunk, nbuf, 1 << 20)
    free1 = torch.cuda.mem_get_info()[0]
    lite = DeviceEngine(0, chunk, nbuf, 1 << 20, lite=True)
    free2 = torch.cuda.mem_get_info()[0]
    assert free0 - free1 >= nbuf * chunk  # the full engine's ring
    assert free1 - free2 < chunk  # the lite one: streams, events, tables
    g = torch.Generator(device="cuda").manual_seed(3)
    src = {"a": torch.randn(3 << 20, device="cuda", generator=g),
           "t": torch.randn(300, 700, device="cuda", generator=g).t()}
    dst = {"a": torch.zeros(3 << 20, device="cuda"), "t": torch.zeros(300, 700, device="cuda").t()}
    plan = PackPlan.from_tensors(src, 1 << 20)
    sig = torch.cuda.current_stream().cuda_stream
    res = lite.copy_segments(plan.segs.copy(), PackPlan.from_tensors(dst, 1 << 20), sig)
    torch.cuda.synchronize()
    assert res.bad_tiles == 0 and all(torch.equal(dst[k], src[k]) for k in src)
    assert torch.cuda.mem_get_info()[0] > free2 - chunk  # still no ring
    region = HostRegion((plan.total + (2 << 20)) // 4096 * 4096, device=True, populate=True)
    try:
        crcs = np.zeros(plan.ntiles, np.uint32)
        lite.save(plan, region.addr, crcs, MODES["sdma"], sig)  # allocates the ring now
        for v in dst.values():
            v.zero_()
        lite.restore(PackPlan.from_tensors(dst, 1 << 20), region.addr, crcs, MODES["sdma"], sig)
        torch.cuda.synchronize()
        assert all(torch.equal(dst[k], src[k]) for k in src)
    finally:
        region.close()
        lite.close()
        full.close()
