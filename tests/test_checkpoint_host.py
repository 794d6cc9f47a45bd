"""Checkpointer on CPU tensors (host C++ path): save/restore/persist/load/corruption."""
import os
import time

import numpy as np
import pytest
import torch

from terraform_provider_iterative_amd.checkpoint import (CheckpointError, Checkpointer,
                                                         describe_checkpoint)


def _model(seed=0):
    g = torch.Generator().manual_seed(seed)
    return {
        "embed": torch.randn(300, 64, generator=g).to(torch.bfloat16),
        "w1": torch.randn(64, 256, generator=g),
        "b1": torch.randn(256, generator=g),
        "step": torch.tensor(17, dtype=torch.int64),
        "view": torch.randn(40, 30, generator=g).t(),
    }


def test_save_restore_anonymous():
    src = _model()
    ref = {k: v.clone() for k, v in src.items()}
    with Checkpointer(src, tile_bytes=8192) as ck:
        res = ck.save({"step": 17})
        assert res.bytes == ck.plan.total and res.crc != 0
        for v in src.values():
            v.zero_()
        out = ck.restore()
        assert out.bad_tiles == 0
        assert ck.header()["metadata"] == {"step": 17}
    for k in ref:
        assert torch.equal(src[k], ref[k]), k


def test_shared_file_survives_object(tmp_path):
    path = str(tmp_path / "spill.bin")
    src = _model(1)
    ref = {k: v.clone() for k, v in src.items()}
    with Checkpointer(src, path=path, tile_bytes=4096) as ck:
        ck.save({"epoch": 3})
    fresh = {k: torch.zeros_like(v) for k, v in ref.items()}
    fresh["view"] = torch.zeros(40, 30).t()
    with Checkpointer(fresh, path=path, tile_bytes=4096) as ck2:
        ck2.restore()
        assert ck2.header()["metadata"]["epoch"] == 3
    for k in ref:
        assert torch.equal(fresh[k], ref[k]), k


def test_persist_load_and_corruption(tmp_path):
    src = _model(2)
    with Checkpointer(src, tile_bytes=4096) as ck:
        ck.save()
        path = ck.persist(str(tmp_path / "ckpt.tpi"))
    info = describe_checkpoint(path)
    assert info["complete"] and info["total"] > 0
    dst = {k: torch.zeros_like(v) for k, v in src.items()}
    dst["view"] = torch.zeros(40, 30).t()
    with Checkpointer(dst, tile_bytes=4096) as ck:
        ck.load(path)
    assert all(torch.equal(dst[k], src[k]) for k in src)
    # flip one payload byte on disk -> strict restore refuses
    with open(path, "r+b") as f:
        f.seek(info["stream_offset"] + 100)
        b = f.read(1)
        f.seek(info["stream_offset"] + 100)
        f.write(bytes([b[0] ^ 1]))
    with Checkpointer(dst, tile_bytes=4096) as ck:
        with pytest.raises(CheckpointError, match="corrupt"):
            ck.load(path)


def test_sync_on_host_is_full_save():
    src = _model(4)
    with Checkpointer(src, tile_bytes=4096) as ck:
        res = ck.sync({"k": 1})
        assert res.dirty_tiles == ck.plan.ntiles
        assert ck.header()["complete"] and ck.header()["metadata"] == {"k": 1}


def test_incomplete_save_is_rejected(tmp_path):
    src = _model(3)
    with Checkpointer(src, tile_bytes=4096) as ck:
        with pytest.raises(CheckpointError):
            ck.restore()


def test_layout_mismatch(tmp_path):
    path = str(tmp_path / "spill.bin")
    with Checkpointer(_model(), path=path, tile_bytes=4096) as ck:
        ck.save()
    other = {"x": torch.zeros(10)}
    with Checkpointer(other, path=path, tile_bytes=4096) as ck:
        with pytest.raises(CheckpointError):
            ck.restore()
    assert os.path.getsize(path) > 0
    assert np.uint32  # keep numpy import used


def test_save_async_on_host_falls_back_to_sync():
    src = _model(5)
    ref = {k: v.clone() for k, v in src.items()}
    with Checkpointer(src, tile_bytes=4096) as ck:
        pending = ck.save_async({"step": 2})
        res = pending.result(timeout=30)
        assert pending.done() and res.bytes == ck.plan.total
        assert ck.header()["complete"] and ck.header()["metadata"] == {"step": 2}
        for v in src.values():
            v.zero_()
        ck.restore()
    for k in ref:
        assert torch.equal(src[k], ref[k]), k


def test_two_slots_keep_the_previous_checkpoint_through_a_failed_save(monkeypatch):
    from terraform_provider_iterative_amd.checkpoint import checkpointer as mod

    src = _model(6)
    with Checkpointer(src, tile_bytes=4096, slots=2) as ck:
        assert ck.size == 2 * ck.slot_bytes
        ck.save({"step": 1})
        first = ck._active()[0].index
        for v in src.values():
            v.add_(1)
        want = {k: v.clone() for k, v in src.items()}
        ck.save({"step": 2})
        assert ck._active()[0].index != first and ck.header()["generation"] == 2

        def killed(*args, **kwargs):  # the process dies in the middle of the next save
            raise RuntimeError("killed mid-save")

        monkeypatch.setattr(mod, "host_pack", killed)
        for v in src.values():
            v.add_(1)
        with pytest.raises(RuntimeError):
            ck.save({"step": 3})
        monkeypatch.undo()
        assert ck.header()["metadata"] == {"step": 2}  # still the newest complete copy
        ck.restore()
        for k in want:
            assert torch.equal(src[k], want[k]), k
        ck.save({"step": 3})  # the interrupted slot is reused
        assert ck.header()["generation"] == 3


def test_single_slot_save_invalidates_first():
    src = _model(7)
    with Checkpointer(src, tile_bytes=4096) as ck:
        ck.save({"step": 1})
        ck._invalidate(ck._target()[0])  # what a save does before writing
        with pytest.raises(CheckpointError):
            ck.restore()


def test_resume_refuses_a_corrupt_region_instead_of_starting_fresh(tmp_path):
    from terraform_provider_iterative_amd.checkpoint import preemption

    path = str(tmp_path / "spill")
    src = _model(8)
    ref = {k: v.clone() for k, v in src.items()}
    with Checkpointer(src, path=path, tile_bytes=4096) as ck:
        ck.save({"step": 5})
        good = ck.persist(str(tmp_path / "good.tpi"))
        ck.region.array(ck.slots[0].base + ck.stream_offset + 100, 1)[0] ^= 0x5A
    for v in src.values():
        v.zero_()
    with Checkpointer(src, path=path, tile_bytes=4096) as ck:
        with pytest.raises(CheckpointError, match="verification"):
            preemption.resume(ck)  # no persisted copy: an error, never a fresh start
        meta = preemption.resume(ck, persist_path=good)  # falls back to the persisted copy
        assert meta == {"step": 5}
    for k in ref:
        assert torch.equal(src[k], ref[k]), k
    os.remove(good)
    with open(path, "r+b") as f:  # make the region unreadable too: both copies bad
        f.seek(0)
        f.write(b"\0" * 8)
    with Checkpointer(src, path=path, tile_bytes=4096) as ck:
        assert preemption.resume(ck) is None  # truly nothing saved: fresh start


def _stream_pair(tmp_path, codec):
    import torch

    from terraform_provider_iterative_amd.checkpoint import Checkpointer

    g = torch.Generator().manual_seed(3)
    src = {"w": torch.randn(70000, generator=g), "b": torch.randn(33, 17, generator=g).t(),
           "i": torch.arange(5000, dtype=torch.int64)}
    dst = {"w": torch.zeros(70000), "b": torch.zeros(17, 33), "i": torch.zeros(5000,
                                                                             dtype=torch.int64)}
    path = str(tmp_path / "spill")
    writer = Checkpointer(src, path=path, tile_bytes=4096, codec=codec)
    reader_holder = {}

    def make_reader():
        reader_holder["ck"] = Checkpointer(dst, path=path, tile_bytes=4096)

    return src, dst, writer, reader_holder, make_reader


@pytest.mark.parametrize("codec", ["none", "tpz1"])
def test_streamed_save_is_restored_by_a_successor(tmp_path, codec):
    """Preemption hand-off: the successor sees the streaming header as soon as the save
    starts and restores once the writer's progress says the data is there."""
    import threading

    import torch

    src, dst, writer, holder, make_reader = _stream_pair(tmp_path, codec)
    result = {}

    def successor():
        make_reader()
        ck = holder["ck"]
        header = ck.latest()
        result["streaming"] = bool(header and header.get("streaming"))
        result["meta"] = header["metadata"]
        result["res"] = ck.restore(stream_timeout=10)

    threads = []

    def on_stream():  # the supervisor would start the successor now
        t = threading.Thread(target=successor)
        t.start()
        threads.append(t)
        time.sleep(0.2)  # let it find the header mid-save

    writer.save({"step": 7}, on_stream=on_stream)
    threads[0].join(30)
    assert result["streaming"] and result["meta"]["step"] == 7
    assert result["res"].bad_tiles == 0
    for k in src:
        assert torch.equal(dst[k], src[k]), k
    # after the save the checkpoint is an ordinary complete one
    assert holder["ck"].latest()["complete"] and holder["ck"]._streaming() is None
    holder["ck"].close()
    writer.close()


def test_failed_streamed_save_fails_the_successor(tmp_path, monkeypatch):
    from terraform_provider_iterative_amd.checkpoint import CheckpointError, Checkpointer

    src, dst, writer, holder, make_reader = _stream_pair(tmp_path, "none")

    def boom(*a, **k):
        raise RuntimeError("device lost")

    monkeypatch.setattr(writer, "_host_save", boom)
    with pytest.raises(RuntimeError):
        writer.save({"step": 1}, on_stream=lambda: None)
    make_reader()
    # the failed stream is not offered for restore
    assert holder["ck"].latest() is None
    with pytest.raises(CheckpointError):
        holder["ck"].restore()
    holder["ck"].close()
    writer.close()


def test_engine_pool_hands_out_the_matching_engine_and_releases_the_rest(monkeypatch):
    # prewarm_engine's pool, with stand-in engines (no GPU): the first Checkpointer on a device
    # takes the engine with its parameters; the device's other prewarmed engines are closed
    from terraform_provider_iterative_amd.checkpoint import engine as ckmod

    class FakeEngine:
        def __init__(self):
            self.closed = False

        def close(self):
            self.closed = True

    monkeypatch.setattr(ckmod, "_engine_pool", {})
    match, other, elsewhere = FakeEngine(), FakeEngine(), FakeEngine()
    ckmod._engine_pool[(0, 256 << 20, 3, 1 << 20)] = [match]
    ckmod._engine_pool[(0, 64 << 20, 2, 1 << 20)] = [other]
    ckmod._engine_pool[(1, 256 << 20, 3, 1 << 20)] = [elsewhere]
    assert ckmod._take_engine(0, 256 << 20, 3, 1 << 20) is match
    assert other.closed and not match.closed and not elsewhere.closed
    assert list(ckmod._engine_pool) == [(1, 256 << 20, 3, 1 << 20)]
    assert ckmod._take_engine(0, 256 << 20, 3, 1 << 20) is None


@pytest.mark.parametrize("slots", [1, 2])
def test_stream_of_a_dead_writer_is_not_waited_for(tmp_path, slots):
    """A slot left 'streaming' by a writer that died (SIGKILL after the grace period, OOM) is
    no checkpoint: resume must not stall TPI_STREAM_TIMEOUT on it and must fall back to the
    older copy (slots=2) or a fresh start (slots=1)."""
    import subprocess
    import sys

    from terraform_provider_iterative_amd.checkpoint import checkpointer as ckmod, preemption

    dead = subprocess.Popen([sys.executable, "-c", "pass"])
    dead.wait()
    state = {"w": torch.arange(5000, dtype=torch.float32)}
    path = str(tmp_path / "spill")
    ck = Checkpointer(state, path=path, tile_bytes=4096, slots=slots)
    ck.save({"step": 1})
    state["w"].add_(1)
    ck.save({"step": 2}) if slots == 2 else None
    slot, generation = ck._target()  # the slot the next save would write
    ck._invalidate(slot)
    header = ck._header(False, 0, {"step": 3}, "none", None, generation)
    header["streaming"] = True
    ck._write_header(slot, header)
    prog = slot.progress
    prog[1], prog[2], prog[3], prog[5] = generation, 0, 0, dead.pid
    prog[4] = ckmod.STREAM_RUNNING
    prog[0] = ckmod.PROGRESS_MAGIC
    fresh = {"w": torch.zeros(5000)}
    ck2 = Checkpointer(fresh, path=path, tile_bytes=4096, slots=slots)
    t0 = time.monotonic()
    meta = preemption.resume(ck2)
    assert time.monotonic() - t0 < 5
    if slots == 2:
        assert meta["step"] == 2 and torch.equal(fresh["w"], state["w"])
    else:
        assert meta is None
    prog[5] = os.getpid()  # the same slot with a live writer is a stream in flight
    assert ck2.latest()["metadata"]["step"] == 3
    ck2.close()
    ck.close()


def test_save_waits_for_a_predecessors_stream_into_the_same_slot(tmp_path):
    """After an HBM hand-off the successor runs while its predecessor still spills into the
    shared host region: the successor's first save must not overwrite that slot mid-write."""
    import threading

    from terraform_provider_iterative_amd.checkpoint import checkpointer as ckmod

    state = {"w": torch.arange(5000, dtype=torch.float32)}
    path = str(tmp_path / "spill")
    ck = Checkpointer(state, path=path, tile_bytes=4096)
    ck.save({"step": 1})
    prog = ck.slots[0].progress
    prog[1], prog[5] = ck.header()["generation"], os.getppid()  # a live foreign writer
    prog[4] = ckmod.STREAM_RUNNING
    prog[0] = ckmod.PROGRESS_MAGIC
    threading.Timer(0.4, lambda: prog.__setitem__(4, ckmod.STREAM_COMPLETE)).start()
    t0 = time.monotonic()
    ck.save({"step": 2})
    assert time.monotonic() - t0 >= 0.35
    assert ck.header()["metadata"]["step"] == 2
    # a writer that died mid-stream: no wait, reported as not completed
    prog[5], prog[4], prog[0] = 2 ** 22 + 12345, ckmod.STREAM_RUNNING, ckmod.PROGRESS_MAGIC
    assert ck.wait_stream(timeout=5) is False
    prog[4] = ckmod.STREAM_COMPLETE
    assert ck.wait_stream() is None
    ck.close()


def test_close_stops_and_joins_a_durability_watcher(tmp_path):
    """A successor that closes its checkpointer while the hand-off's durability watcher still
    waits on the predecessor's spill: close() stops the wait (None, not a false 'failed') and
    joins the watcher before the region is unmapped under it."""
    from terraform_provider_iterative_amd.checkpoint import checkpointer as ckmod

    state = {"w": torch.arange(5000, dtype=torch.float32)}
    ck = Checkpointer(state, path=str(tmp_path / "spill"), tile_bytes=4096)
    ck.save({"step": 1})
    prog = ck.slots[0].progress
    prog[1], prog[5] = ck.header()["generation"], os.getppid()  # a live foreign writer
    prog[4] = ckmod.STREAM_RUNNING
    prog[0] = ckmod.PROGRESS_MAGIC
    seen = []
    watcher = ck.watch(lambda: seen.append(ck.wait_stream(timeout=60)), "test-watcher")
    time.sleep(0.1)
    assert watcher.is_alive()
    t0 = time.monotonic()
    ck.close()
    assert time.monotonic() - t0 < 2
    assert not watcher.is_alive() and seen == [None]


def test_durable_reports_a_complete_copy_of_a_generation(tmp_path):
    state = {"w": torch.arange(5000, dtype=torch.float32)}
    ck = Checkpointer(state, path=str(tmp_path / "spill"), tile_bytes=4096, slots=2)
    assert not ck.durable(1)
    ck.save({"step": 1})
    gen = ck.header()["generation"]
    assert ck.durable(gen) and not ck.durable(gen + 1)
    ck.save({"step": 2})
    assert ck.durable(gen) and ck.durable(gen + 1)
    ck.close()


def test_save_async_codec_override_and_periodic_policy(tmp_path, monkeypatch):
    """A periodic background spill goes out without the codec by default (TPI_SYNC_CODEC);
    the header records what the spill used, and the restore follows it."""
    from terraform_provider_iterative_amd.checkpoint import preemption

    g = torch.Generator().manual_seed(3)
    t = {"w": torch.randn(1 << 16, generator=g), "b": torch.randn(999, generator=g)}
    ref = {k: v.clone() for k, v in t.items()}
    ck = Checkpointer(t, path=str(tmp_path / "spill"), tile_bytes=1 << 14, codec="tpz1")
    ck.save_async({"step": 1}, codec="none").result()
    assert ck.latest()["codec"] == "none" and ck.codec == "tpz1"
    for v in t.values():
        v.zero_()
    ck.restore()
    assert all(torch.equal(t[k], ref[k]) for k in t)
    ck.save_async({"step": 2}).result()
    assert ck.latest()["codec"] == "tpz1"
    with pytest.raises(ValueError):
        ck.save_async({"step": 3}, codec="zstd")
    ck.close()
    monkeypatch.delenv("TPI_SYNC_CODEC", raising=False)
    assert preemption.sync_codec() == "none"
    monkeypatch.setenv("TPI_SYNC_CODEC", "tpz1")
    assert preemption.sync_codec() == "tpz1"
    monkeypatch.setenv("TPI_SYNC_CODEC", "auto")
    assert preemption.sync_codec() is None


def test_release_schedule_frees_a_storage_after_its_last_tensor(tmp_path):
    """VERDICT r3 #3 (big state): a preempted rank frees each storage as soon as the spill has
    published every tile of every bound tensor in it -- views of one storage go together, at
    the end of the last of them in the packed stream, and storages go in stream order."""
    import torch

    from terraform_provider_iterative_amd.checkpoint import Checkpointer

    base = torch.zeros(3000)
    state = {"a": torch.ones(5000), "v1": base[:1000], "b": torch.ones(7000),
             "v2": base[1000:], "c": torch.ones(10)}
    with Checkpointer(state, tile_bytes=4096) as ck:
        schedule = ck.release_schedule()
        ends = {e.name: e.offset + e.nbytes for e in ck.plan.entries}
        got = [(end, st.data_ptr()) for end, st in schedule]
        want = [(ends["a"], state["a"].untyped_storage().data_ptr()),
                (ends["b"], state["b"].untyped_storage().data_ptr()),
                (ends["v2"], base.untyped_storage().data_ptr()),  # with its last view
                (ends["c"], state["c"].untyped_storage().data_ptr())]
        assert got == want
        assert [end for end, _ in schedule] == sorted(end for end, _ in schedule)
        assert ck.release_schedule(device_only=True) == []


def test_save_refuses_a_slot_a_live_foreign_writer_still_streams(tmp_path, monkeypatch):
    """when wait_stream() gives up on a foreign writer that is still alive, a save
    must not go on to write the slot that writer is streaming into."""
    import subprocess
    import sys

    import torch

    from terraform_provider_iterative_amd.checkpoint import CheckpointError, Checkpointer
    from terraform_provider_iterative_amd.checkpoint.checkpointer import (PROGRESS_MAGIC,
                                                                          STREAM_RUNNING)

    monkeypatch.setenv("TPI_STREAM_TIMEOUT", "0.2")
    state = {"w": torch.ones(4096)}
    writer = subprocess.Popen([sys.executable, "-c", "import time; time.sleep(30)"])
    try:
        with Checkpointer(state, path=str(tmp_path / "spill"), tile_bytes=4096) as ck:
            ck.save({"step": 1})
            prog = ck.slots[0].progress  # another live process "is streaming" into it
            prog[1], prog[4], prog[5] = 2, STREAM_RUNNING, writer.pid
            prog[0] = PROGRESS_MAGIC
            with pytest.raises(CheckpointError, match="still streaming"):
                ck.save({"step": 2})
            writer.kill()
            writer.wait()
            ck.save({"step": 3})  # its writer is gone: the slot is free again
            assert ck.header()["metadata"] == {"step": 3}
    finally:
        if writer.poll() is None:
            writer.kill()


@pytest.mark.parametrize("codec,slots", [("none", 1), ("tpz1", 1), ("none", 2), ("tpz1", 2)])
@pytest.mark.parametrize("group_bytes", [1, 40_000, 1 << 30])
def test_materialize_allocates_and_restores_group_by_group(tmp_path, codec, slots, group_bytes):
    """Checkpointer.materialize() rebuilds a region's tensors without being handed any: one
    tensor per group, groups sharing boundary tiles, or everything at once; the checkpointer
    it returns is bound to them and saves again into the same region."""
    path = str(tmp_path / "spill.bin")
    src = _model(5)
    ref = {k: v.clone() for k, v in src.items()}
    with Checkpointer(src, path=path, tile_bytes=4096, codec=codec, slots=slots) as ck:
        ck.save({"step": 1})
        if slots == 2:  # the newest of two complete copies is the one materialized
            for v in src.values():
                v.mul_(2) if v.is_floating_point() else v.add_(1)
            ref = {k: v.clone() for k, v in src.items()}
            ck.save({"step": 2})
    ck2, tensors, res = Checkpointer.materialize(path, "cpu", group_bytes=group_bytes)
    try:
        assert res.bad_tiles == 0 and res.bytes == ck2.plan.total
        assert ck2.materialize_stats["alloc"] == "nogil"  # the _tpi_torch extension is built
        assert list(tensors) == list(ref)
        for k in ref:
            assert tensors[k].is_contiguous() and torch.equal(tensors[k], ref[k]), k
        expect_groups = len(ref) if group_bytes == 1 else (1 if group_bytes > 1e6 else None)
        if expect_groups is not None:
            assert ck2.materialize_stats["groups"] == expect_groups
        assert ck2.header()["metadata"]["step"] == (2 if slots == 2 else 1)
        # the device engine needs every (sub-)plan to start with a segment at offset 0
        lead = torch.empty(4096, dtype=torch.uint8)
        for lo, hi in ck2._groups(1):
            sub, ta, tb = ck2._sub_plan(lo, hi, [tensors[e.name] for e in
                                                 ck2.plan.entries[lo:hi]], lead)
            assert sub.entries[0].offset == 0 and 0 <= ta < tb <= ck2.plan.ntiles
            assert sub.total <= (tb - ta) * 4096
        tensors["w1"].fill_(0.5)
        ck2.save({"step": 9})
    finally:
        ck2.close()
    fresh = {k: torch.zeros_like(v) for k, v in ref.items()}
    with Checkpointer(fresh, path=path, tile_bytes=4096, codec=codec, slots=slots) as ck3:
        ck3.restore()
        assert ck3.header()["metadata"]["step"] == 9
    assert torch.equal(fresh["w1"], torch.full_like(fresh["w1"], 0.5))
    assert torch.equal(fresh["embed"], ref["embed"])


def test_materialize_reports_corruption_and_missing_checkpoints(tmp_path):
    path = str(tmp_path / "spill.bin")
    with Checkpointer(_model(6), path=path, tile_bytes=4096) as ck:
        ck.save()
        stream_at = ck.stream_offset
    with open(path, "r+b") as f:  # flip one byte of the stream
        f.seek(stream_at + 5000)
        b = f.read(1)
        f.seek(stream_at + 5000)
        f.write(bytes([b[0] ^ 0xFF]))
    with pytest.raises(CheckpointError, match="corrupt tile"):
        Checkpointer.materialize(path, "cpu", group_bytes=1)
    empty = str(tmp_path / "empty.bin")
    with open(empty, "wb") as f:
        f.write(b"\0" * 8192)
    with pytest.raises(CheckpointError, match="no checkpoint header"):
        Checkpointer.materialize(empty, "cpu")


def test_preemption_materialize_journals_and_tells_the_supervisor(tmp_path, monkeypatch):
    from terraform_provider_iterative_amd.checkpoint import preemption

    events = tmp_path / "events.jsonl"
    monkeypatch.setenv("TPI_EVENTS_FILE", str(events))
    rfd, wfd = os.pipe()
    monkeypatch.setenv("TPI_NOTIFY_FD", str(wfd))
    try:
        assert preemption.materialize(str(tmp_path / "missing.spill"), "cpu") is None
        path = str(tmp_path / "spill.bin")
        ref = _model(7)
        with Checkpointer(ref, path=path, tile_bytes=4096, codec="tpz1") as ck:
            ck.save({"step": 41})
        ck2, tensors, meta = preemption.materialize(path, "cpu", group_bytes=1)
        ck2.close()
        assert meta["step"] == 41
        assert all(torch.equal(tensors[k], ref[k]) for k in ref)
        assert os.read(rfd, 64) == b"restored\n"
    finally:
        os.close(rfd)
        os.close(wfd)
    text = events.read_text()
    assert "checkpoint-restored" in text and "materialized in 5 groups" in text


def test_wait_pinned_without_a_prefetch_returns_none(tmp_path):
    from terraform_provider_iterative_amd.checkpoint.host import wait_pinned

    assert wait_pinned(str(tmp_path / "never-prefetched.spill"), timeout=0.1) is None


def test_materialize_on_host_waits_for_a_streamed_save_to_complete(tmp_path):
    """Host tensors: materialize() of a region whose writer is still streaming waits for the
    writer's completion (no device engine to restore behind it), then restores."""
    import threading

    from terraform_provider_iterative_amd.checkpoint import checkpointer as ckmod

    path = str(tmp_path / "spill.bin")
    src = _model(8)
    writer = Checkpointer(src, path=path, tile_bytes=4096)
    writer.save({"step": 4})
    slot = writer.slots[0]
    header = writer.header()
    header.update(complete=False, streaming=True)
    writer._write_header(slot, header)
    prog = slot.progress
    prog[1], prog[2], prog[3], prog[4] = header["generation"], 0, 0, ckmod.STREAM_RUNNING
    prog[5] = os.getpid()
    prog[0] = ckmod.PROGRESS_MAGIC
    box = {}
    th = threading.Thread(target=lambda: box.update(out=Checkpointer.materialize(
        path, "cpu", group_bytes=1, stream_timeout=20)))
    th.start()
    time.sleep(0.3)
    assert th.is_alive()  # still waiting for the writer
    prog[2] = writer.plan.ntiles
    header.update(complete=True, streaming=False)
    writer._write_header(slot, header)
    prog[4] = ckmod.STREAM_COMPLETE
    th.join(30)
    ck, tensors, res = box["out"]
    assert res.bad_tiles == 0 and not ck.materialize_stats["streamed"]
    assert all(torch.equal(tensors[k], src[k]) for k in src)
    ck.close()
    writer.close()


def test_materialize_falls_back_to_the_older_copy_when_the_stream_fails(tmp_path):
    """slots=2: the predecessor's streamed save of generation 2 fails; materialize() restores
    generation 1, the complete copy the region still holds (and says so)."""
    import threading

    from terraform_provider_iterative_amd.checkpoint import checkpointer as ckmod

    path = str(tmp_path / "spill.bin")
    src = _model(9)
    ref = {k: v.clone() for k, v in src.items()}
    writer = Checkpointer(src, path=path, tile_bytes=4096, slots=2)
    writer.save({"step": 1})
    slot, generation = writer._target()  # the slot a second save would stream into
    header = writer._header(False, 0, {"step": 2}, "none", None, generation)
    header["streaming"] = True
    writer._write_header(slot, header)
    prog = slot.progress
    prog[1], prog[2], prog[3], prog[4] = generation, 0, 0, ckmod.STREAM_RUNNING
    prog[5] = os.getpid()
    prog[0] = ckmod.PROGRESS_MAGIC
    box = {}
    th = threading.Thread(target=lambda: box.update(out=Checkpointer.materialize(
        path, "cpu", group_bytes=1, stream_timeout=20)))
    th.start()
    time.sleep(0.3)
    prog[4] = ckmod.STREAM_FAILED
    th.join(30)
    ck, tensors, res = box["out"]
    assert res.bad_tiles == 0 and ck.materialized_metadata["step"] == 1
    assert "failed" in ck.materialize_stats["fallback"]
    assert all(torch.equal(tensors[k], ref[k]) for k in ref)
    ck.close()
    writer.close()


def test_materialize_refuses_a_persisted_file(tmp_path):
    """A persisted checkpoint is one slot cut after its stream, not a spill region: mapping
    it as a region would grow the file, so materialize() says to use load() instead."""
    persisted = str(tmp_path / "ckpt.tpi")
    with Checkpointer(_model(10), tile_bytes=4096) as ck:
        ck.save()
        ck.persist(persisted)
    size = os.path.getsize(persisted)
    with pytest.raises(CheckpointError, match="persisted checkpoint"):
        Checkpointer.materialize(persisted, "cpu")
    assert os.path.getsize(persisted) == size
