"""Workdir fan-out over torch.distributed with gloo (world 2 and 4) on CPU."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, root, results, method):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from terraform_provider_iterative_amd.runtime.workdir import stage_workdir

        staged = stage_workdir(root, device=torch.device("cpu"), method=method,
                               exclude=["skip.bin"])
        names = sorted(f.path for f in staged.files)
        a = bytes(staged.tensor("a.txt").tolist())
        big = staged.tensor("sub/big.bin")
        expect = torch.from_numpy(
            __import__("numpy").frombuffer(open(os.path.join(root, "sub/big.bin"), "rb").read(),
                                           dtype="uint8").copy())
        results[rank] = (names, a, bool(torch.equal(big, expect)),
                         staged.stats.get("verified"), staged.stats.get("method"))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,method", [(2, "broadcast"), (4, "sharded"), (3, "auto")])
def test_stage_workdir_on_cpu_ranks(tmp_path, world, method):
    """The library staging path with gloo ranks on CPU: host images are read by every rank
    (the GPU schedules -- sharded all-gather, broadcast -- run the RCCL task communicator and
    are covered by tests/test_gpu_stage.py); the file list comes from rank 0 and the copies
    are verified by digest."""
    root = tmp_path / "wd"
    (root / "sub").mkdir(parents=True)
    (root / "a.txt").write_bytes(b"hello workdir")
    (root / "sub" / "big.bin").write_bytes(os.urandom(300001))
    (root / "skip.bin").write_bytes(b"x" * 10)
    (root / "main.tf").write_text("# excluded by default")
    manager = mp.Manager()
    results = manager.dict()
    mp.spawn(_worker, args=(world, _free_port(), str(root), results, method), nprocs=world)
    assert len(results) == world
    for rank in range(world):
        names, a, big_ok, verified, used = results[rank]
        assert names == ["a.txt", "sub/big.bin"]
        assert a == b"hello workdir" and big_ok
        assert verified is True and used == "independent"


def test_write_back(tmp_path):
    from terraform_provider_iterative_amd.runtime.workdir import stage_workdir

    root = tmp_path / "src"
    root.mkdir()
    (root / "x.bin").write_bytes(b"abc" * 1000)
    staged = stage_workdir(str(root), device=torch.device("cpu"))
    staged.tensor("x.bin")[:3] = torch.tensor([120, 121, 122], dtype=torch.uint8)
    out = tmp_path / "out"
    staged.write_back(str(out))
    assert (out / "x.bin").read_bytes()[:6] == b"xyzabc"


def test_sync_writes_back_only_dirty_shards(tmp_path):
    from terraform_provider_iterative_amd.runtime.workdir import stage_workdir

    root = tmp_path / "src"
    root.mkdir()
    (root / "a.bin").write_bytes(bytes(range(256)) * 8192)   # 2 MiB: 2 shards
    (root / "b.bin").write_bytes(b"b" * 5000)
    staged = stage_workdir(str(root), device=torch.device("cpu"))
    assert staged.sync(str(root))["dirty_shards"] == 0
    staged.tensor("a.bin")[(1 << 20) + 5] = 7       # second shard of a.bin only
    res = staged.sync(str(root))
    assert res["dirty_shards"] == 1 and res["bytes"] == 1 << 20
    data = (root / "a.bin").read_bytes()
    assert data[(1 << 20) + 5] == 7 and data[:1 << 20] == (bytes(range(256)) * 4096)
    assert staged.sync(str(root))["dirty_shards"] == 0


def _resume_worker(rank, world, port, root, results, steps):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from terraform_provider_iterative_amd.checkpoint import TrainingState

        torch.manual_seed(rank)
        model = torch.nn.Linear(8, 8)
        opt = torch.optim.SGD(model.parameters(), lr=0.1)
        spill = os.path.join(root, "rank%d" % rank)
        with TrainingState(model, opt, path=spill, tile_bytes=4096) as state:
            if steps[rank] is not None:  # this rank's previous incarnation saved at that step
                state.save({"step": steps[rank]})
            with torch.no_grad():
                model.weight.zero_()
            meta = state.resume_consistent()
            results[rank] = (None if meta is None else meta["step"],
                             float(model.weight.abs().sum()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("steps,agree", [((5, 5, 5), True), ((5, 4, 5), False),
                                         ((5, None, 5), False)])
def test_resume_consistent_all_or_nothing(tmp_path, steps, agree):
    manager = mp.Manager()
    results = manager.dict()
    world = len(steps)
    mp.spawn(_resume_worker, args=(world, _free_port(), str(tmp_path), results, steps),
             nprocs=world)
    for rank in range(world):
        step, weight = results[rank]
        if agree:
            assert step == 5 and weight > 0  # restored
        else:
            assert step is None and weight == 0  # fresh start everywhere


def _corrupt_worker(rank, world, port, root, results):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from terraform_provider_iterative_amd.checkpoint import CheckpointError, TrainingState

        torch.manual_seed(rank)
        model = torch.nn.Linear(64, 64)
        opt = torch.optim.SGD(model.parameters(), lr=0.1)
        with TrainingState(model, opt, path=os.path.join(root, "rank%d" % rank),
                           tile_bytes=4096) as state:
            state.save({"step": 7})
            ck = state.checkpointer
            if rank == 1:  # this rank's spill got corrupted: every rank must abort together
                ck.region.array(ck.slots[0].base + ck.stream_offset + 10, 1)[0] ^= 0xFF
            try:
                state.resume_consistent()
                results[rank] = "resumed"
            except CheckpointError as error:
                results[rank] = "aborted: %s" % error
    finally:
        dist.destroy_process_group()


def test_resume_consistent_aborts_every_rank_when_one_restore_fails(tmp_path):
    manager = mp.Manager()
    results = manager.dict()
    mp.spawn(_corrupt_worker, args=(3, _free_port(), str(tmp_path), results), nprocs=3)
    assert sorted(results) == [0, 1, 2]
    for rank in range(3):
        assert results[rank].startswith("aborted") and "[1]" in results[rank], results[rank]


def _tick_worker(rank, world, port, root, results, agreement):
    """Periodic checkpoints in a coupled job (an all-reduce per step, like DDP): rank 0's
    clock proposes, every rank checkpoints at the same steps; rank 1 runs slower per step."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), TPI_SYNC_INTERVAL="0.2",
                      TPI_EVENTS_FILE=os.path.join(root, "events.jsonl"), RANK=str(rank),
                      TPI_AGREEMENT=agreement)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import time

        from terraform_provider_iterative_amd.checkpoint import Checkpointer, preemption

        state = {"w": torch.zeros(2048)}
        ck = Checkpointer(state, path=os.path.join(root, "rank%d" % rank), tile_bytes=4096,
                          slots=2)
        preemption.register(ck)
        saved_at = []
        for i in range(1, 25):
            grad = torch.ones(4)
            dist.all_reduce(grad)
            state["w"].fill_(i)
            time.sleep(0.02 if rank == 0 else 0.035)
            if preemption.step(i):
                saved_at.append(i)
        ck.wait_pending()
        results[rank] = (saved_at, ck.header()["metadata"].get("step"),
                         preemption._agreement.kind)
        ck.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("agreement", ["auto", "collective"])
def test_periodic_tick_is_collective(tmp_path, agreement):
    manager = mp.Manager()
    results = manager.dict()
    mp.spawn(_tick_worker, args=(2, _free_port(), str(tmp_path), results, agreement),
             nprocs=2)
    saved0, last0, kind = results[0]
    assert kind == ("shm" if agreement == "auto" else "collective")
    assert len(saved0) >= 2, saved0
    for rank in range(2):
        saved, last, _ = results[rank]
        assert saved == saved0, (rank, saved, saved0)
        assert last == saved0[-1]
    lines = (tmp_path / "events.jsonl").read_text().splitlines()
    assert sum('"checkpoint-synced"' in l for l in lines) == 2 * len(saved0)
