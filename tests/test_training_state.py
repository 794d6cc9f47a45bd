"""TrainingState: model + optimizer round trip, host-side optimizer scalars in the header."""
import pytest
import torch

from terraform_provider_iterative_amd.checkpoint import TrainingState, collect


def _setup(seed=0):
    torch.manual_seed(seed)
    model = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.LayerNorm(32),
                                torch.nn.Linear(32, 4))
    opt = torch.optim.AdamW(model.parameters(), lr=1e-2)
    return model, opt


def _train(model, opt, steps, seed):
    g = torch.Generator().manual_seed(seed)
    for _ in range(steps):
        x = torch.randn(8, 16, generator=g)
        model(x).pow(2).mean().backward()
        opt.step()
        opt.zero_grad()


def _snapshot(model, opt):
    tensors, host = collect(model, opt)
    return {k: v.clone() for k, v in {**tensors, **host}.items()}


def test_collect_names_and_split():
    model, opt = _setup()
    _train(model, opt, 1, 0)
    tensors, host = collect(model, opt, device="cpu")
    assert "model.0.weight" in tensors and "optim.0.exp_avg" in tensors
    assert "optim.0.step" in tensors  # CPU model: step counters live with the rest
    # checkpointing "on another device": the CPU tensors become header-carried host tensors
    tensors2, host2 = collect(model, opt, device="meta")
    assert not tensors2 and "optim.0.step" in host2


def test_collect_rejects_large_off_device_tensor():
    model, opt = _setup()
    with pytest.raises(ValueError):
        collect(model, opt, extra={"big": torch.zeros(10000)}, device="meta")


def test_round_trip_resumes_exact_training_state(tmp_path):
    model, opt = _setup()
    _train(model, opt, 3, 1)
    state = TrainingState(model, opt, extra={"epoch": torch.tensor(7)},
                          path=str(tmp_path / "spill"), tile_bytes=4096)
    want = _snapshot(model, opt)
    state.save({"step": 3})
    _train(model, opt, 2, 2)  # diverge
    assert not torch.equal(_snapshot(model, opt)["model.0.weight"], want["model.0.weight"])
    meta = state.resume()
    assert meta["step"] == 3
    got = _snapshot(model, opt)
    assert set(got) == set(want)
    for k in want:
        assert torch.equal(got[k], want[k]), k
    state.close()
    # a fresh process (new model/optimizer objects) resumes from the shared spill file
    model2, opt2 = _setup(seed=5)
    _train(model2, opt2, 1, 9)
    with TrainingState(model2, opt2, extra={"epoch": torch.tensor(0)},
                       path=str(tmp_path / "spill"), tile_bytes=4096) as fresh:
        assert fresh.resume()["step"] == 3
        got2 = _snapshot(model2, opt2)
    for k in want:
        if k.startswith(("model.", "optim.")):
            assert torch.equal(got2[k], want[k]), k


def test_save_async_captures_host_tensors_at_call_time(tmp_path):
    model, opt = _setup()
    _train(model, opt, 2, 3)
    with TrainingState(model, opt, path=str(tmp_path / "s"), tile_bytes=4096) as state:
        want = _snapshot(model, opt)
        pending = state.save_async({"step": 2})
        pending.result(timeout=30)
        _train(model, opt, 1, 4)
        assert state.resume()["step"] == 2
        got = _snapshot(model, opt)
    for k in want:
        assert torch.equal(got[k], want[k]), k
