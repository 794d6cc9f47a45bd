"""The first-log probe reports the start gate's wait beside the latency it is part of."""
import json
import os

from terraform_provider_iterative_amd import bench_latency


def test_gate_wait_sums_the_tasks_gpu_drain_events(tmp_path):
    events = tmp_path / "mi355x" / "task-a" / "supervisor"
    events.mkdir(parents=True)
    lines = [{"time": 1, "code": "gpu-drain",
              "description": ["gpu 0", "waited 1.250 s", "VRAM in use 60.0 -> 2.0 GB"]},
             {"time": 2, "code": "rank-start", "description": ["rank 0", "waited 9 s"]},
             {"time": 3, "code": "gpu-drain", "description": ["gpu 1", "waited 0.500 s"]}]
    (events / "events.jsonl").write_text("".join(json.dumps(e) + "\n" for e in lines))
    assert bench_latency._gate_wait(str(tmp_path)) == 1.75
    assert bench_latency._gate_wait(os.path.join(str(tmp_path), "nothing")) == 0.0
