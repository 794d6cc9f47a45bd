"""bench.py contract on the multi-rank path the driver uses for N > 1 (``torch.distributed.run
--nproc-per-node N``): rehearsed with 2 gloo ranks on CPU tensors -- one JSON line from rank 0,
the whole-job aggregate, max-over-ranks timing, a verified restore."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(tmp_path, *extra):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--device", "cpu", "--total-gb", "0.02",
           "--steps", "2", "--warmup", "1", "--no-latency", "--hidden", "256", *extra]
    env = dict(os.environ, OMP_NUM_THREADS="2")
    out = subprocess.run(cmd, cwd=str(tmp_path), capture_output=True, text=True, timeout=300,
                         env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    assert "bench: " not in out.stdout, out.stdout  # the heartbeat goes to stderr
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]  # (gloo prints too)
    assert len(lines) == 1, out.stdout
    return json.loads(lines[0])


def test_two_rank_rehearsal_prints_one_json_line(tmp_path):
    d = _run(tmp_path)
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"):
        assert key in d, key
    assert d["n_gpus"] == 2 and d["steps"] == 2 and d["warmup"] == 1
    assert d["value"] > 0 and d["higher_is_better"] is True and d["scaling"] == "strong"
    assert d["config"]["parallelism"] == "shard2"
    assert d["config"]["checkpoint_bytes"] >= 0.02e9
    # value = both directions of the whole job's checkpoint bytes per timed second
    expect = 2 * d["config"]["checkpoint_bytes"] * d["steps"] / (d["ms_per_step"] * d["steps"] / 1e3) / 1e9
    assert abs(d["value"] - expect) / expect < 0.02
    assert d["restore_verified"] is True
    assert "CPU rehearsal" in d["data"]
    # N > 1 evidence: every rank's process-group size; RCCL's fields null under gloo
    comm = d["comm"]
    assert [c["rank"] for c in comm["ranks"]] == [0, 1]
    assert all(c["torch_pg_size"] == 2 and c["backend"] == "gloo" for c in comm["ranks"])
    assert comm["pg_sizes_match"] is True and comm["rccl_nranks_match"] is None
    assert d["config"]["gpu_max_hw_queues"] >= 1 and "env_knobs" in d["config"]


def test_side_measurement_watchdog_keeps_the_headline(tmp_path):
    # a side measurement that outlives --side-timeout must not cost the headline line
    d = _run(tmp_path, "--side-timeout", "0.001")
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["restore_verified"] is True
    # N > 1 prints the headline before the side measurements: they are deferred to stderr
    assert d["save_async"] == {"deferred": "stderr: bench-side"}, d


def test_bench_launches_its_own_ranks_without_torchrun(tmp_path):
    # `python bench.py --gpus N` with no launcher around it starts the N ranks itself
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3", "--device", "cpu",
           "--total-gb", "0.012", "--steps", "1", "--warmup", "1", "--no-latency",
           "--hidden", "256"]
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "2"
    out = subprocess.run(cmd, cwd=str(tmp_path), capture_output=True, text=True, timeout=300,
                         env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 3 and d["config"]["parallelism"] == "shard3"
    assert d["restore_verified"] is True
    side = [l for l in out.stderr.splitlines() if l.startswith("bench-side ")]
    assert side and "GBps" in json.loads(side[0][len("bench-side "):])["raw_GBps"]


def test_bench_refuses_a_world_that_disagrees_with_gpus(tmp_path):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--device", "cpu",
           "--total-gb", "0.01", "--no-latency"]
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    out = subprocess.run(cmd, cwd=str(tmp_path), capture_output=True, text=True, timeout=120,
                         env=env)
    assert out.returncode != 0
    assert "disagree" in out.stderr


def test_first_log_latency_probe_reports_every_rank(tmp_path, monkeypatch):
    # The headline's apply->first-log probe renders main.tf with parallelism = N; a missing
    # template key once turned every bench's first_log_latency_s into null.
    monkeypatch.setenv("TMPDIR", str(tmp_path))
    from terraform_provider_iterative_amd.bench_latency import measure_first_log_latency

    out = measure_first_log_latency(timeout=30, cloud="local", repeats=1, parallelism=2)
    assert out["parallelism"] == 2 and out["samples"] == 1
    assert out["cli_s"] is not None and out["api_s"] is not None
    assert out["cli_all_s"] is not None and out["cli_all_s"] >= out["cli_s"]


def test_first_log_latency_probe_gives_up_when_apply_fails(tmp_path, monkeypatch):
    # a failing apply (here: more GPUs than the node has) must not hold the bench for the
    # probe's whole timeout
    monkeypatch.setenv("TMPDIR", str(tmp_path))
    import time

    from terraform_provider_iterative_amd import bench_latency

    t0 = time.perf_counter()
    try:
        out = bench_latency.measure_first_log_latency(timeout=60, cloud="mi355x", repeats=1,
                                                      parallelism=64)
        assert out["cli_s"] is None
    except Exception:
        pass  # the in-process create refuses too; the bench catches that
    assert time.perf_counter() - t0 < 30


def test_eight_rank_rehearsal_finishes_inside_the_watchdog(tmp_path):
    """The driver's N=8 launch (torch.distributed.run --nproc-per-node 8) rehearsed on CPU:
    every side measurement finishes (no watchdog note) and rank 0 prints one line."""
    import time

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "8", "--device", "cpu", "--total-gb",
           "0.04", "--steps", "2", "--warmup", "1", "--no-latency", "--hidden", "256",
           "--side-timeout", "120"]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    t0 = time.time()
    out = subprocess.run(cmd, cwd=str(tmp_path), capture_output=True, text=True, timeout=400,
                         env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 8 and d["config"]["parallelism"] == "shard8"
    assert d["restore_verified"] is True
    # N > 1: the headline line comes before the side measurements, whose results follow on
    # stderr (a crash in a collective never rehearsed on 8 GPUs cannot lose the headline)
    assert d["save_async"] == {"deferred": "stderr: bench-side"}, d
    side = [l for l in out.stderr.splitlines() if l.startswith("bench-side ")]
    assert len(side) == 1, out.stderr[-3000:]
    side = json.loads(side[0][len("bench-side "):])
    assert "stall_ms" in side["save_async"] and "GBps" in side["raw_GBps"], side
    assert time.time() - t0 < 120 + 60


def test_a_restore_that_stops_rewriting_fails_the_bench(tmp_path):
    """every step poisons every successor tensor outside the timed window, so a
    restore that skips tensors after the first step (fault injected) cannot print
    ``restore_verified: true`` -- the bench says so and exits non-zero.  The same run without
    the fault verifies."""
    def run(fault):
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--device", "cpu",
               "--total-gb", "0.01", "--steps", "3", "--warmup", "1", "--no-latency",
               "--hidden", "256", "--broadcast-gb", "0"]
        env = dict(os.environ, OMP_NUM_THREADS="2")
        env.pop("TPI_BENCH_FAULT", None)
        if fault:
            env["TPI_BENCH_FAULT"] = fault
        return subprocess.run(cmd, cwd=str(tmp_path), capture_output=True, text=True,
                              timeout=300, env=env)

    good = run(None)
    assert good.returncode == 0, good.stderr[-2000:]
    d = json.loads([l for l in good.stdout.splitlines() if l.startswith("{")][0])
    assert d["restore_verified"] is True and d["value_kind"] == "overlapped_duplex"
    assert d["value_sequential"] and d["value_sequential"] > 0
    bad = run("skip-restore-after-first")
    assert bad.returncode != 0, bad.stdout[-2000:]
    d = json.loads([l for l in bad.stdout.splitlines() if l.startswith("{")][0])
    assert d["restore_verified"] is False
    assert "restore NOT verified" in bad.stderr


def test_region_placement_report_on_a_two_socket_node():
    """8 ranks, GPUs 0-3 on socket 0 and 4-7 on socket 1 (the MI355X node layout): regions on
    their own socket pass; one spilled to the other socket is named; the per-socket host-DRAM
    traffic adds up the ranks' wire bytes in proportion to where their pages are."""
    from terraform_provider_iterative_amd.parallel.placement import region_placement_report

    gb = 10 ** 9
    entries = [{"rank": r, "gpu_numa": 0 if r < 4 else 1,
                "bytes_per_node": {"N%d" % (0 if r < 4 else 1): 12 * gb},
                "wire_bytes_per_step": 20 * gb} for r in range(8)]
    report, problems = region_placement_report(entries)
    assert problems == []
    assert report["host_dram_bytes_per_step"] == {"N0": 80 * gb, "N1": 80 * gb}
    entries[5]["bytes_per_node"] = {"N0": 9 * gb, "N1": 3 * gb}  # node 1 ran short
    report, problems = region_placement_report(entries)
    assert len(problems) == 1 and problems[0].startswith("rank 5:") and "node 1" in problems[0]
    assert report["host_dram_bytes_per_step"] == {"N0": 95 * gb, "N1": 65 * gb}
    entries[5]["gpu_numa"] = -1  # unknown GPU socket: reported, not judged
    assert region_placement_report(entries)[1] == []


def _eight_rank_cpu_bench(tmp_path, fake_numa, *extra):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "8", "--device", "cpu", "--total-gb",
           "0.016", "--steps", "1", "--warmup", "1", "--no-latency", "--hidden", "128",
           "--broadcast-gb", "0", "--no-async", *extra]
    env = dict(os.environ, OMP_NUM_THREADS="1", TPI_FAKE_GPU_NUMA=fake_numa)
    return subprocess.run(cmd, cwd=str(tmp_path), capture_output=True, text=True, timeout=400,
                          env=env)


def test_eight_ranks_report_their_placement_and_flag_off_socket_regions(tmp_path):
    """8 gloo ranks: every rank's GPU socket and region placement reaches rank 0's JSON.  This
    container has one NUMA node, so on a fake 2-socket topology ranks 4-7 ("GPUs on socket 1")
    hold regions on the wrong socket: the bench warns and names them in its JSON, and with
    --strict-numa stops before timing."""
    ok = _eight_rank_cpu_bench(tmp_path, "0")
    assert ok.returncode == 0, ok.stderr[-3000:]
    d = json.loads([l for l in ok.stdout.splitlines() if l.startswith("{")][0])
    ranks = d["rank_placement"]["ranks"]
    assert [e["rank"] for e in ranks] == list(range(8))
    assert all(e["gpu_numa"] == 0 and e["bytes_per_node"].get("N0") for e in ranks), ranks
    per_node = d["rank_placement"]["host_dram_bytes_per_step"]
    assert per_node["N0"] == sum(e["wire_bytes_per_step"] for e in ranks) > 0
    bad = _eight_rank_cpu_bench(tmp_path, "0,0,0,0,1,1,1,1")
    assert bad.returncode == 0, bad.stderr[-3000:]
    assert "off their GPU's socket" in bad.stderr
    flagged = json.loads([l for l in bad.stdout.splitlines() if l.startswith("{")][0])[
        "rank_placement"]["remote_numa_ranks"]
    assert [p.split(":")[0] for p in flagged] == ["rank %d" % r for r in (4, 5, 6, 7)]
    strict = _eight_rank_cpu_bench(tmp_path, "0,0,0,0,1,1,1,1", "--strict-numa")
    assert strict.returncode != 0  # each rank exits 4; torchrun reports the failure as 1
    for r in (4, 5, 6, 7):
        assert "rank %d:" % r in strict.stderr
    assert "rank 3:" not in strict.stderr


def test_preempt_bench_rank_script_renders():
    """bench/bench_preempt.py's rank script is a %-template: every literal % in it must be
    escaped, or the driver bench's preempt_e2e block dies before the task starts."""
    import importlib.util

    spec = importlib.util.spec_from_file_location(
        "bench_preempt", os.path.join(ROOT, "bench", "bench_preempt.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    for extra in ([], [4.2, 2.5]):
        text = mod.RANK % {"python": sys.executable, "root": ROOT, "spill": "/dev/shm/x",
                           "gb": 100.0, "codec": "tpz1", "prefetch": True, "early": False,
                           "standby": True, "step_s": 0.002, "boundary": True,
                           "materialize": False, "extra": extra}
        compile(text, "rank", "exec")
